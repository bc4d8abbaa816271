#!/bin/bash
# Scan prefetch A/B on the box's CPUs (16 workers, alternating off / on), the small-kernel probe
# with the shader clock, the e2e probe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5p
mkdir -p $OUT
AB=1 timeout -k 10 400 python -u tools/scan_cpu_bench.py 1000000 16 10 > $OUT/scan_ab.log 2>&1 || { tail -c 3000 $OUT/scan_ab.log; exit 1; }
cat $OUT/scan_ab.log
PLENUM_EDVERIFY_LIB=tools/variants/lib_sprof.so timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_sprof.log 2>&1 || { tail -c 3000 $OUT/small_probe_sprof.log; exit 1; }
tail -10 $OUT/small_probe_sprof.log
EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0 > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^authenticate_batch|^single" $OUT/e2e_probe.log
EDV_SCAN_PREFETCH=1 EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0 > $OUT/e2e_probe_pf.log 2>&1 || { tail -c 3000 $OUT/e2e_probe_pf.log; exit 1; }
echo "prefetch:"; grep -E "^authenticate_batch|^single" $OUT/e2e_probe_pf.log
echo done
