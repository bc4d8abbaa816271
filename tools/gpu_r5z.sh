#!/bin/bash
# The small kernel's product order 0 (zero-started chains, carries after) vs 2, with the phase
# events now off by default; single-request latency through the default library.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5z
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_authn.py -k "small or single or drain" -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_small.log 2>&1 || { tail -c 4000 $OUT/pytest_small.log; exit 1; }
tail -n 1 $OUT/pytest_small.log
for v in sprof sprof0 sprof sprof0; do
  PLENUM_EDVERIFY_LIB=tools/variants/lib_$v.so timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_$v.log 2>&1 || { tail -c 3000 $OUT/small_probe_$v.log; exit 1; }
  echo "== $v"; grep "engine call\|decode total\|hash  \|end  " $OUT/small_probe_$v.log
done
timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_default.log 2>&1 || { tail -c 3000 $OUT/small_probe_default.log; exit 1; }
echo "== default"; grep "engine call" $OUT/small_probe_default.log
echo done
