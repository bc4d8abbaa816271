#!/bin/bash
# rocprof kernel stats of the latency paths: the single-request kernel (small probe) and the
# BLS verify forms (probe at 25 checks per launch in each form).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6e
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_small -o run -- python tools/small_probe.py 14 > $OUT/prof_small.log 2>&1 || exit $?
grep "engine call" $OUT/prof_small.log
for f in quad pair one; do
  BLS_FORM=$f BLS_SIZES=25,25,25 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_bls_$f -o run -- python tools/bls_probe.py > $OUT/prof_bls_$f.log 2>&1 || exit $?
  grep "^n=" $OUT/prof_bls_$f.log | tail -1
done
echo done
