#!/bin/bash
# BLS two lanes per check (small batches) vs one: GPU BLS tests in both forms, the probe in both.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5r
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu_bls.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu_bls.log; exit 1; }
tail -n 1 $OUT/pytest_gpu_bls.log
for m in 32768 0; do
  BLS_PAIR=$m BLS_SIZES=1,25,64,1024,16384,65536 timeout -k 10 400 python -u tools/bls_probe.py > $OUT/bls_probe_$m.log 2>&1 || { tail -c 3000 $OUT/bls_probe_$m.log; exit 1; }
  echo "pair lanes up to $m:"; grep "^n=" $OUT/bls_probe_$m.log
done
echo done
