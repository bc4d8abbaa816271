#!/bin/bash
# BLS four lanes per check with each Miller loop split over two lanes: the GPU BLS tests in every form, the probe per form.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5x
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu_bls.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu_bls.log; exit 1; }
tail -n 1 $OUT/pytest_gpu_bls.log
for f in quad pair one; do
  BLS_FORM=$f BLS_SIZES=1,25,1024,16384 timeout -k 10 300 python -u tools/bls_probe.py > $OUT/bls_probe_$f.log 2>&1 || { tail -c 3000 $OUT/bls_probe_$f.log; exit 1; }
  echo "form $f:"; grep "^n=" $OUT/bls_probe_$f.log
done
echo done
