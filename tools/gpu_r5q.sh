#!/bin/bash
# BLS with Granger-Scott cyclotomic squarings in the final exponentiation: GPU BLS tests, the
# latency / throughput probe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5q
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu_bls.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu_bls.log; exit 1; }
tail -n 1 $OUT/pytest_gpu_bls.log
BLS_SIZES=1,25,64,1024,65536 timeout -k 10 400 python -u tools/bls_probe.py > $OUT/bls_probe.log 2>&1 || { tail -c 3000 $OUT/bls_probe.log; exit 1; }
cat $OUT/bls_probe.log | grep "^n="
echo done
