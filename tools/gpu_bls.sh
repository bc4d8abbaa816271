#!/bin/bash
# BLS on the GPU: parity tests, then a throughput probe of edv_bls_verify_batch.
export TMPDIR=/tmp
OUT=gpurun_out/bls
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bls.py -p no:cacheprovider > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -5 $OUT/t.log
timeout -k 10 300 python -u tools/bls_probe.py > $OUT/probe.log 2>&1 || { tail -20 $OUT/probe.log; exit 1; }
cat $OUT/probe.log
