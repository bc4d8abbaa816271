#!/bin/bash
# Low-latency small-batch kernel: parity vs the batch path, the authenticator tests, the
# single-request latency (e2e probe) and the bench's e2e legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5h
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_authn.py -x -v --timeout 300 --timeout-method thread -m gpu -k "small or authn or drain or promotion or keyed_random or golden" > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0 > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^authenticate_batch|^single|^phases" $OUT/e2e_probe.log
echo done
