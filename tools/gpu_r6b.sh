#!/bin/bash
# Closing check: the full GPU suite (incl. verify_one_keyed vs the batch path) and smoke.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6b
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -c 2000 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
echo done
