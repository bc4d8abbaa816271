#!/bin/bash
# Full GPU suite, smoke, and the default bench line (c1) after the general-path dedupe / split tables.
set -o pipefail
OUT=gpurun_out/r2g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -n 3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -c 2000 $OUT/smoke.log; exit 1; }
tail -n 2 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
tail -c 3000 $OUT/bench_c1.log
