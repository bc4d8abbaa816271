#!/bin/bash
# GPU-box pass at the W = 13 key window: gpu tests, smoke, bench c1-c4,
# rocprof kernel stats, then the PMC passes (tools/pmc_passes.sh).
export TMPDIR=/tmp
OUT=gpurun_out/r13
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench_c1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > $OUT/bench_c2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c3 --no-cpu > $OUT/bench_c3.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c4 --no-cpu > $OUT/bench_c4.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --general-steps 3 > $OUT/prof.log 2>&1 &&
bash tools/pmc_passes.sh
rc=$?
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log
exit $rc
