#!/bin/bash
# One GPU-box pass: gpu tests, smoke, bench (c1 + c2), rocprof kernel stats.
# Every GPU step has its own time limit; steps are chained with &&.
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench_c1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --config c2 --no-cpu > $OUT/bench_c2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu --general-steps 3 > $OUT/prof.log 2>&1
rc=$?
find $OUT -name "*stats*.csv" | sort
tail -3 $OUT/pytest_gpu.log; tail -1 $OUT/smoke.log; tail -1 $OUT/bench_c1.log; tail -1 $OUT/bench_c2.log
exit $rc
