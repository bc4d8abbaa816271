#!/bin/bash
# Full pass: GPU tests, bench c1..c4 + general, rocprof kernel stats of c1 and c3.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r2c
bash tools/gpu_tests.sh || exit $?
for c in c1 c2 c3 c4; do
  extra=""
  [ $c != c1 ] && extra="--no-cpu --e2e-n 0 --e2e-c0 0 --dropin-steps 0"
  timeout -k 10 600 python -u bench.py --config $c $extra > gpurun_out/r2c/bench_$c.log 2>&1 || exit $?
  tail -c 600 gpurun_out/r2c/bench_$c.log
done
timeout -k 10 300 python -u bench.py --path general --steps 5 --warmup 1 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > gpurun_out/r2c/bench_general.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c/prof_c1 -o run -- python bench.py --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > gpurun_out/r2c/prof_c1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r2c/prof_c3 -o run -- python bench.py --config c3 --steps 10 --no-cpu --general-steps 0 > gpurun_out/r2c/prof_c3.log 2>&1 || exit $?
echo done
