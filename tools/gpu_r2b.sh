#!/bin/bash
# GPU tests, then the default bench (configs[1]) with the new legs.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_tests.sh || exit $?
timeout -k 10 600 python -u bench.py > gpurun_out/bench_c1.log 2>&1
rc=$?
tail -c 3000 gpurun_out/bench_c1.log
exit $rc
