#!/bin/bash
# Profiles of the current build: kernel-trace stats (csv) for c1 and c3, PMC passes (c1 + general).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2d
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c1 -o run -- python3 bench.py --steps 10 --no-cpu --general-steps 2 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/prof_c1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --config c3 --steps 10 --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/prof_c3.log 2>&1 || exit $?
bash tools/pmc_passes.sh > $OUT/pmc_passes.log 2>&1 || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc 1000000 $OUT/pmc_traffic.json > $OUT/pmc_summary.txt 2>&1
cat $OUT/pmc_summary.txt
