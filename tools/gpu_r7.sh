export TMPDIR=/tmp
OUT=gpurun_out/r7
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --config c3 --no-cpu --general-steps 1 --pipeline 1 --steps 10 > $OUT/bench_c3_p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 bench.py --config c3 --no-cpu --general-steps 0 --pipeline 1 --steps 3 --warmup 1 > $OUT/prof.log 2>&1
rc=$?
tail -1 $OUT/bench_c3_p1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'], d['other_path'])"
head -8 $OUT/prof/run_kernel_stats.csv | cut -c1-160
exit $rc
