# auto length buckets: all GPU tests, c1 + c3 bench, c3 kernel stats
export TMPDIR=/tmp
OUT=gpurun_out/r10
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config c3 --no-cpu --general-steps 2 --steps 10 > $OUT/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config c1 --no-cpu --general-steps 2 --steps 10 > $OUT/c1.log 2>&1 &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --config c3 --no-cpu --general-steps 0 --steps 3 --warmup 1 > $OUT/prof_c3.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
for f in c3 c1; do tail -1 $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['length_buckets'], d.get('phase_ms'), d.get('other_path',{}).get('value'))"; done
exit $rc
