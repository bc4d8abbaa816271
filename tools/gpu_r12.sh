# sub-batch cap with sorted lanes: GPU tests + c3/c1 bench
export TMPDIR=/tmp
OUT=gpurun_out/r12
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $OUT/gpu_tests.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config c3 --no-cpu --general-steps 2 --steps 20 > $OUT/c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --config c1 --no-cpu --general-steps 2 --steps 20 > $OUT/c1.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log
for f in c3 c1; do tail -1 $OUT/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['length_buckets'], d.get('phase_ms'), d.get('other_path',{}).get('value'))"; done
exit $rc
