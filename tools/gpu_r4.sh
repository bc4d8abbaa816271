export TMPDIR=/tmp
OUT=gpurun_out/r4
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --general-steps 0 > $OUT/bench_c1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --general-steps 0 --no-length-buckets > $OUT/bench_c1_nb.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config c3 --no-cpu --general-steps 0 > $OUT/bench_c3.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config c3 --no-cpu --general-steps 0 --no-length-buckets > $OUT/bench_c3_nb.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log
for f in $OUT/bench_*.log; do echo $f; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['phase_ms'])"; done
exit $rc
