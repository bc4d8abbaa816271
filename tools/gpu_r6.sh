export TMPDIR=/tmp
OUT=gpurun_out/r6
mkdir -p $OUT
timeout -k 10 300 python -u bench.py --no-cpu --general-steps 0 --pipeline 1 > $OUT/bench_c1_p1.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --general-steps 0 --pipeline 4 > $OUT/bench_c1_p4.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --general-steps 0 --pipeline 2 > $OUT/bench_c1_p2.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu --general-steps 0 --pipeline 4 > $OUT/bench_c1_p4b.log 2>&1
rc=$?
for f in $OUT/bench_*.log; do echo $f; tail -1 $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; done
exit $rc
