export TMPDIR=/tmp
OUT=gpurun_out/r6
mkdir -p $OUT
for p in 1 4 2 1 4; do
timeout -k 10 300 python -u bench.py --no-cpu --general-steps 0 --pipeline $p --steps 40 > $OUT/bench_c1_p$p.log 2>&1 || exit 1
echo p$p $(tail -1 $OUT/bench_c1_p$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
done
