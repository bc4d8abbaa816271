export TMPDIR=/tmp
OUT=gpurun_out/r5
mkdir -p $OUT
true &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --requests 200000 --dist-backend gloo --same-device --general-steps 2 > $OUT/bench_gloo2.log 2>&1 &&
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --config c4 --steps 3 --warmup 1 --requests 200000 --dist-backend gloo --same-device --general-steps 0 > $OUT/bench_gloo2_c4.log 2>&1
rc=$?
for f in $OUT/bench_*.log; do echo $f; grep '^{' $f | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['n_gpus'], d['ms_per_step'], d['parity'], d.get('tally'), d['config']['workload'][:200])" || tail -5 $f; done
exit $rc
