#!/bin/bash
# c1 bench with every leg (e2e, drop-in window, CPU baselines), then a 2-rank gloo rehearsal of N>1 on one GPU.
set -o pipefail
OUT=gpurun_out/r2e
mkdir -p $OUT
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || exit $?
tail -c 2500 $OUT/bench_c1.log
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --same-device --general-steps 0 > $OUT/rehearsal_gloo2_c1.log 2>&1 || exit $?
tail -c 1200 $OUT/rehearsal_gloo2_c1.log
