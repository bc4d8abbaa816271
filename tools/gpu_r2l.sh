#!/bin/bash
# e2e probe (where the drop-in's time goes), then a 2-rank gloo rehearsal of bench.py N>1 on one GPU
# (c1 and c4: the collective timing legs).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2l
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_authn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_authn.log 2>&1 || { tail -c 3000 $OUT/pytest_authn.log; exit 1; }
tail -n 1 $OUT/pytest_authn.log
EDV_SCAN_PROFILE=1 timeout -k 10 300 python -u tools/e2e_probe.py > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
head -c 4000 $OUT/e2e_probe.log
for c in c1 c4; do
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 2 --dist-backend gloo --same-device --general-steps 0 --config $c --no-cpu --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/rehearsal_gloo2_$c.log 2>&1 || { tail -c 3000 $OUT/rehearsal_gloo2_$c.log; exit 1; }
python - $OUT/rehearsal_gloo2_$c.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[1], d['n_gpus'], round(d['value']/1e6,1), d['parity'], d['collective'], (d.get('tally') or {}).get('quorum_match'))
PY
done
echo done
