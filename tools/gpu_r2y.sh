#!/bin/bash
# Scan helper threads: a persistent pool (hostpack_pool) vs threads spawned per call (hostpack_spawn),
# alternating: e2e probe (1M) and the bench's end_to_end legs (configs[0] 10k, configs[1] 1M).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2y
mkdir -p $OUT
SO=indy-plenum_amd/plenum_amd/_hostpack.cpython-310-x86_64-linux-gnu.so
cp $SO $OUT/hostpack_head.so.bak
for rep in 1 2; do
for v in spawn pool; do
  cp tools/variants/hostpack_$v.cpython-310-x86_64-linux-gnu.so $SO
  EDV_SCAN_PROFILE=1 timeout -k 10 300 python -u tools/e2e_probe.py > $OUT/e2e_${v}_$rep.log 2>&1 || { tail -c 3000 $OUT/e2e_${v}_$rep.log; exit 1; }
  echo "$v rep=$rep"; grep -E "^auth" $OUT/e2e_${v}_$rep.log
  timeout -k 10 600 python -u bench.py --steps 2 --warmup 1 --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_${v}_$rep.log 2>&1 || { tail -c 3000 $OUT/bench_${v}_$rep.log; exit 1; }
  python - $OUT/bench_${v}_$rep.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items(): print(' ', k, round(v['value']/1e6,2), 'M/s', round(v['seconds']*1e3,2), 'ms', 'first', round(v['first_batch_value']/1e6,2), 'gpu', round(v['gpu_call_ms'],2))
PY
done
done
cp tools/variants/hostpack_pool.cpython-310-x86_64-linux-gnu.so $SO
rm -f $OUT/hostpack_head.so.bak
echo done
