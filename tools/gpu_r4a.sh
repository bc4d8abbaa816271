#!/bin/bash
# Round 3 first pass: the whole -m gpu suite at HEAD (BATCH-framed verify-ahead,
# BLS identity-point rejection), smoke, one default bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -c 3000 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { tail -c 3000 $OUT/bench.log; exit 1; }
python - $OUT/bench.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print('value', round(d['value']/1e6,1), 'M/s', 'frac', round(d['roofline']['frac'],3))
for k,v in d['end_to_end'].items(): print(k, round(v['value']/1e6,2), 'M/s', 'gpu_call_ms', round(v['gpu_call_ms'],2))
PY
echo done
