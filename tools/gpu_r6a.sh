#!/bin/bash
# The scan's workers walking dict entries directly (EDV_SCAN_DIRECT A/B, 16 workers, alternating
# in one process), then the bench's end-to-end legs with it on.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6a
mkdir -p $OUT
AB=EDV_SCAN_DIRECT timeout -k 10 400 python -u tools/scan_cpu_bench.py 1000000 16 10 > $OUT/scan_ab.log 2>&1 || { tail -c 3000 $OUT/scan_ab.log; exit 1; }
grep "^scan" $OUT/scan_ab.log
timeout -k 10 600 python -u bench.py --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_e2e.log 2>&1 || { tail -c 3000 $OUT/bench_e2e.log; exit 1; }
python - $OUT/bench_e2e.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items():
    if k == 'by_devices': print(k, {kk: (round(vv['value']/1e6,2) if isinstance(vv, dict) else vv) for kk, vv in v.items() if kk != 'note'}); continue
    print(k, round(v['value']/1e6,2), 'M/s', 'scan', round(v['host_scan_ms'],1), 'single', round(v['single_authenticate_us']['p50'],1), {kk: round(vv,2) for kk,vv in (v.get('in_batch_ms') or {}).items()})
PY
echo done
