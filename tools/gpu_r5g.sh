#!/bin/bash
# The full GPU suite at HEAD (scan writes text slots in its workers; streamed batches), the e2e
# probe with streaming on / off, the default bench line.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5g
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0 > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^authenticate_batch|^single" $OUT/e2e_probe.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
python - $OUT/bench_c1.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
r=d['roofline']
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],3), 'frac', round(r['frac'],3), 'valu_busy', r.get('valu_busy'), 'hbm_GBps', r.get('hbm_GBps'), 'clock', r.get('clock_GHz'))
for k,v in (d.get('end_to_end') or {}).items():
    if k == 'by_devices': print(k, {kk: (round(vv['value']/1e6,2) if isinstance(vv, dict) else vv) for kk, vv in v.items() if kk != 'note'}); continue
    print(k, round(v['value']/1e6,2), 'M/s', 'scan', round(v['host_scan_ms'],1), 'gpu_call', round(v['gpu_call_ms'],2), 'single', v['single_authenticate_us'])
PY
echo done
