#!/bin/bash
# Closing: authenticator GPU tests and the default bench line at HEAD (2^17 streamed submits).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6d
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_authn.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu_authn.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu_authn.log; exit 1; }
tail -n 1 $OUT/pytest_gpu_authn.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
python - $OUT/bench_c1.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
r=d['roofline']
print(round(d['value']/1e6,1), round(d['ms_per_step'],3), 'frac', round(r['frac'],3), 'busy', r.get('valu_busy') and round(r['valu_busy'],3), 'GBps', r.get('hbm_GBps') and round(r['hbm_GBps']), 'clk', r.get('clock_GHz') and round(r['clock_GHz'],3), 'cpu', round(d['cpu_baseline']['value']/1e3,1), 'k/s')
for k,v in (d.get('end_to_end') or {}).items():
    if k == 'by_devices': print(' ', k, {kk: (round(vv['value']/1e6,2) if isinstance(vv, dict) else vv) for kk, vv in v.items() if kk != 'note'}); continue
    print(' ', k, round(v['value']/1e6,2), 'M/s', 'single', round(v['single_authenticate_us']['p50'],1), {kk: round(vv,2) for kk,vv in (v.get('in_batch_ms') or {}).items()})
PY
echo done
