#!/bin/bash
# Probes after the closing pass: small-kernel phases, BLS latency (pair lanes), the e2e probe and
# the bench's end-to-end legs with the in-batch breakdown.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5t
mkdir -p $OUT
PLENUM_EDVERIFY_LIB=tools/variants/lib_sprof.so timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_sprof.log 2>&1 || { tail -c 3000 $OUT/small_probe_sprof.log; exit 1; }
tail -10 $OUT/small_probe_sprof.log
BLS_SIZES=1,25,1024,16384,65536 timeout -k 10 300 python -u tools/bls_probe.py > $OUT/bls_probe.log 2>&1 || { tail -c 3000 $OUT/bls_probe.log; exit 1; }
grep "^n=" $OUT/bls_probe.log
timeout -k 10 600 python -u bench.py --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_e2e.log 2>&1 || { tail -c 3000 $OUT/bench_e2e.log; exit 1; }
python - $OUT/bench_e2e.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items():
    if k == 'by_devices': print(k, {kk: (round(vv['value']/1e6,2) if isinstance(vv, dict) else vv) for kk, vv in v.items() if kk != 'note'}); continue
    print(k, round(v['value']/1e6,2), 'M/s', 'scan', round(v['host_scan_ms'],1), 'gpu_call', round(v['gpu_call_ms'],2), 'single', round(v['single_authenticate_us']['p50'],1), {kk: round(vv,2) for kk,vv in (v.get('in_batch_ms') or {}).items()})
PY
echo done
