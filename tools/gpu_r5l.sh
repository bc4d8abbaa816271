#!/bin/bash
# Staged batches (the scan's workers DMA each chunk as they finish it): authenticator GPU tests,
# the e2e probe (staged / streamed / plain), the bench's e2e legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_authn.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0 > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^authenticate_batch|^single|^scan" $OUT/e2e_probe.log | tail -14
timeout -k 10 600 python -u bench.py --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_e2e.log 2>&1 || { tail -c 3000 $OUT/bench_e2e.log; exit 1; }
python - $OUT/bench_e2e.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items():
    if k == 'by_devices': print(k, {kk: (round(vv['value']/1e6,2) if isinstance(vv, dict) else vv) for kk, vv in v.items() if kk != 'note'}); continue
    print(k, round(v['value']/1e6,2), 'M/s', 'scan', round(v['host_scan_ms'],1), 'gpu_call', round(v['gpu_call_ms'],2), 'single', v['single_authenticate_us'])
PY
echo done
