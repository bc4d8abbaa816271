#!/bin/bash
# Async key builds (edv_keys_add_async / set_async) and the by-devices e2e leg: authenticator GPU
# tests, then the default bench line (end_to_end.by_devices).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_authn.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
timeout -k 10 600 python -u bench.py --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
python - $OUT/bench_c1.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print('value', round(d['value']/1e6,1), 'frac', round(d['roofline']['frac'],3))
for k,v in d['end_to_end'].items():
    if k == 'by_devices': print(k, v); continue
    print(k, round(v['value']/1e6,2), 'M/s', 'scan', round(v['host_scan_ms'],1), 'gpu_call', round(v['gpu_call_ms'],2), 'single', v['single_authenticate_us'])
PY
echo done
