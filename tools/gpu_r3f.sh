#!/bin/bash
# Scan bookkeeping on the workers: GPU tests of the host-pointer paths, the e2e
# probe, and the bench's end_to_end legs alone.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_authn.py tests/test_gpu_parity.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
EDV_SCAN_PROFILE=1 timeout -k 10 300 python -u tools/e2e_probe.py > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^auth|^scan: n=1000000" $OUT/e2e_probe.log
timeout -k 10 600 python -u bench.py --steps 5 --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_e2e.log 2>&1 || { tail -c 3000 $OUT/bench_e2e.log; exit 1; }
python - $OUT/bench_e2e.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items(): print(k, round(v['value']/1e6,2), 'M/s', round(v['seconds']*1e3,1), 'ms', 'first', round(v['first_batch_value']/1e6,2), 'scan', round(v['host_scan_us_per_request'],3), 'us/req', 'gpu', round(v['gpu_call_ms'],2))
PY
echo done
