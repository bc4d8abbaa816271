#!/bin/bash
# Pipelined authenticate_batch (async submit / collect): GPU tests of the host paths, the e2e
# probe with part-size A/B and the single-request latency breakdown, the bench's e2e legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4c
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_authn.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0,131072,262144 > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^authenticate_batch|^single|^phases" $OUT/e2e_probe.log
timeout -k 10 600 python -u bench.py --steps 5 --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_e2e.log 2>&1 || { tail -c 3000 $OUT/bench_e2e.log; exit 1; }
python - $OUT/bench_e2e.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items():
    print(k, round(v['value']/1e6,2), 'M/s', round(v['seconds']*1e3,1), 'ms', 'scan', round(v['host_scan_ms'],1), 'ms', 'gpu_call', round(v['gpu_call_ms'],2), 'stage', v['stage_ms'], 'h2d_ce_ms', v['h2d_ms_copy_engine'], 'single', v['single_authenticate_us'])
PY
echo done
