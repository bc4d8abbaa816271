#!/bin/bash
# Staging-free host path: signature slots (base58 decoded on the GPU) written by the scan into
# pinned host memory.  GPU tests of the changed paths, the e2e probe, the bench's e2e legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r4b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_authn.py tests/test_gpu_parity.py tests/test_gpu_bls.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
EDV_SCAN_PROFILE=1 timeout -k 10 300 python -u tools/e2e_probe.py > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^auth|^scan: n=1000000" $OUT/e2e_probe.log | tail -8
timeout -k 10 600 python -u bench.py --steps 5 --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_e2e.log 2>&1 || { tail -c 3000 $OUT/bench_e2e.log; exit 1; }
python - $OUT/bench_e2e.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items():
    print(k, round(v['value']/1e6,2), 'M/s', round(v['seconds']*1e3,1), 'ms', 'scan', round(v['host_scan_ms'],1), 'ms', 'gpu_call', round(v['gpu_call_ms'],2), 'stage', v['stage_ms'], 'h2d_bytes', v['h2d_bytes'], 'h2d_ce_ms', v['h2d_ms_copy_engine'], 'direct', v['inputs_direct_from_pinned'], 'single', v['single_authenticate_us'])
PY
echo done
