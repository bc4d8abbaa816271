#!/bin/bash
# Host-path check after the scan's buffer reuse: e2e probe (3 timed batches + scan phases) and the default
# bench line (every leg, incl. end_to_end configs[0] / configs[1]).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2p
mkdir -p $OUT
EDV_SCAN_PROFILE=1 timeout -k 10 300 python -u tools/e2e_probe.py > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^auth|^scan: n=1000000" $OUT/e2e_probe.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
python - $OUT/bench_c1.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3))
for k,v in d['end_to_end'].items(): print(k, round(v['value']/1e6,2), 'M/s', round(v['seconds']*1e3,1), 'ms', 'scan', round(v['host_scan_us_per_request'],3), 'us/req', 'gpu', round(v['gpu_call_ms'],2))
PY
echo done
