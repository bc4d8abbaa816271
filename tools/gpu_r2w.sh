#!/bin/bash
# Scan worker pinning A/B at HEAD (staging copy unpinned): e2e probe with EDV_SCAN_PIN=1 (default) and 0,
# alternating processes, then the bench's end_to_end legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2w
mkdir -p $OUT
for rep in 1 2; do
for pin in 1 0; do
  EDV_SCAN_PIN=$pin EDV_SCAN_PROFILE=1 timeout -k 10 300 python -u tools/e2e_probe.py > $OUT/e2e_pin${pin}_$rep.log 2>&1 || { tail -c 3000 $OUT/e2e_pin${pin}_$rep.log; exit 1; }
  echo "pin=$pin rep=$rep"; grep -E "^auth|^scan: n=1000000" $OUT/e2e_pin${pin}_$rep.log
done
done
timeout -k 10 600 python -u bench.py --steps 5 --no-cpu --general-steps 0 --dropin-steps 0 > $OUT/bench_e2e.log 2>&1 || { tail -c 3000 $OUT/bench_e2e.log; exit 1; }
python - $OUT/bench_e2e.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items(): print(k, round(v['value']/1e6,2), 'M/s', round(v['seconds']*1e3,1), 'ms', 'first', round(v['first_batch_value']/1e6,2), 'scan', round(v['host_scan_us_per_request'],3), 'us/req', 'gpu', round(v['gpu_call_ms'],2))
PY
echo done
