#!/bin/bash
# Why the bench's end_to_end leg is slower than tools/e2e_probe.py: scan phases inside the bench, and the
# same leg with OMP_NUM_THREADS=1 (spinning OpenMP workers of torch competing with the scan threads?).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2r
mkdir -p $OUT
for omp in 16 1; do
EDV_SCAN_PROFILE=1 OMP_NUM_THREADS=$omp timeout -k 10 600 python -u bench.py --steps 5 --no-cpu --general-steps 0 --dropin-steps 0 --e2e-c0 0 > $OUT/bench_e2e_omp$omp.log 2>&1 || { tail -c 3000 $OUT/bench_e2e_omp$omp.log; exit 1; }
grep -E "^scan: n=1000000" $OUT/bench_e2e_omp$omp.log
python - $OUT/bench_e2e_omp$omp.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
for k,v in d['end_to_end'].items(): print(k, round(v['value']/1e6,2), 'M/s', round(v['seconds']*1e3,1), 'ms', 'first', round(v['first_batch_value']/1e6,2), 'scan', round(v['host_scan_us_per_request'],3), 'us/req', 'gpu', round(v['gpu_call_ms'],2))
PY
done
echo done
