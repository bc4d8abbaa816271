#!/bin/bash
# Small-kernel phase probes (order 1 vs 2), authenticator GPU tests, the e2e probe with the
# staged scan's copier thread, the bench's e2e legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5n
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_authn.py tests/test_gpu_parity.py -k "authn or small or staged or drain" -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
for v in sprof; do
  PLENUM_EDVERIFY_LIB=tools/variants/lib_$v.so timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_$v.log 2>&1 || { tail -c 3000 $OUT/small_probe_$v.log; exit 1; }
  echo "== $v"; cat $OUT/small_probe_$v.log | tail -9
done
timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_default.log 2>&1 || { tail -c 3000 $OUT/small_probe_default.log; exit 1; }
echo "== default"; tail -2 $OUT/small_probe_default.log
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
