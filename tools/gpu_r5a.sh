#!/bin/bash
# Round-3 pass at HEAD: the full GPU suite, smoke, the PMC passes (-> pmc_traffic.json that the
# bench's roofline.utilisation reads), the default bench line, rocprof kernel stats of c1.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -c 2000 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
bash tools/pmc_passes.sh > $OUT/pmc_passes.log 2>&1 || { tail -c 2000 $OUT/pmc_passes.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc 1000000 $OUT/pmc_traffic.json r5a > $OUT/pmc_summary.txt 2>&1 || { cat $OUT/pmc_summary.txt; exit 1; }
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
cat $OUT/pmc_summary.txt
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
python - $OUT/bench_c1.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
r=d['roofline']
print('value', round(d['value']/1e6,1), 'ms', round(d['ms_per_step'],3), 'frac', round(r['frac'],3), 'valu_busy', r.get('valu_busy'), 'hbm_GBps', r.get('hbm_GBps'), 'clock', r.get('clock_GHz'))
for k,v in (r.get('utilisation') or {}).items(): print(' ', k, v)
for k,v in (d.get('end_to_end') or {}).items():
    print(k, round(v['value']/1e6,2), 'M/s', 'scan', round(v['host_scan_ms'],1), 'gpu_call', round(v['gpu_call_ms'],2), 'single', v['single_authenticate_us'])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c1 -o run -- python bench.py --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/prof_c1.log 2>&1 || exit $?
echo done
