#!/bin/bash
# Round-3 closing pass at HEAD: the full GPU suite, smoke, the PMC passes (-> pmc_traffic.json for
# the bench's roofline.utilisation), the default bench line, configs[2]/[3]/[4] lines, rocprof
# kernel stats of c1 and c3, the single-request probe, the BLS latency probe.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5s
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -c 2000 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
bash tools/pmc_passes.sh > $OUT/pmc_passes.log 2>&1 || { tail -c 2000 $OUT/pmc_passes.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc 1000000 $OUT/pmc_traffic.json r5s > $OUT/pmc_summary.txt 2>&1 || { cat $OUT/pmc_summary.txt; exit 1; }
cp $OUT/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
for c in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 --e2e-devices 0 > $OUT/bench_$c.log 2>&1 || { tail -c 3000 $OUT/bench_$c.log; exit 1; }
done
for f in $OUT/bench_c1.log $OUT/bench_c2.log $OUT/bench_c3.log $OUT/bench_c4.log; do python - $f <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
r=d['roofline']
print(sys.argv[1].split('/')[-1], round(d['value']/1e6,1), round(d['ms_per_step'],3), 'frac', round(r['frac'],3), 'busy', r.get('valu_busy') and round(r['valu_busy'],3), 'GBps', r.get('hbm_GBps') and round(r['hbm_GBps']), 'clk', r.get('clock_GHz') and round(r['clock_GHz'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, 'tally', (d.get('tally') or {}).get('quorum_match'))
for k,v in (d.get('end_to_end') or {}).items():
    if k == 'by_devices': print(' ', k, {kk: (round(vv['value']/1e6,2) if isinstance(vv, dict) else vv) for kk, vv in v.items() if kk != 'note'}); continue
    print(' ', k, round(v['value']/1e6,2), 'M/s', 'scan', round(v['host_scan_ms'],1), 'gpu_call', round(v['gpu_call_ms'],2), 'single', v['single_authenticate_us'])
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c1 -o run -- python bench.py --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 --e2e-devices 0 > $OUT/prof_c1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python bench.py --config c3 --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 --e2e-devices 0 > $OUT/prof_c3.log 2>&1 || exit $?
PLENUM_EDVERIFY_LIB=tools/variants/lib_sprof.so timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_sprof.log 2>&1 || { tail -c 3000 $OUT/small_probe_sprof.log; exit 1; }
tail -10 $OUT/small_probe_sprof.log
BLS_SIZES=1,25,1024,65536 timeout -k 10 300 python -u tools/bls_probe.py > $OUT/bls_probe.log 2>&1 || { tail -c 3000 $OUT/bls_probe.log; exit 1; }
grep "^n=" $OUT/bls_probe.log
echo done
