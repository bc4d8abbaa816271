#!/bin/bash
# Final round-2 pass at HEAD (pooled host helpers): GPU tests, smoke, bench c1 (every leg) / c2 / c3 / c4, BLS probe,
# rocprof kernel stats of c1 and c3, then the PMC passes (traffic of edv_comb_kernel<14>).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3b
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -c 2000 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
for c in c2 c3 c4; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/bench_$c.log 2>&1 || { tail -c 3000 $OUT/bench_$c.log; exit 1; }
done
timeout -k 10 300 python -u tools/bls_probe.py > $OUT/bls_probe.log 2>&1 || { tail -20 $OUT/bls_probe.log; exit 1; }
for f in $OUT/bench_c1.log $OUT/bench_c2.log $OUT/bench_c3.log $OUT/bench_c4.log; do python - $f <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[1], round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, 'create_s', d.get('engine_create_s'))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c1 -o run -- python bench.py --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/prof_c1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python bench.py --config c3 --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/prof_c3.log 2>&1 || exit $?
echo done
