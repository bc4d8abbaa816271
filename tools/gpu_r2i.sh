#!/bin/bash
# Full GPU pass at HEAD (rebuilt container): all -m gpu tests, smoke, bench c1 (default), c3, BLS probe.
export TMPDIR=/tmp
OUT=gpurun_out/r2i
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -n 3 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -c 2000 $OUT/smoke.log; exit 1; }
tail -n 1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
timeout -k 10 300 python -u bench.py --config c3 --no-cpu --general-steps 0 > $OUT/bench_c3.log 2>&1 || { tail -c 3000 $OUT/bench_c3.log; exit 1; }
timeout -k 10 300 python -u tools/bls_probe.py > $OUT/bls_probe.log 2>&1 || { tail -20 $OUT/bls_probe.log; exit 1; }
cat $OUT/bls_probe.log
for f in $OUT/bench_c1.log $OUT/bench_c3.log; do python - $f <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[1], round(d['value']/1e6,1), round(d['ms_per_step'],3), d['roofline']['frac'], {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'})
PY
done
