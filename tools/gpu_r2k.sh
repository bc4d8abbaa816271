#!/bin/bash
# End-to-end drop-in after the threaded native scan: c1 bench with every leg (e2e configs[0] / configs[1],
# drop-in window, CPU baselines); rocprof kernel stats (csv) of the c1 and c3 benches.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r2k
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_authn.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_authn.log 2>&1 || { tail -c 3000 $OUT/pytest_authn.log; exit 1; }
tail -n 1 $OUT/pytest_authn.log
timeout -k 10 600 python -u bench.py > $OUT/bench_c1.log 2>&1 || { tail -c 3000 $OUT/bench_c1.log; exit 1; }
python - $OUT/bench_c1.log <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(round(d['value']/1e6,1), round(d['roofline']['frac'],3), json.dumps(d['end_to_end'])[:1500])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c1 -o run -- python bench.py --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/prof_c1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python bench.py --config c3 --steps 10 --no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 > $OUT/prof_c3.log 2>&1 || exit $?
find $OUT -name "*stats*"
echo done
