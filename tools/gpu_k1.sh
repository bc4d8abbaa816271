#!/bin/bash
# Packed SoA units (mode 3): parity tests, then same-box A/B vs sorted in-place (mode 1) on c3 and c1.
export TMPDIR=/tmp
OUT=gpurun_out/k1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "packed or spans or mixed or golden" -p no:cacheprovider > $OUT/t.log 2>&1 || { tail -40 $OUT/t.log; exit 1; }
tail -2 $OUT/t.log
for r in 1 2; do
for c in c3 c1; do
  for m in on packed; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --config $c --length-buckets $m > $OUT/b_${c}_${m}_$r.log 2>&1 || { tail -20 $OUT/b_${c}_${m}_$r.log; exit 1; }
    python - $OUT/b_${c}_${m}_$r.log $m $c <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'})
PY
  done
done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o k1 -- python3 bench.py --steps 5 --warmup 1 --no-cpu --general-steps 0 --config c3 --length-buckets packed > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -c1-160 {} | head -12'
