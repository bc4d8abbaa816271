#!/bin/bash
# Same-box A/B: interleaved multiplication pairs (fe_mul_n) in the comb's mixed addition.
# c0 = serial (with the full-rate doublings), c1 = the (y+x)/(y-x) pair, c2 = + two pairs in p1p1 -> p3,
# c0nodbl = round-2 HEAD arithmetic (doublings as v_lshlrev), c2w3 = c2 at 3 waves / SIMD.
export TMPDIR=/tmp PLENUM_EDVERIFY_LENIENT=1
OUT=gpurun_out/ab_muln
mkdir -p $OUT
VARS="c0nodbl c0 c1 c2 c2w3"
for v in c2; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "golden or keyed_random" -p no:cacheprovider > $OUT/t_$v.log 2>&1 || { tail -30 $OUT/t_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/t_$v.log)"
done
for rep in 1 2; do
for v in $VARS; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  for c in c1; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --dropin-steps 0 --e2e-n 0 --e2e-c0 0 --config $c > $OUT/b_${c}_${v}_$rep.log 2>&1 || { tail -20 $OUT/b_${c}_${v}_$rep.log; exit 1; }
    python - $OUT/b_${c}_${v}_$rep.log $v $c <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), round(d['ms_per_step'],3), d['roofline']['frac'], {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, flush=True)
PY
  done
done
done
