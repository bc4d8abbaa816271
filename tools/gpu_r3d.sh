#!/bin/bash
# Same-box A/B of the batched encode group: EDV_ENCODE_M 16 (1 wave/SIMD at 1M) vs 8 (2 waves, twice the inversions); c1, c3.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r3d
mkdir -p $OUT
export PLENUM_EDVERIFY_LENIENT=1
for rep in 1 2; do
for v in m16 m8; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  for c in c1 c3; do
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --dropin-steps 0 --e2e-n 0 --e2e-c0 0 --config $c > $OUT/b_${c}_${v}_$rep.log 2>&1 || { tail -20 $OUT/b_${c}_${v}_$rep.log; exit 1; }
    python - $OUT/b_${c}_${v}_$rep.log $v $c <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, d['parity'].get('mismatches_vs_construction'), flush=True)
PY
  done
done
done
echo done
