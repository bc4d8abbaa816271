#!/bin/bash
# Same-box A/B: comb entries with 16-B aligned y+x / y-x blocks, the digit sign applied by
# swapping the two block addresses (lib_sel) vs 20 per-limb selects (lib_head); c1, c2, c3 + general.
export TMPDIR=/tmp PLENUM_EDVERIFY_LENIENT=1
OUT=gpurun_out/ab_sel
mkdir -p $OUT
export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_sel.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "golden or keyed_random or large or headline or general or random_batch" -p no:cacheprovider > $OUT/t_sel.log 2>&1 || { tail -30 $OUT/t_sel.log; exit 1; }
echo "sel: $(tail -1 $OUT/t_sel.log)"
for rep in 1 2; do
for v in head sel; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  for c in c1 c2 c3; do
    gs=0; [ $c = c1 ] && gs=3
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps $gs --dropin-steps 0 --e2e-n 0 --e2e-c0 0 --config $c > $OUT/b_${c}_${v}_$rep.log 2>&1 || { tail -20 $OUT/b_${c}_${v}_$rep.log; exit 1; }
    python - $OUT/b_${c}_${v}_$rep.log $v $c <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
g=d.get('other_path') or {}
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), round(d['ms_per_step'],3), round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, 'general', round(g.get('value',0)/1e6,1), d['parity']['mismatches_vs_construction'], flush=True)
PY
  done
done
done
