#!/bin/bash
# Same-box A/B: comb digit-sign selects as v_bitop3 (selb3) vs v_cmp+v_cndmask (selcnd); plus the op-rate microbench.
export TMPDIR=/tmp
OUT=gpurun_out/ab_sel
mkdir -p $OUT
true
true
export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_new.so
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -p no:cacheprovider > $OUT/t_new.log 2>&1 || { tail -30 $OUT/t_new.log; exit 1; }
tail -1 $OUT/t_new.log
for v in old new old new; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  for c in c1 c2; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps $([ $c = c1 ] && echo 3 || echo 0) --config $c > $OUT/b_${c}_$v.log 2>&1 || { tail -20 $OUT/b_${c}_$v.log; exit 1; }
    python - $OUT/b_${c}_$v.log $v $c <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, 'sa', round(d['roofline']['standalone']['avg_launch_ms'],3), 'general', round((d.get('other_path') or {}).get('value',0)/1e6,1))
PY
  done
done
