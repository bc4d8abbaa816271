#!/bin/bash
# Same-box A/B: SHA-512 rounds with v_bitop3 (lib_bop3) vs before (lib_base); c1 and c3.
export TMPDIR=/tmp
OUT=gpurun_out/ab_bop3
mkdir -p $OUT
export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_bop3.so
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "golden or keyed_random or mixed" -p no:cacheprovider > $OUT/t_bop3.log 2>&1 || { tail -30 $OUT/t_bop3.log; exit 1; }
tail -1 $OUT/t_bop3.log
for v in base bop3 base bop3; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  for c in c1 c3; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --config $c > $OUT/b_${c}_$v.log 2>&1 || { tail -20 $OUT/b_${c}_$v.log; exit 1; }
    python - $OUT/b_${c}_$v.log $v $c <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[2], sys.argv[3], round(d['value']/1e6,1), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'})
PY
  done
done
timeout -k 10 120 tools/microbench/ubench_int > $OUT/ubench_int.txt 2>&1 || exit 1
cat $OUT/ubench_int.txt
