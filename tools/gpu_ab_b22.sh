#!/bin/bash
# A/B of the base comb window 22 (EDV_BASE_W=22 build) (ab/lib_*.so) against the default build, one box.
export TMPDIR=/tmp
OUT=gpurun_out/ab22
mkdir -p $OUT
for v in def b22 def2 b222; do
  case $v in def|def2) unset PLENUM_EDVERIFY_LIB;; *) export PLENUM_EDVERIFY_LIB=$PWD/ab/lib_${v:0:3}.so;; esac
  timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "golden or keyed_random" -p no:cacheprovider > $OUT/t_$v.log 2>&1 || exit 1
  for c in c1 c2 c3; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --config $c > $OUT/b_${c}_$v.log 2>&1 || exit 1
  done
done
