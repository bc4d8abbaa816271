#!/bin/bash
# A/B of the base-point comb window (EDV_BASE_W 16 / 18 / 20 builds) on configs[1] / configs[2].
export TMPDIR=/tmp
OUT=gpurun_out/basew
mkdir -p $OUT
for v in 16 18 20; do
  if [ $v = 16 ]; then unset PLENUM_EDVERIFY_LIB; else export PLENUM_EDVERIFY_LIB=$PWD/ab/lib_b$v.so; fi
  timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py -k "golden or keyed_random" -p no:cacheprovider > $OUT/t_$v.log 2>&1 || exit 1
  for c in c1 c2; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --general-steps 0 --config $c > $OUT/b_${c}_$v.log 2>&1 || exit 1
  done
done
