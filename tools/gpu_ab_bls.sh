#!/bin/bash
# BLS A/B: Fp / Fp2 products inline (EDV_BN_INLINE_LEVEL 0/1/2) and batch size (occupancy 2 waves/SIMD
# needs >= 128k checks per launch); parity via tests/test_gpu_bls.py on each variant.
export TMPDIR=/tmp PLENUM_EDVERIFY_LENIENT=1
OUT=gpurun_out/ab_bls
mkdir -p $OUT
for v in bls1 bls2; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  timeout -k 10 300 python -u -m pytest -x -q --timeout 250 --timeout-method thread tests/test_gpu_bls.py -p no:cacheprovider > $OUT/t_$v.log 2>&1 || { tail -30 $OUT/t_$v.log; exit 1; }
  echo "$v: $(tail -1 $OUT/t_$v.log)"
done
for v in bls0 bls1 bls2; do
  export PLENUM_EDVERIFY_LIB=$PWD/tools/variants/lib_$v.so
  BLS_SIZES=64,65536,131072,262144 timeout -k 10 400 python -u tools/bls_probe.py > $OUT/probe_$v.log 2>&1 || { tail -20 $OUT/probe_$v.log; exit 1; }
  echo "== $v"; grep "n=" $OUT/probe_$v.log
done
