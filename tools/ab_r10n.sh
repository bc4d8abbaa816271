#!/bin/bash
# round-6 A/B of the R decode's lane arithmetic: the lane-square microbenchmark, the small-kernel
# tests on the default build, then the single-request latency of each variant library
set -o pipefail
OUT=gpurun_out/r10n
mkdir -p $OUT
timeout -k 10 60 ./tools/microbench/ubench_lanesq2 > $OUT/lanesq2.log 2>&1 || exit $?
cat $OUT/lanesq2.log
bash tools/gpu.sh r10n tests:small+or+resident+or+verify_one+or+single+or+edge py:lat:tools/single_latency.py:300 || exit $?
cat $OUT/lat.log
for v in edges0 carry2 form1 both; do
  lib=abtmp/lib_$v.so
  [ $v = edges0 ] && lib=abtmp/libedges0.so
  PLENUM_EDVERIFY_LIB=$PWD/$lib timeout -k 10 300 python -u tools/single_latency.py 300 > $OUT/lat_$v.log 2>&1 || { echo "variant $v failed"; tail -5 $OUT/lat_$v.log; exit 1; }
  echo "== $v"; grep -v amdgpu.ids $OUT/lat_$v.log
done
