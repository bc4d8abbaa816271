#!/bin/bash
# A/B of EDV_LANE_SCALE (fe_lanes.h): the small-kernel / single-request tests on the variant
# library, then the single-request latency of the default build and of the variant
set -o pipefail
OUT=gpurun_out/r10s
mkdir -p $OUT
PLENUM_EDVERIFY_LIB=$PWD/abtmp/lib_scale.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 \
  --timeout-method thread -k "small or resident or verify_one or single or edge" > $OUT/pytest_scale.log 2>&1 || { tail -30 $OUT/pytest_scale.log; exit 1; }
tail -1 $OUT/pytest_scale.log
for v in default scale default2 scale2; do
  lib=$PWD/indy-plenum_amd/libplenum_edverify.so
  case $v in scale*) lib=$PWD/abtmp/lib_scale.so ;; esac
  PLENUM_EDVERIFY_LIB=$lib timeout -k 10 300 python -u tools/single_latency.py 300 > $OUT/lat_$v.log 2>&1 || { tail -5 $OUT/lat_$v.log; exit 1; }
  echo "== $v"; grep resident $OUT/lat_$v.log
done
