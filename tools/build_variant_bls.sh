#!/bin/bash
# Build an A/B variant of the whole library (edverify.hip + bls.hip) for BLS probes:
# tools/build_variant_bls.sh NAME [-DFLAG=V ...] -> tools/variants/lib_NAME.so
set -e
name=$1; shift
mkdir -p tools/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -Wno-unused-function \
  '-DEDV_KEY_WINDOWS(X)=X(10) X(14)' "$@" -o tools/variants/lib_$name.so indy-plenum_amd/csrc/edverify.hip indy-plenum_amd/csrc/bls.hip
echo built tools/variants/lib_$name.so
