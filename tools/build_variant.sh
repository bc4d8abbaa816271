#!/bin/bash
# Build a variant of libplenum_edverify.so with another BLS wave program (A/B runs on the GPU box:
# PLENUM_EDVERIFY_LIB=varlib/lib_NAME.so).  usage: tools/build_variant.sh NAME [gen_bls_program.py flags]
set -e
NAME=$1
shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$ROOT/varlib/$NAME"
python3 "$ROOT/tools/gen_bls_program.py" --out "$ROOT/varlib/$NAME/bls_program.h" "$@"
cd "$ROOT/indy-plenum_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
  -DEDV_BLS_PROGRAM_H="\"$ROOT/varlib/$NAME/bls_program.h\"" -c -o "$ROOT/varlib/$NAME/bls.o" csrc/bls.hip
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared --offload-arch=gfx950 -o "$ROOT/varlib/lib_$NAME.so" \
  build/edverify.o "$ROOT/varlib/$NAME/bls.o"
rm -f "$ROOT/varlib/$NAME/bls.o"
echo "built varlib/lib_$NAME.so"
