#!/bin/bash
# General-path key dedupe: parity tests for the general path, then A/B of the
# previous library (per-lane tables) against the dedupe build on c1 (1,000
# signers) and distinct keys (1M signers).
set -o pipefail
OUT=gpurun_out/r2f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "general or random or golden or sub_batch or large_batch or offsets" > $OUT/pytest_general.log 2>&1 || { tail -c 3000 $OUT/pytest_general.log; exit 1; }
tail -c 1500 $OUT/pytest_general.log
timeout -k 10 400 python -u tools/ab_libs.py --rounds 2 --path general --config c1 tools/variants/lib_gen1.so indy-plenum_amd/libplenum_edverify.so > $OUT/ab_general_c1.log 2>&1 || { cat $OUT/ab_general_c1.log; exit 1; }
cat $OUT/ab_general_c1.log
timeout -k 10 500 python -u tools/ab_libs.py --rounds 1 --path general --config distinct tools/variants/lib_gen1.so indy-plenum_amd/libplenum_edverify.so > $OUT/ab_general_distinct.log 2>&1 || { cat $OUT/ab_general_distinct.log; exit 1; }
cat $OUT/ab_general_distinct.log
