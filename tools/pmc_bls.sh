#!/bin/bash
# PMC passes over the BLS wave-form probe (25 checks): one counter group per rocprofv3 run.
# usage (GPU box, repo root): bash tools/pmc_bls.sh OUTDIR [LIB]
export TMPDIR=/tmp
OUT=${1:?out dir}
[ -n "$2" ] && export PLENUM_EDVERIFY_LIB=$2
mkdir -p "$OUT"
P="tools/bls_probe.py wave 25"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sq" -o run -- python3 $P > "$OUT/sq.log" 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH --output-format csv -d "$OUT/sq2" -o run -- python3 $P > "$OUT/sq2.log" 2>&1
rc=$?
find "$OUT" -name "*counter_collection*.csv" | sort
exit $rc
