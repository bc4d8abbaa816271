#!/bin/bash
# PMC passes for the bench workload (run on the GPU box from the repo root).
# One counter group per rocprofv3 run (gfx950 slot limits: TCC 4 -- FETCH_SIZE
# takes 3, WRITE_SIZE 2 -- SQ 8, GRBM 2); --pmc is never combined with tracing
# domains.  Summaries: python tools/pmc_summary.py gpurun_out/pmc
export TMPDIR=/tmp
ARGS="--steps 2 --warmup 1 --no-cpu --general-steps 1 --pipeline 1 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 --churn-signers 0 --drain-n 0 --bls-checks 0"
OUT=gpurun_out/pmc
mkdir -p $OUT
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/sq2 -o run -- python3 bench.py $ARGS > $OUT/sq2.log 2>&1
rc=$?
find $OUT -name "*.csv" | sort
exit $rc
