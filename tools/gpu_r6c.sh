#!/bin/bash
# Streamed path chunk size A/B (2^18 / 2^17 / 2^16, alternating in one process).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r6c
mkdir -p $OUT
timeout -k 10 500 python -u tools/stream_ab.py 1000000 4 > $OUT/stream_ab.log 2>&1 || { tail -c 3000 $OUT/stream_ab.log; exit 1; }
grep "^chunk" $OUT/stream_ab.log
echo done
