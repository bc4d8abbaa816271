#!/bin/bash
# Key window 13 vs 14 at the current base window, alternating on one box.
export TMPDIR=/tmp
OUT=gpurun_out/abkw
mkdir -p $OUT
for v in 13 14 13b 14b; do
  for c in c1 c2 c3; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --config $c --key-window ${v:0:2} > $OUT/w${v}_$c.log 2>&1 || exit 1
  done
done
