#!/bin/bash
# Launch-parameter sweep on one box: sub-batches per chunk and key window (configs[1] / [2]).
export TMPDIR=/tmp
OUT=gpurun_out/abp
mkdir -p $OUT
for p in 4 2 3; do
  for c in c1 c2; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --config $c --pipeline $p > $OUT/p${p}_$c.log 2>&1 || exit 1
  done
done
for w in 12 14 13; do
  for c in c1 c2; do
    timeout -k 10 200 python -u bench.py --steps 30 --warmup 3 --no-cpu --general-steps 0 --config $c --key-window $w > $OUT/w${w}_$c.log 2>&1 || exit 1
  done
done
