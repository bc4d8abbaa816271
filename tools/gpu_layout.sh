#!/bin/bash
# Row-major key store: parity tests, then c1 / c2 / c3 at several key windows.
export TMPDIR=/tmp
OUT=gpurun_out/layout
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "keyed" -p no:cacheprovider > $OUT/tests.log 2>&1 || exit 1
for w in 10 13 14 16; do
  for c in c1 c2 c3; do
    timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --general-steps 0 --config $c --key-window $w > $OUT/b_${c}_$w.log 2>&1 || exit 1
  done
done
