#!/bin/bash
# rocprof kernel statistics of the BLS verify forms at a COMMIT round's 25 checks (GPU box, repo root).
# usage: bash tools/prof_bls.sh OUTDIR
export TMPDIR=/tmp
OUT=${1:?out dir}
mkdir -p "$OUT"
for form in wave quad; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$form" -o run \
    -- python3 tools/bls_probe.py $form 25 25 25 25 25 > "$OUT/$form.log" 2>&1 || exit $?
done
find "$OUT" -name "*kernel_stats*.csv" | sort
