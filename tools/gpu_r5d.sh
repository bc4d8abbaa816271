#!/bin/bash
# A/B of the comb's gather locality: key windows 14 / 16 with the batch in arrival order (request i
# signed by signer i % 1000, every lane of a wave on a different key) and sorted by signer.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5d
mkdir -p $OUT
A="--no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 --e2e-devices 0"
for w in 14 16; do for o in arrival sorted; do
  timeout -k 10 300 python -u bench.py $A --key-window $w --key-order $o > $OUT/c1_w${w}_$o.log 2>&1 || { tail -c 3000 $OUT/c1_w${w}_$o.log; exit 1; }
done; done
for w in 14 16; do
  timeout -k 10 300 python -u bench.py $A --config c2 --key-window $w > $OUT/c2_w${w}.log 2>&1 || { tail -c 3000 $OUT/c2_w${w}.log; exit 1; }
done
for f in $OUT/*.log; do python - $f <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[1].split('/')[-1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms frac', round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, 'build_ms', round(d['key_table_build_ms'],1), 'mism', d['parity']['mismatches_vs_construction'])
PY
done
echo done
