#!/bin/bash
# Key-sorted comb order (edv_set_key_sort): the parity tests of the keyed path, then the A/B of
# key windows 14 / 16 with the sort on and off for configs[1] (arrival order) and configs[2]
# (key ids in np.unique order).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "keyed or key_sorted or sub_batch" > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 2 $OUT/pytest_gpu.log
A="--no-cpu --general-steps 0 --e2e-n 0 --e2e-c0 0 --dropin-steps 0 --e2e-devices 0"
for c in c1 c2; do for w in 14 16; do for k in off auto; do
  timeout -k 10 300 python -u bench.py $A --config $c --key-window $w --key-sort $k > $OUT/${c}_w${w}_$k.log 2>&1 || { tail -c 3000 $OUT/${c}_w${w}_$k.log; exit 1; }
done; done; done
for f in $OUT/c*.log; do python - $f <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{"metric')][-1]; d=json.loads(l)
print(sys.argv[1].split('/')[-1], round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],3), 'ms frac', round(d['roofline']['frac'],3), {k:round(v,3) for k,v in d['phase_ms'].items() if k!='note'}, 'mism', d['parity']['mismatches_vs_construction'])
PY
done
echo done
