#!/bin/bash
# Scan with the flat identifier table: e2e probe at part sizes 0 / 2^17 / 2^18, shared-object
# requests and wire-decoded requests (each json-decoded on its own).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5c
mkdir -p $OUT
EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0,131072,262144 > $OUT/e2e_probe.log 2>&1 || { tail -c 3000 $OUT/e2e_probe.log; exit 1; }
grep -E "^authenticate_batch|^single|^built" $OUT/e2e_probe.log
WIRE=1 EDV_SCAN_PROFILE=1 timeout -k 10 400 python -u tools/e2e_probe.py 1000000 0,262144 > $OUT/e2e_probe_wire.log 2>&1 || { tail -c 3000 $OUT/e2e_probe_wire.log; exit 1; }
grep -E "^authenticate_batch|^built" $OUT/e2e_probe_wire.log
grep -E "^scan: n=1000000" $OUT/e2e_probe.log | tail -2
grep -E "^scan: n=1000000" $OUT/e2e_probe_wire.log | tail -2
echo done
