#!/bin/bash
# Small-kernel phase probes (order 1 vs 2), authenticator GPU tests, the e2e probe with the
# staged scan's copier thread, the bench's e2e legs.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5o
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_authn.py tests/test_gpu_parity.py -k "small or drain or single" -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu.log; exit 1; }
tail -n 1 $OUT/pytest_gpu.log
for v in sprof sprof3; do
  PLENUM_EDVERIFY_LIB=tools/variants/lib_$v.so timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_$v.log 2>&1 || { tail -c 3000 $OUT/small_probe_$v.log; exit 1; }
  echo "== $v"; cat $OUT/small_probe_$v.log | tail -9
done
timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_default.log 2>&1 || { tail -c 3000 $OUT/small_probe_default.log; exit 1; }
echo "== default"; tail -2 $OUT/small_probe_default.log
echo done
