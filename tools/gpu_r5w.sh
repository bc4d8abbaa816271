#!/bin/bash
# The small keyed path reading its inputs from pinned host memory (EDV_SMALL_ZC=1) vs the H2D
# copy, and BLS with four lanes per check for small batches (every form tested and probed).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r5w
mkdir -p $OUT
EDV_SMALL_ZC=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_authn.py -k "small or single or drain" -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_zc.log 2>&1 || { tail -c 4000 $OUT/pytest_zc.log; exit 1; }
tail -n 1 $OUT/pytest_zc.log
for zc in 0 1 0 1; do
  if [ $zc = 1 ]; then export EDV_SMALL_ZC=1; else unset EDV_SMALL_ZC; fi
  PLENUM_EDVERIFY_LIB=tools/variants/lib_sprof.so timeout -k 10 200 python -u tools/small_probe.py 14 > $OUT/small_probe_zc$zc.log 2>&1 || { tail -c 3000 $OUT/small_probe_zc$zc.log; exit 1; }
  echo "== zero-copy $zc"; head -1 $OUT/small_probe_zc$zc.log | grep -v amdgpu.ids; grep "engine call\|end  " $OUT/small_probe_zc$zc.log
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_bls.py -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu_bls.log 2>&1 || { tail -c 4000 $OUT/pytest_gpu_bls.log; exit 1; }
tail -n 1 $OUT/pytest_gpu_bls.log
for f in quad pair one; do
  BLS_FORM=$f BLS_SIZES=1,25,1024,16384 timeout -k 10 300 python -u tools/bls_probe.py > $OUT/bls_probe_$f.log 2>&1 || { tail -c 3000 $OUT/bls_probe_$f.log; exit 1; }
  echo "form $f:"; grep "^n=" $OUT/bls_probe_$f.log
done
echo done
