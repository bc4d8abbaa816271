export TMPDIR=/tmp
OUT=gpurun_out/r3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
AB_GENERAL=1 timeout -k 10 500 python -u tools/ab_keyed.py tools/variants/lib_base.so:10 tools/variants/lib_tw2.so:10 tools/variants/lib_tw3.so:10 tools/variants/lib_dw3.so:10 > $OUT/ab.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/ab.log
exit $rc
