export TMPDIR=/tmp
OUT=gpurun_out/r3
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
AB_GENERAL=0 timeout -k 10 500 python -u tools/ab_keyed.py indy-plenum_amd/libplenum_edverify.so:8 tools/variants/lib_b12.so:10 tools/variants/lib_b14.so:10 tools/variants/lib_b16.so:10 tools/variants/lib_b16.so:8 > $OUT/ab.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/ab.log
exit $rc
