export TMPDIR=/tmp
OUT=gpurun_out/r2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 &&
timeout -k 10 400 python -u tools/ab_keyed.py indy-plenum_amd/libplenum_edverify.so:8 indy-plenum_amd/libplenum_edverify.so:6 indy-plenum_amd/libplenum_edverify.so:4 tools/variants/lib_cw4.so:8 tools/variants/lib_m8.so:8 tools/variants/lib_m32.so:8 > $OUT/ab.log 2>&1 &&
timeout -k 10 300 python -u bench.py > $OUT/bench_c1.log 2>&1
rc=$?
tail -3 $OUT/pytest_gpu.log; cat $OUT/ab.log; tail -1 $OUT/bench_c1.log
exit $rc
