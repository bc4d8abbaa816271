set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_libs.py --rounds 2 tools/variants/lib_base.so tools/variants/lib_lds.so > gpurun_out/ab1_c1.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --rounds 1 --config c2 tools/variants/lib_base.so tools/variants/lib_lds.so > gpurun_out/ab1_c2.log 2>&1
