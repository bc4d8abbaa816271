set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_libs.py --rounds 2 --path general tools/variants/lib_gen0.so tools/variants/lib_gen1.so > gpurun_out/ab4_gen.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab_libs.py --rounds 1 tools/variants/lib_gen0.so tools/variants/lib_gen1.so > gpurun_out/ab4_keyed.log 2>&1
