set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/ab_libs.py --rounds 2 tools/variants/lib_base.so tools/variants/lib_sha1.so > gpurun_out/ab2_c1.log 2>&1
