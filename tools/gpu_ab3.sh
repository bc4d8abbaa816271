set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u tools/ab_libs.py --rounds 2 tools/variants/lib_sha1.so tools/variants/lib_mc2.so > gpurun_out/ab3_c1.log 2>&1
