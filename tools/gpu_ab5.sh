set -o pipefail
mkdir -p gpurun_out
L=tools/variants/lib_kw.so
for c in c1 c2; do
for w in 14 15 16; do
timeout -k 10 300 python -u tools/ab_libs.py --rounds 1 --window $w --config $c $L >> gpurun_out/ab5_kw.log 2>&1 || exit $?
done
done
for w in 16 15 14; do
timeout -k 10 300 python -u tools/ab_libs.py --rounds 1 --window $w --config c2 $L >> gpurun_out/ab5_kw.log 2>&1 || exit $?
done
