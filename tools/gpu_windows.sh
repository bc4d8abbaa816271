set -e
export PYTHONPATH=$PWD/indy-plenum_amd:$PWD
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "every_window or keyed" -p no:cacheprovider > gpurun_out/w_tests.log 2>&1
for w in 10 12 13 14 16; do
  timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --key-window $w > gpurun_out/w_bench_$w.log 2>&1
done
