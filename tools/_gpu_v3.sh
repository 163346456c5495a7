set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "pool" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pool.log 2>&1 || exit 1
timeout -k 10 60 python tools/bench_layer.py --case b1c2fwd --reps 10 > gpurun_out/v3.log 2>&1 || exit 1
DV_NO_POOL_V3=1 timeout -k 10 60 python tools/bench_layer.py --case b1c2fwd --reps 10 >> gpurun_out/v3.log 2>&1 || exit 1
timeout -k 10 100 python bench.py > gpurun_out/bench.log 2>&1
