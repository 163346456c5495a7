set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "first_layer or stats or deprocess" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_c8.log 2>&1 || exit 1
timeout -k 10 60 python tools/bench_layer.py --case b1c1fwd --reps 10 > gpurun_out/c8.log 2>&1 || exit 1
DV_NO_C8_STREAM=1 timeout -k 10 60 python tools/bench_layer.py --case b1c1fwd --reps 10 >> gpurun_out/c8.log 2>&1 || exit 1
timeout -k 10 100 python bench.py > gpurun_out/bench.log 2>&1
