set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo_stream or relu_in or large_m or unpool" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hs.log 2>&1 || exit 1
DV_NO_HSU=1 timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_hsu_off.txt 2>&1 || exit 1
timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_hsu_on.txt 2>&1 || exit 1
timeout -k 10 100 python bench.py > gpurun_out/bench_hs.log 2>&1
