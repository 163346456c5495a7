set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "kw3 or large_m or unpool_out or fwd_bf16 or residual or splitk" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_kw3.log 2>&1 || exit 1
DV_KW3=0 timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_kw3_off.txt 2>&1 || exit 1
DV_KW3_FP=0 timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_kw3_nofp.txt 2>&1 || exit 1
timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_kw3_on.txt 2>&1 || exit 1
timeout -k 10 100 python bench.py > gpurun_out/bench_kw3.log 2>&1
