set -o pipefail
mkdir -p gpurun_out
S="--shape 1024,112,112,128,128,3,1 --shape 1024,56,56,256,128,3,1 --shape 256,112,112,64,128,3,1 --shape 256,112,112,128,128,3,1"
timeout -k 10 120 python tools/bench_conv.py $S --iters 10 > gpurun_out/t128.log 2>&1 || exit 1
DV_TILE128_M=512 timeout -k 10 120 python tools/bench_conv.py $S --iters 10 >> gpurun_out/t128.log 2>&1 || exit 1
DV_TILE128_M=512 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t128_tests.log 2>&1 || exit 1
DV_TILE128_M=512 timeout -k 10 100 python bench.py > gpurun_out/bench512.log 2>&1
