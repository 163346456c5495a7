set -o pipefail
mkdir -p gpurun_out
S="--shape 1024,112,112,128,128,3,1 --shape 1024,56,56,256,128,3,1 --shape 1024,28,28,512,512,3,1 --shape 1024,14,14,512,512,3,1 --shape 1024,56,56,256,256,3,1"
timeout -k 10 120 python tools/bench_conv.py $S --iters 10 > gpurun_out/wide.log 2>&1 || exit 1
DV_WIDE_WAVES=3 timeout -k 10 120 python tools/bench_conv.py $S --iters 10 >> gpurun_out/wide.log 2>&1 || exit 1
DV_WIDE_WAVES=3 timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/wide_tests.log 2>&1 || exit 1
DV_WIDE_WAVES=3 timeout -k 10 100 python bench.py > gpurun_out/bench_wide.log 2>&1
