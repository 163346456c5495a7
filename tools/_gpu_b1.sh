# b1 merged into the Inception head GEMM (two-destination epilogue): tests + config 3 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_deepdream.py -m gpu > gpurun_out/b1_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/b1_on.log 2>&1 || exit 1
DV_MERGE_B1=0 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/b1_off.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/b1_on2.log 2>&1 || exit 1
DV_MERGE_B1=0 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/b1_off2.log 2>&1 || exit 1
