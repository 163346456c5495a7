# epilogue batch A/B: targeted kernel tests, then configs 5 and 3 with / without DV_NO_EPI_BATCH
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "residual or emask or accumulate" tests/test_deepdream.py -k "bottleneck or inception_block or residual or emask or accumulate" > gpurun_out/epi_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/epi_c5_on.log 2>&1 || exit 1
DV_NO_EPI_BATCH=1 timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/epi_c5_off.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/epi_c3_on.log 2>&1 || exit 1
DV_NO_EPI_BATCH=1 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/epi_c3_off.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py > gpurun_out/epi_c2_on.log 2>&1
