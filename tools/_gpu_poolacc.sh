# accumulating pool backward in the Inception max branch: tests + config 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deepdream.py tests/test_kernels_gpu.py -m gpu > gpurun_out/pa_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/pa_c3.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/pa_c3b.log 2>&1
