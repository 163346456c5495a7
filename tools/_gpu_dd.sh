# deepdream GPU tests + the accumulating pool-backward kernel test
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deepdream.py tests/test_kernels_gpu.py -m gpu > gpurun_out/dd_tests.log 2>&1
