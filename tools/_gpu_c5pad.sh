# conv2d_5 on the halo-stream kernels (80 -> 96 channel padding, 192-channel split) + min-width knob
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_deepdream.py -m gpu > gpurun_out/c5p_tests.log 2>&1 || exit 1
c3() { env "$@" timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299; }
c3 DV_PAD_STEM=1 > gpurun_out/c5p_on.log 2>&1 || exit 1
c3 DV_PAD_STEM=0 > gpurun_out/c5p_off.log 2>&1 || exit 1
c3 DV_HS_MIN_W=48 > gpurun_out/c5p_w48.log 2>&1 || exit 1
c3 DV_HS_MIN_W=32 > gpurun_out/c5p_w32.log 2>&1 || exit 1
c3 DV_PAD_STEM=1 > gpurun_out/c5p_on2.log 2>&1 || exit 1
