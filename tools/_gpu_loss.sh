# pool specialization + fused loss partials: tests + configs 3/5 (A/B on the fused loss)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deepdream.py tests/test_kernels_gpu.py -m gpu > gpurun_out/loss_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/loss_c3_on.log 2>&1 || exit 1
DV_DREAM_FUSED_LOSS=0 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/loss_c3_off.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/loss_c5_on.log 2>&1 || exit 1
DV_DREAM_FUSED_LOSS=0 timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/loss_c5_off.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/dream_octave_times.py --split 2 > gpurun_out/loss_oct.log 2>&1
