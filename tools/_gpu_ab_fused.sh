# Inception one-node blocks: GPU tests + A/B on config 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_deepdream.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_dream.log 2>&1 || exit 1
DV_INCEPTION_FUSED=0 timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/c3_fused0.log 2>&1 || exit 1
DV_INCEPTION_FUSED=1 timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/c3_fused1.log 2>&1 || exit 1
