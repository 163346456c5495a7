# A/B: InceptionV3 branch streams on/off (config 3) + the DeepDream GPU tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_deepdream.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_dream.log 2>&1 || exit 1
DV_BRANCH_STREAMS=0 timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/c3_streams0.log 2>&1 || exit 1
DV_BRANCH_STREAMS=1 timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/c3_streams1.log 2>&1 || exit 1
