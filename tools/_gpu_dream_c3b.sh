set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 300 python -u -m pytest tests/test_deepdream.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/t_dream.log 2>&1 || exit 1
timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/c3_$TAG.log 2>&1 || exit 1
timeout -k 10 200 python tools/profile_dream.py --model inception_v3 --batch 64 --size 299 --top 30 > gpurun_out/dream_layers_c3_$TAG.txt 2>&1 || exit 1
