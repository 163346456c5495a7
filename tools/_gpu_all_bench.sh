# GPU suite + flagship bench + DeepDream configs 3 and 5
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 150 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/c3_$TAG.log 2>&1 || exit 1
timeout -k 10 200 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 > gpurun_out/c5_$TAG.log 2>&1 || exit 1
