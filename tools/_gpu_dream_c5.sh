# DeepDream GPU tests + config 5 bench (tiled 1024^2, whole-octave graph)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 300 python -u -m pytest tests/test_deepdream.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_dream.log 2>&1 || exit 1
timeout -k 10 200 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 > gpurun_out/c5_$TAG.log 2>&1 || exit 1
