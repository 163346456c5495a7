# tile-config x split-K sweep on every conv launch of one DeepDream step (configs 3 and 5 shapes)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 400 python tools/tune_dma.py --model inception_v3 --batch 64 --size 299 --json gpurun_out/tune_c3_$TAG.json > gpurun_out/tune_c3_$TAG.txt 2>&1 || exit 1
timeout -k 10 400 python tools/tune_dma.py --model resnet50 --batch 32 --size 512 --octaves 1 --dtype fp16 --json gpurun_out/tune_c5_$TAG.json > gpurun_out/tune_c5_$TAG.txt 2>&1 || exit 1
