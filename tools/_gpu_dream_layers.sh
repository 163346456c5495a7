# per-conv-launch timing of one DeepDream step (configs 3 and 5 shapes)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 200 python tools/profile_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/dream_layers_c3_$TAG.txt 2>&1 || exit 1
timeout -k 10 200 python tools/profile_dream.py --model resnet50 --batch 32 --size 512 --octaves 1 --dtype fp16 > gpurun_out/dream_layers_c5_$TAG.txt 2>&1 || exit 1
