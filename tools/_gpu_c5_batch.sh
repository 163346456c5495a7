set -o pipefail
mkdir -p gpurun_out
for b in 2 4 8 16; do
timeout -k 10 300 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch $b --dtype fp16 > gpurun_out/c5_b$b.log 2>&1 || exit 1
done
