set -o pipefail
mkdir -p gpurun_out
for e in 0 1; do
  if [ $e = 1 ]; then export DV_NO_HS=1; fi
  timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/dream_c3_hs$e.log 2>&1 || exit 1
  timeout -k 10 200 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 > gpurun_out/dream_c5_hs$e.log 2>&1 || exit 1
done
