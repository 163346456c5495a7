#!/bin/bash
# round 6: config 2 DV_POOL_SPLIT A/B (3 interleaved pairs) + configs 3 and 5 at HEAD (3 runs each)
set -o pipefail
O=gpurun_out/${OUT:-val6}
mkdir -p $O
for i in 1 2 3; do
  DV_POOL_SPLIT= timeout -k 10 200 python bench.py > $O/c2_fused_$i.log 2>&1 || exit 1
  DV_POOL_SPLIT=block3_conv3,block4_conv3 timeout -k 10 200 python bench.py > $O/c2_split_$i.log 2>&1 || exit 2
done
echo c2 done
for i in 1 2 3; do
  timeout -k 10 300 python bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3 > $O/c3_$i.log 2>&1 || exit 3
done
echo c3 done
for i in 1 2 3; do
  timeout -k 10 400 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 3 > $O/c5_$i.log 2>&1 || exit 4
done
echo c5 done
