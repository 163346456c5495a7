#!/bin/bash
# configs 5 and 3: smallest map side routed to the halo-stream 3x3 kernels (DV_HS_MIN_W, default 64)
set -o pipefail
export DV_ABLATIONS=1
O=gpurun_out/hsminw
mkdir -p $O
C5="bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 2"
C3="bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3"
for r in 1 2; do
  for w in 64 96 128; do
    DV_HS_MIN_W=$w timeout -k 10 300 python $C5 > $O/c5_w${w}_$r.json 2>/dev/null || exit 1
  done
done
for w in 96; do
  DV_HS_MIN_W=$w timeout -k 10 300 python $C3 > $O/c3_w${w}.json 2>/dev/null || exit 2
done
