#!/bin/bash
# sweep: small-problem split-K ceiling (DV_SMALL_SPLITK_MN) on configs 3 and 5
set -o pipefail
export DV_ABLATIONS=1
O=gpurun_out/splitk
mkdir -p $O
C3="bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3"
C5="bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 2"
for i in 1 2; do
  for mn in 300000 1000000 3000000; do
    DV_SMALL_SPLITK_MN=$mn timeout -k 10 300 python $C3 > $O/c3_mn${mn}_$i.log 2>&1 || exit 1
  done
done
echo c3 done
for mn in 300000 1000000 3000000; do
  DV_SMALL_SPLITK_MN=$mn timeout -k 10 400 python $C5 > $O/c5_mn${mn}.log 2>&1 || exit 2
done
echo c5 done
