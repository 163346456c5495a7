#!/bin/bash
# config-2 re-check of A/B switches after round 6's defaults changed (pool split, probed streams)
set -o pipefail
export DV_ABLATIONS=1
O=gpurun_out/c2sweep
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/base_$i.log 2>&1 || exit 1
  DV_KW3_SK=all timeout -k 10 200 python bench.py > $O/skall_$i.log 2>&1 || exit 1
  DV_KW3_TILE=512x128 timeout -k 10 200 python bench.py > $O/t512_$i.log 2>&1 || exit 1
  DV_NO_KW3_SK=1 timeout -k 10 200 python bench.py > $O/nosk_$i.log 2>&1 || exit 1
  DV_POOL_SPLIT=block2_conv2,block3_conv3,block4_conv3,block5_conv3 timeout -k 10 200 python bench.py > $O/split4_$i.log 2>&1 || exit 1
  DV_POOL_SPLIT=block3_conv3,block4_conv3,block5_conv3 timeout -k 10 200 python bench.py > $O/split3_$i.log 2>&1 || exit 1
done
