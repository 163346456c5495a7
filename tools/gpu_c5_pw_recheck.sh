#!/bin/bash
# config 5 re-check of the persistent 1x1 kernel's switches at HEAD: default, 1 workgroup per CU, pw off, K-min of the small tile
set -o pipefail
export DV_ABLATIONS=1
O=gpurun_out/c5pw
mkdir -p $O
C5="bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 2"
for r in 1 2; do
  timeout -k 10 300 python $C5 > $O/base_$r.json 2>/dev/null || exit 1
  DV_PW_WG_PER_CU=1 timeout -k 10 300 python $C5 > $O/wg1_$r.json 2>/dev/null || exit 2
  DV_NO_PW=1 timeout -k 10 300 python $C5 > $O/nopw_$r.json 2>/dev/null || exit 3
  DV_PW_MIN_TILES=512 timeout -k 10 300 python $C5 > $O/min512_$r.json 2>/dev/null || exit 4
done
