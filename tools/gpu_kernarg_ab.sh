#!/bin/bash
# configs 3 and 5 (hipGraph replays of many small launches): HIP_FORCE_DEV_KERNARG=1 (kernel arguments in device
# memory) vs default
set -o pipefail
O=gpurun_out/kernarg
mkdir -p $O
C3="bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3"
C5="bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 2"
for r in 1 2; do
  timeout -k 10 300 python $C3 > $O/c3_base_$r.json 2>/dev/null || exit 1
  HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python $C3 > $O/c3_dev_$r.json 2>/dev/null || exit 2
done
timeout -k 10 300 python $C5 > $O/c5_base.json 2>/dev/null || exit 3
HIP_FORCE_DEV_KERNARG=1 timeout -k 10 300 python $C5 > $O/c5_dev.json 2>/dev/null || exit 4
