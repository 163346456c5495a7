#!/bin/bash
# config 5: is the host (graph launch / AQL queue back-pressure) on the critical path? ROC_AQL_QUEUE_SIZE A/B
set -o pipefail
O=gpurun_out/c5aql
mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 3 > $O/$n.json 2>$O/$n.err || exit 1
}
run base DV_NOP=1
run q16k ROC_AQL_QUEUE_SIZE=16384
run q64k ROC_AQL_QUEUE_SIZE=65536
run base2 DV_NOP=1
