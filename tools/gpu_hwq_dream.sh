#!/bin/bash
# A/B: GPU_MAX_HW_QUEUES (hardware queues per process) for the DeepDream configs, whose sub-batches /
# chunks run as parallel graph branches; plus wider splits with more queues
set -o pipefail
export DV_ABLATIONS=1
O=gpurun_out/hwq
mkdir -p $O
C3="bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3"
C5="bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 2"
for i in 1 2; do
  timeout -k 10 300 python $C3 > $O/c3_q4_$i.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python $C3 > $O/c3_q8_$i.log 2>&1 || exit 1
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python $C3 > $O/c3_q16_$i.log 2>&1 || exit 1
done
GPU_MAX_HW_QUEUES=16 DV_DREAM_SPLIT=3 timeout -k 10 300 python $C3 > $O/c3_q16_s3.log 2>&1 || exit 1
GPU_MAX_HW_QUEUES=16 DV_DREAM_SPLIT=4 timeout -k 10 300 python $C3 > $O/c3_q16_s4.log 2>&1 || exit 1
echo c3 done
for i in 1 2; do
  timeout -k 10 400 python $C5 > $O/c5_q4_$i.log 2>&1 || exit 2
  GPU_MAX_HW_QUEUES=8 timeout -k 10 400 python $C5 > $O/c5_q8_$i.log 2>&1 || exit 2
  GPU_MAX_HW_QUEUES=16 timeout -k 10 400 python $C5 > $O/c5_q16_$i.log 2>&1 || exit 2
done
GPU_MAX_HW_QUEUES=16 DV_TILE_LOCAL_CHUNKS=4 DV_TILE_CHUNK_STREAMS=4 timeout -k 10 400 python $C5 > $O/c5_q16_c4.log 2>&1 || exit 2
echo c5 done
