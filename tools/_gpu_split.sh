# DeepDream sub-batch split x hardware-queue count sweep (config 3)
set -o pipefail
mkdir -p gpurun_out
for cfg in "2 4" "2 8" "4 8" "4 16" "8 16"; do
  set -- $cfg
  DV_DREAM_SPLIT=$1 GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/split_$1_q$2.log 2>&1 || exit 1
done
