#!/bin/bash
# A/B: stream probing (independent copy stream) vs plain pool streams vs 8 hardware queues, config 2 bench.py
set -o pipefail
export DV_ABLATIONS=1  # the A/B switches below are honoured only in ablation mode (knobs.py)
O=gpurun_out/ab_streams
mkdir -p $O
for i in 1 2 3; do
  DV_NO_STREAM_PROBE=1 timeout -k 10 200 python bench.py > $O/plain_$i.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py > $O/probe_$i.log 2>&1 || exit 2
  GPU_MAX_HW_QUEUES=8 timeout -k 10 200 python bench.py > $O/hwq8_$i.log 2>&1 || exit 3
done
grep -h '"value"' $O/*.log | cut -c1-120
