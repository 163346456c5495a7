#!/bin/bash
# config 5, all four octaves, 2 steps each, eager: per-kernel bytes (FETCH_SIZE / WRITE_SIZE) and MFMA busy
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc5
mkdir -p $O
CMD="python3 bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --steps 2 --runs 1 --warmup 0 --no-graphs"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/f -o f -- $CMD > $O/f.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES -d $O/w -o w -- $CMD > $O/w.log 2>&1 || exit 2
