#!/bin/bash
# config-2 stall counters (one pass, 8 SQ + 1 GRBM), summarized per kernel
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/pmc6
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/raw -o c2 -- python3 bench.py --steps 2 --warmup 1 > $O/run.log 2>&1 || exit 1
python tools/pmc_summary.py $O/raw --top 14 > $O/summary.txt 2>&1 || exit 2
