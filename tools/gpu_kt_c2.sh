#!/bin/bash
# config-2 kernel trace (timed steps only) with idle-gap report
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/kt6
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace -d $O/raw -o c2 -- python3 bench.py --steps 8 --warmup 2 > $O/run.log 2>&1 || exit 1
python tools/kstats.py $(ls $O/raw/*.db $O/raw/*/*.db 2>/dev/null | head -1) --last-frac 0.55 --gaps --top 25 > $O/kstats.txt 2>&1 || exit 2
