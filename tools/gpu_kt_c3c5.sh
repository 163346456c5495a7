#!/bin/bash
# kernel traces of configs 3 and 5 at HEAD, summarized per kernel (tools/kstats.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/kt35
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/c3 -o c3 -- python3 bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 2 --warmup 1 > $O/c3.log 2>&1 || exit 1
python tools/kstats.py $(ls $O/c3/*.db $O/c3/*/*.db 2>/dev/null | head -1) --last-frac 0.45 --top 25 > $O/kstats_c3.txt 2>&1 || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/c5 -o c5 -- python3 bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 2 --warmup 1 > $O/c5.log 2>&1 || exit 3
python tools/kstats.py $(ls $O/c5/*.db $O/c5/*/*.db 2>/dev/null | head -1) --last-frac 0.45 --top 25 > $O/kstats_c5.txt 2>&1 || exit 4
