#!/bin/bash
# the 4-wave / two-workgroups-per-CU tail kernel: bit identity + timing vs the shipped v2 schedule
set -o pipefail
O=gpurun_out/tailv4
mkdir -p $O
timeout -k 10 150 python tools/tail_ab.py --vars 3,32,32f --rounds 5 --reps 10 > $O/ab.txt 2>&1 || exit 1
