#!/bin/bash
# v3 tail kernel: bit-identity + timing vs the shipped v2 schedule, then the tail GPU test
set -o pipefail
O=gpurun_out/tailv3
mkdir -p $O
timeout -k 10 120 python tools/tail_ab.py --vars 3,19 --rounds 5 --reps 10 > $O/ab.txt 2>&1 || exit 1
DV_ABLATIONS=1 timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "tail" -m gpu > $O/test.txt 2>&1 || exit 2
