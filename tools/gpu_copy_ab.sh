#!/bin/bash
# config 2: where the mosaics' copy-back is issued (step start vs block3_conv1 hook) vs none (diagnostic)
set -o pipefail
O=gpurun_out/copyab
mkdir -p $O
for r in 1 2; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 > $O/base_$r.json 2>$O/base_$r.err || exit 1
  DV_BENCH_COPY_AT=block3_conv1 timeout -k 10 150 python bench.py --steps 20 --warmup 3 > $O/at_b3_$r.json 2>$O/at_$r.err || exit 1
  DV_BENCH_COPY_AT=block4_conv1 timeout -k 10 150 python bench.py --steps 20 --warmup 3 > $O/at_b4_$r.json 2>$O/at4_$r.err || exit 1
  timeout -k 10 150 python bench.py --steps 20 --warmup 3 --no-copyback > $O/nocopy_$r.json 2>$O/nocopy_$r.err || exit 1
done
