#!/bin/bash
# config 3 (InceptionV3 DeepDream, batch 64, 299^2): bf16 vs fp16 storage (same MFMA rate; some fused paths bf16-only)
set -o pipefail
O=gpurun_out/c3dtype
mkdir -p $O
for r in 1 2; do
  for dt in bf16 fp16; do
    timeout -k 10 300 python bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3 --dtype $dt > $O/${dt}_$r.json 2>$O/${dt}_$r.err || exit 1
  done
done
