#!/bin/bash
# HTTP batcher with bucket trimming (max_batch 32 vs 64) + the config-2 knob re-check
set -o pipefail
O=gpurun_out/http5
mkdir -p $O
run() {  # name, frontends, max_batch, png_every
  DV_MAX_BATCH=$3 DV_LOAD_SERVER_LOG=$O/server_$1.log timeout -k 10 180 python tools/http_load.py --spawn --frontends $2 \
    --png-every $4 --url http://127.0.0.1:18080 --clients 256 --procs 4 --seconds 8 --warmup 4 --out $O/$1.json \
    > $O/$1.log 2>&1
}
run j8_b32 8 32 0 && run j8_b64 8 64 0 && run m8_b32 8 32 4 && run m8_b64 8 64 4 || exit 1
echo http done
bash tools/gpu_c2_knob_sweep.sh || exit 2
