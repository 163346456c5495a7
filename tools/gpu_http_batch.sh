#!/bin/bash
# HTTP: batcher max_batch sweep with 8 / 12 front ends (JPEG-only and mixed corpora)
set -o pipefail
O=gpurun_out/http4
mkdir -p $O
run() {  # name, frontends, max_batch, png_every
  DV_MAX_BATCH=$3 DV_LOAD_SERVER_LOG=$O/server_$1.log timeout -k 10 180 python tools/http_load.py --spawn --frontends $2 \
    --png-every $4 --url http://127.0.0.1:18080 --clients 256 --procs 4 --seconds 8 --warmup 4 --out $O/$1.json \
    > $O/$1.log 2>&1
}
run j8_b16 8 16 0 && run j8_b32 8 32 0 && run j8_b64 8 64 0 && run j12_b32 12 32 0 && run m8_b32 8 32 4 && run m12_b32 12 32 4 || exit 1
