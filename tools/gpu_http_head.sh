#!/bin/bash
# HTTP load at HEAD (8 front ends under the supervisor): mixed corpus and JPEG-only, 64 and 256 clients
set -o pipefail
O=gpurun_out/httphead
mkdir -p $O
DV_LOAD_SERVER_LOG=$O/server_mixed.log timeout -k 10 200 python tools/http_load.py --spawn --frontends 8 \
  --url http://127.0.0.1:18080 --clients 64,256 --procs 4 --seconds 8 --warmup 4 --out $O/mixed.json > $O/mixed.log 2>&1 || exit 1
DV_LOAD_SERVER_LOG=$O/server_jpeg.log timeout -k 10 200 python tools/http_load.py --spawn --frontends 8 --png-every 0 \
  --url http://127.0.0.1:18081 --clients 64,256 --procs 4 --seconds 8 --warmup 4 --out $O/jpeg.json > $O/jpeg.log 2>&1 || exit 2
