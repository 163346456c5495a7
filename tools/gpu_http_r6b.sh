#!/bin/bash
# HTTP load after the front-end CPU fixes (fast JSON string body, counter request ids, GIL kept for tiny
# native calls): 8 front ends, mixed and JPEG-only corpora
set -o pipefail
O=gpurun_out/http3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_frontends.py -m gpu -x -v --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
mkdir -p $O
for fe in 8; do
  DV_LOAD_SERVER_LOG=$O/server_fe$fe.log timeout -k 10 180 python tools/http_load.py --spawn --frontends $fe \
    --url http://127.0.0.1:18080 --clients 64,256 --procs 4 --seconds 8 --warmup 4 --out $O/http_fe$fe.json \
    > $O/http_fe$fe.log 2>&1 || exit 2
done
DV_LOAD_SERVER_LOG=$O/server_jpeg.log timeout -k 10 180 python tools/http_load.py --spawn --frontends 8 --png-every 0 \
  --url http://127.0.0.1:18080 --clients 64,256 --procs 4 --seconds 8 --warmup 4 --out $O/http_fe8_jpeg.json \
  > $O/http_fe8_jpeg.log 2>&1 || exit 3
DV_LOAD_SERVER_LOG=$O/server_jpeg12.log timeout -k 10 180 python tools/http_load.py --spawn --frontends 12 --png-every 0 \
  --url http://127.0.0.1:18080 --clients 256 --procs 4 --seconds 8 --warmup 4 --out $O/http_fe12_jpeg.json \
  > $O/http_fe12_jpeg.log 2>&1 || exit 4
timeout -k 10 300 python tools/aten_trace.py --model inception_v3 --batch 64 --size 299 > $O/aten_c3.log 2>&1 || exit 5
