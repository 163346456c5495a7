#!/bin/bash
# front ends through the supervisor on a GPU box: the GPU front-end test, then a short HTTP load run
set -o pipefail
O=gpurun_out/fecheck
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 280 --timeout-method thread tests/test_frontends.py -m gpu > $O/test.txt 2>&1 || exit 1
DV_LOAD_SERVER_LOG=$O/server_http.log timeout -k 10 180 python tools/http_load.py --spawn --frontends 8 \
  --url http://127.0.0.1:18080 --clients 256 --procs 4 --seconds 8 --warmup 4 --out $O/http.json > $O/http.log 2>&1 || exit 2
