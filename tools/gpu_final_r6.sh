#!/bin/bash
# round-6 end validation in one gpurun call: GPU suite, smoke, config-2 bench x3, configs 3 and 5, HTTP load
set -o pipefail
O=gpurun_out/final6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 1
echo suite ok
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/bench_$i.log 2>&1 || exit 3
done
timeout -k 10 300 python bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3 > $O/c3.log 2>&1 || exit 4
timeout -k 10 400 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 3 > $O/c5.log 2>&1 || exit 5
DV_LOAD_SERVER_LOG=$O/server_http.log timeout -k 10 180 python tools/http_load.py --spawn --frontends 8 \
  --url http://127.0.0.1:18080 --clients 64,256 --procs 4 --seconds 8 --warmup 4 --out $O/http_fe8.json \
  > $O/http_fe8.log 2>&1 || exit 6
echo validated
