#!/bin/bash
# round 6: new GPU tests (fp16 engine, B=256 engine, sharded streams after them) + HTTP load through uvicorn
# (tools/http_load.py) for several front-end counts
set -o pipefail
O=gpurun_out/${OUT:-http2}
mkdir -p $O
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_fp16_and_bench_shape_gpu.py tests/test_sharded_streams_gpu.py} -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo tests ok
for fe in ${FES:-8 12}; do
  DV_LOAD_SERVER_LOG=$O/server_fe$fe.log timeout -k 10 180 python tools/http_load.py --spawn --frontends $fe \
    --url http://127.0.0.1:18080 --clients 64,256 --procs ${PROCS:-4} --seconds 8 --warmup 4 --out $O/http_fe$fe.json \
    > $O/http_fe$fe.log 2>&1 || exit 2
  echo fe $fe done
done
DV_LOAD_SERVER_LOG=$O/server_jpeg.log timeout -k 10 180 python tools/http_load.py --spawn --frontends 8 --png-every 0 \
  --url http://127.0.0.1:18080 --clients 64,256 --procs ${PROCS:-4} --seconds 8 --warmup 4 --out $O/http_fe8_jpeg.json \
  > $O/http_fe8_jpeg.log 2>&1 || exit 3
echo jpeg done
