#!/bin/bash
set -o pipefail
O=gpurun_out/merge
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_subpixel_merge_gpu.py tests/test_deepdream.py -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/aten_trace.py --model inception_v3 --batch 64 --size 299 > $O/aten_c3.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 300 python bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 3 > $O/c3_$i.log 2>&1 || exit 3
done
timeout -k 10 400 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 2 > $O/c5.log 2>&1 || exit 4
