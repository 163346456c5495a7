#!/bin/bash
# round-end validation in one gpurun call: GPU suite, smoke, config-2 bench (default vs DV_POOL_SPLIT
# pairs), then a config-2 kernel trace (summaries are copied into profiles/ by hand)
set -o pipefail
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_$i.log 2>&1 || exit 3
  DV_POOL_SPLIT=block3_conv3,block4_conv3 timeout -k 10 200 python bench.py > $O/bench_split_$i.log 2>&1 || exit 3
done
echo validated
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/prof_final2 -o bench -- python3 bench.py --steps 5 --warmup 2 > $O/prof.log 2>&1 || exit 6
echo profiled
