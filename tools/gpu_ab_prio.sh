#!/bin/bash
# bench.py N=1 (default stream) and 1-rank RCCL (probed compute stream) + the RCCL GPU tests
set -o pipefail
O=gpurun_out/ab_prio2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_rccl_gpu.py -m gpu -x -v --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/n1_$i.log 2>&1 || exit 2
  timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2955$i bench.py --steps 10 --warmup 3 > $O/rccl1_$i.log 2>&1 || exit 3
done
