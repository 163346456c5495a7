#!/bin/bash
# one gpurun call: fused-stem tests, config-2 A/B (3 interleaved pairs), full GPU suite, smoke
set -o pipefail
mkdir -p gpurun_out
O=gpurun_out/stem
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_stem_fused_gpu.py "tests/test_kernels_gpu.py::test_seed_deconv" -x -v --timeout 120 --timeout-method thread > $O/pytest_stem.log 2>&1 || exit 1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/bench_fused_$i.log 2>&1 || exit 2
  DV_STEM_FUSE=0 timeout -k 10 200 python bench.py > $O/bench_unfused_$i.log 2>&1 || exit 3
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 4
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 5
echo done
