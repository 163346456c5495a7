# full GPU suite + flagship bench + smoke
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 150 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
