# GPU suite + flagship bench + serving latency/throughput (staging ring)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit 1
timeout -k 10 150 python bench.py > gpurun_out/bench_$TAG.log 2>&1 || exit 1
timeout -k 10 300 python tools/latency.py --clients 1,16,64,128 --requests 1024 > gpurun_out/latency_$TAG.json 2>gpurun_out/latency_$TAG.err || exit 1
