# DeepDream GPU tests + config 3 bench (+ kernel trace when PROF=1)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
timeout -k 10 300 python -u -m pytest tests/test_deepdream.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_dream.log 2>&1 || exit 1
timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/c3_$TAG.log 2>&1 || exit 1
if [ "${PROF:-0}" = "1" ]; then TAG=$TAG bash tools/_gpu_trace_c3.sh || exit 1; fi
