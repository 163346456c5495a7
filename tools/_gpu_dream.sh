# DeepDream configs 3 and 5 (1 GPU): GPU tests + benches (+ kernel-trace profile of config 5 with PROF=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_deepdream.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/t_dream.log 2>&1 || exit 1
timeout -k 10 200 python bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/dream_c3.log 2>&1 || exit 1
timeout -k 10 200 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 > gpurun_out/dream_c5.log 2>&1 || exit 1
if [ "${PROF:-0}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_c5 -o c5 -- python3 bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 1 > gpurun_out/prof_c5.log 2>&1 || exit 1
  python tools/kstats.py $(find /tmp/prof_c5 -name '*.db' | head -n 1) --top 40 --last-frac 0.5 --gaps > gpurun_out/kstats_c5.txt 2>&1
fi
