# full GPU suite + smoke + flagship bench + kernel-trace profile of the flagship (used between milestones)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 150 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_flag -o flag -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_bench.log 2>&1 || exit 1
python tools/kstats.py $(find /tmp/prof_flag -name '*.db' | head -n 1) --top 30 --last-frac 0.6 --gaps > gpurun_out/kstats_flag.txt 2>&1
