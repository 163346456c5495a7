# kernel trace of config 3 (branch streams on): concurrency check
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_c3 -o c3 -- python3 bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 1 ${EXTRA:-} > gpurun_out/prof_c3_$TAG.log 2>&1 || exit 1
python tools/kstats.py $(find /tmp/prof_c3 -name '*.db' | head -n 1) --top 45 --last-frac 0.4 --gaps > gpurun_out/kstats_c3_$TAG.txt 2>&1
