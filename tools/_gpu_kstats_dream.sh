# kernel traces of DeepDream configs 3 and 5 -> kstats tables (TAG names the outputs)
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_c3 -o c3 -- python3 bench_dream.py --model inception_v3 --batch 64 --size 299 --runs 1 > gpurun_out/prof_c3_$TAG.log 2>&1 || exit 1
python tools/kstats.py $(find /tmp/prof_c3 -name '*.db' | head -n 1) --top 40 --last-frac 0.45 --gaps > gpurun_out/kstats_c3_$TAG.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_c5 -o c5 -- python3 bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 1 > gpurun_out/prof_c5_$TAG.log 2>&1 || exit 1
python tools/kstats.py $(find /tmp/prof_c5 -name '*.db' | head -n 1) --top 40 --last-frac 0.45 --gaps > gpurun_out/kstats_c5_$TAG.txt 2>&1
