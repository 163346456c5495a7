set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ks2.log 2>&1 || exit 1
DV_KS2=0 timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_ks2_off.txt 2>&1 || exit 1
timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_ks2_on.txt 2>&1 || exit 1
timeout -k 10 100 python bench.py > gpurun_out/bench_ks2.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/prof_c5 -o c5 -- python3 bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 --runs 1 > gpurun_out/prof_c5.log 2>&1 || exit 1
python tools/kstats.py $(find /tmp/prof_c5 -name '*.db' | head -n 1) --top 25 --last-frac 0.5 --gaps > gpurun_out/kstats_c5_gaps.txt 2>&1
