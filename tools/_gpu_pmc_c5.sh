# PMC passes (one counter group per run) over a short eager config-5 workload
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 --octaves 1 --steps 2 --runs 1 --warmup 0 --no-graphs"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_MFMA --output-format csv -d /tmp/pmc1 -o p1 -- python3 $ARGS > gpurun_out/pmc_c5_p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc2 -o p2 -- python3 $ARGS > gpurun_out/pmc_c5_p2.log 2>&1 || exit 1
python tools/pmc_summary.py /tmp/pmc1 --top 12 > gpurun_out/pmc_c5_sum1.txt 2>&1
python tools/pmc_summary.py /tmp/pmc2 --top 12 > gpurun_out/pmc_c5_sum2.txt 2>&1
mkdir -p gpurun_out/pmc_c5 && cp $(find /tmp/pmc1 /tmp/pmc2 -name '*counter_collection.csv') gpurun_out/pmc_c5/ 2>/dev/null; ls gpurun_out/pmc_c5
