set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/copy_overlap_probe.py > gpurun_out/cp_default.log 2>&1 || exit 1
GPU_BLIT_ENGINE_TYPE=2 timeout -k 10 120 python -u tools/copy_overlap_probe.py > gpurun_out/cp_engine2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/cp_prof -o cp -- python -u tools/copy_overlap_probe.py > gpurun_out/cp_prof.log 2>&1 || exit 1
