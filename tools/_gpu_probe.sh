set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_now.txt 2>&1 || exit 1
timeout -k 10 180 python tools/gemm_ceiling.py > gpurun_out/gemm_ceiling.txt 2>&1
