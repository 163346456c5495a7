set -o pipefail
mkdir -p gpurun_out
DV_DMA_VARIANT=5 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "large_m" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_dmav.log 2>&1 || exit 1
DV_DMA_VARIANT=6 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "large_m" -x -q --timeout 120 --timeout-method thread >> gpurun_out/t_dmav.log 2>&1 || exit 1
for v in 0 5 6; do
  DV_DMA_VARIANT=$v timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_dmav$v.txt 2>&1 || exit 1
done
