set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo_stream" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_hs.log 2>&1 || exit 1
DV_HS_RING=5 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "halo_stream" -x -q --timeout 120 --timeout-method thread >> gpurun_out/t_hs.log 2>&1 || exit 1
for r in 3 4 5; do
  DV_HS_RING=$r timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_hs_ring$r.txt 2>&1 || exit 1
done
timeout -k 10 100 python bench.py > gpurun_out/bench_hs.log 2>&1
