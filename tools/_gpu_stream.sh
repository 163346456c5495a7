set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -k "halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_halo.log 2>&1 || exit 1
for P in 1 2 3; do DV_STREAM_P=$P timeout -k 10 60 python tools/bench_layer.py --case b1c1down --reps 10 >> gpurun_out/stream_p.log 2>&1 || exit 1; done
DV_HALO_V1=1 timeout -k 10 60 python tools/bench_layer.py --case b1c1down --reps 10 >> gpurun_out/stream_p.log 2>&1 || exit 1
timeout -k 10 100 python bench.py > gpurun_out/bench.log 2>&1
