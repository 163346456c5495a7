set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "pool or halo" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_ab.log 2>&1 || exit 1
timeout -k 10 120 python tools/profile_layers.py > gpurun_out/layers_ab0.txt 2>&1 || exit 1
timeout -k 10 100 python bench.py > gpurun_out/bench_ab.log 2>&1 || exit 1
for e in 0 1; do
  if [ $e = 1 ]; then export DV_NO_HS=1; fi
  timeout -k 10 200 python bench_dream.py --model resnet50 --size 1024 --tile 512 --batch 8 --dtype fp16 > gpurun_out/dream_c5_hs$e.log 2>&1 || exit 1
done
