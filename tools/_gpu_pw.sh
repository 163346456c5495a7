# persistent pointwise kernel: targeted tests, then config 5 / 3 / 2 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pointwise" > gpurun_out/pw_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_deepdream.py -m gpu > gpurun_out/pw_tests_all.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/pw_c5_on.log 2>&1 || exit 1
DV_NO_PW=1 timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/pw_c5_off.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/pw_c3_on.log 2>&1 || exit 1
DV_NO_PW=1 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/pw_c3_off.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py > gpurun_out/pw_c2.log 2>&1
