# ResNet conv1 direct input gradient: tests + config 5 A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deepdream.py -m gpu > gpurun_out/s7_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/s7_c5_on.log 2>&1 || exit 1
DV_STEM_DIRECT=0 timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/s7_c5_off.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/s7_c3.log 2>&1
