# direct stem conv kernels: tests + config 3 A/B + layer table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_deepdream.py -m gpu > gpurun_out/stem_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/stem_c3_on.log 2>&1 || exit 1
DV_STEM_DIRECT=0 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/stem_c3_off.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/profile_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/stem_layers_c3.txt 2>&1
