set -e
timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_c2.log 2>&1
timeout -k 10 300 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/dream_c3.log 2>&1
timeout -k 10 300 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8 > gpurun_out/dream_c5.log 2>&1
