# persistent pointwise threshold sweep (config 5, then config 3)
set -o pipefail
mkdir -p gpurun_out
c5() { env "$@" timeout -k 10 200 python -u bench_dream.py --model resnet50 --size 1024 --tile 512 --dtype fp16 --batch 8; }
c5 DV_PW_MIN_TILES=0 > gpurun_out/pwm_c5_def.log 2>&1 || exit 1
c5 DV_PW_MIN_TILES=512 > gpurun_out/pwm_c5_512.log 2>&1 || exit 1
c5 DV_PW_MIN_TILES=256 > gpurun_out/pwm_c5_256.log 2>&1 || exit 1
c5 DV_PW_MIN_TILES=2048 > gpurun_out/pwm_c5_2048.log 2>&1 || exit 1
DV_PW_MIN_TILES=256 timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/pwm_c3_256.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/pwm_c3_def.log 2>&1
