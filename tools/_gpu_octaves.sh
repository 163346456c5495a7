# per-octave graphed DeepDream time, split 1 and 2 (config 3) and config-5-like resnet untiled 512
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/dream_octave_times.py --split 2 > gpurun_out/oct_s2.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/dream_octave_times.py --split 1 > gpurun_out/oct_s1.log 2>&1 || exit 1
