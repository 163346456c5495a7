# per-layer tables: config 2 (deconvnet) and config 3 (DeepDream), bench.py x3 for noise
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/profile_layers.py > gpurun_out/layers_c2_r2.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/profile_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/dream_layers_c3_r2hs.txt 2>&1 || exit 1
for i in 1 2 3; do timeout -k 10 120 python -u bench.py > gpurun_out/c2_rep$i.log 2>&1 || exit 1; done
