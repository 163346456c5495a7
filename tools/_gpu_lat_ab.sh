set -o pipefail
mkdir -p gpurun_out
for cfg in "2 64" "2 16" "2 4" "0.5 8" "1 8"; do
  set -- $cfg
  timeout -k 10 200 python tools/latency.py --sizes 1 --reps 3 --clients 16,128 --requests 2048 --timeout-ms $1 --chunk $2 > gpurun_out/lat_t$1_c$2.json 2>/dev/null || exit 1
done
