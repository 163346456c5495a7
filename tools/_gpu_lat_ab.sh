set -o pipefail
mkdir -p gpurun_out
for cfg in "4 4" "8 2" "2 8"; do
  set -- $cfg
  timeout -k 10 200 python tools/latency.py --sizes 1 --reps 3 --clients 128 --requests 3072 --enc-workers $1 --enc-threads $2 > gpurun_out/lat_e$1_$2.json 2>/dev/null || exit 1
done
