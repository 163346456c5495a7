set -o pipefail
mkdir -p gpurun_out
for d in 1 0 1 0; do
  DV_BENCH_DEFER_COPY=$d timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > gpurun_out/df_bench_$d.log 2>&1 || exit 1
  echo "defer=$d $(tail -1 gpurun_out/df_bench_$d.log)" >> gpurun_out/df_ab.txt
done
