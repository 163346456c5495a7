# D2H copy-back on a CU-masked stream: bench A/B over the CU count + kernel trace of the default
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in 8 0 16 4 8 0; do
  DV_COPY_CUS=$c timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > gpurun_out/cc_bench_$c.log 2>&1 || exit 1
  echo "cus=$c $(tail -1 gpurun_out/cc_bench_$c.log)" >> gpurun_out/cc_ab.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/cc_prof -o cc -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/cc_prof.log 2>&1 || exit 1
