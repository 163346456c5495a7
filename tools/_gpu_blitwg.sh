# copy-back blit kernel: limit its workgroups (runtime flag) vs default, bench A/B + trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 4 16 0 4; do
  if [ $v = 0 ]; then unset DEBUG_CLR_LIMIT_BLIT_WG; else export DEBUG_CLR_LIMIT_BLIT_WG=$v; fi
  timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bw_bench_$v.log 2>&1 || exit 1
  echo "wg=$v $(tail -1 gpurun_out/bw_bench_$v.log)" >> gpurun_out/bw_ab.txt
done
export DEBUG_CLR_LIMIT_BLIT_WG=4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/bw_prof -o bw -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/bw_prof.log 2>&1 || exit 1
