# fused deconvnet tail: kernel test, engine parity tests, bench A/B, kernel stats
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "deconv_tail or stream_stats" -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_t.log 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tail_engine.log 2>&1 || exit 1
for e in 1 0 1 0; do
  DV_FUSED_TAIL=$e timeout -k 10 150 python -u bench.py --steps 20 --warmup 5 > gpurun_out/tail_bench_$e.log 2>&1 || exit 1
  tail -1 gpurun_out/tail_bench_$e.log >> gpurun_out/tail_ab.txt
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tail_prof -o tail -- python -u bench.py --steps 5 --warmup 2 > gpurun_out/tail_prof.log 2>&1 || exit 1
