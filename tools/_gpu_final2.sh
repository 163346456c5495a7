# end-of-session checkpoint: full GPU suite, smoke, flagship bench x2, DeepDream config 3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/fin2_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin2_smoke.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/fin2_bench.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py > gpurun_out/fin2_bench_default.log 2>&1 || exit 1
timeout -k 10 200 python -u bench_dream.py --model inception_v3 --batch 64 --size 299 > gpurun_out/fin2_c3.log 2>&1 || exit 1
