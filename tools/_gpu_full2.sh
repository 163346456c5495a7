# checkpoint: full GPU suite, smoke, flagship bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/full_tests.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/full_smoke.log 2>&1 || exit 1
timeout -k 10 120 python -u bench.py > gpurun_out/full_bench.log 2>&1
