#!/bin/bash
# round 6: the whole GPU suite + smoke + two config-2 bench runs
set -o pipefail
O=gpurun_out/${OUT:-suite}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 1
echo suite ok
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
for i in 1 2; do
  timeout -k 10 200 python bench.py > $O/bench_$i.log 2>&1 || exit 3
done
echo done
