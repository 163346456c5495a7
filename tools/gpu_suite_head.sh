#!/bin/bash
# the driver's round-end GPU tiers at HEAD: pytest -m gpu, smoke(), one bench.py run
set -o pipefail
O=gpurun_out/suite_head
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 200 python bench.py > $O/bench.log 2>&1 || exit 3
