#!/bin/bash
# One GPU-box validation pass (results under gpurun_out/$1): the new runtime /
# exchange tests, the -m gpu suite, smoke, the default bench line.
set -o pipefail
R=${1:-g}
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_runtime_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_runtime.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
echo rc=$?
