#!/bin/bash
# GPU-box check of a tree: the -m gpu suite, then the default bench line.
# Usage: tools/gpu_check.sh <out-subdir> [extra bench args]
set -o pipefail
R=${1:-check}
shift
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 420 python bench.py "$@" > $O/bench.json 2> $O/bench.err
rc=$?
tail -3 $O/pytest.log
echo rc=$rc
