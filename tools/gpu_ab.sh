#!/bin/bash
# A/B of box-kernel builds: the LK GPU tests on the product library, then
# isolated launch times (tools/bx_time.py) of each library given -> gpurun_out/$1
set -o pipefail
R=${1:-ab}
shift
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lk_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_lk.log 2>&1 || { tail -5 $O/pytest_lk.log; exit 1; }
tail -1 $O/pytest_lk.log
for lib in "$@"; do
  timeout -k 10 120 python tools/bx_time.py --reps 40 --lib $lib > $O/time_$(basename $lib .so).json 2>&1 || exit 1
  cat $O/time_$(basename $lib .so).json
done
