#!/bin/bash
# isolated launch times (tools/bx_time.py) of each library given, twice, interleaved -> gpurun_out/$1
set -o pipefail
R=${1:-ab}
shift
O=gpurun_out/$R
mkdir -p $O
for rep in 1 2; do
for lib in "$@"; do
  timeout -k 10 120 python tools/bx_time.py --reps 40 --lib $lib > $O/t.json 2>&1 || { cat $O/t.json; exit 1; }
  echo "$(basename $lib) $(cat $O/t.json)"
done
done
