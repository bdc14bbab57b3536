#!/bin/bash
# kernel trace of the default bench line -> gpurun_out/$1/trace
set -o pipefail
R=${1:-tr}
O=$GRAFT_REPO_ROOT/gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-secondary --no-legs > $O/bench.json 2> $O/trace.log
echo rc=$?
