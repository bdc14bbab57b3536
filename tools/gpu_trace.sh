#!/bin/bash
# Kernel trace (+ stats) of the default bench on the GPU box -> gpurun_out/$1/trace
set -o pipefail
R=${1:-t}
O=$GRAFT_REPO_ROOT/gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 40 --warmup 3 --no-cpu-baseline --no-secondary > $O/trace_bench.json 2> $O/trace.log
echo rc=$?
