#!/bin/bash
# kernel trace + stats of the configs[1] kernel-mode line -> gpurun_out/ktrace
set -e -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/ktrace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode kernel --steps 300 --no-cpu-baseline --no-secondary --no-legs > $O/bench.json 2> $O/trace.log
