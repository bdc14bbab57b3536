#!/bin/bash
# SQ counters of the default bench's kernels (one --pmc pass) -> gpurun_out/$1/sq
set -o pipefail
R=${1:-sq}
O=$GRAFT_REPO_ROOT/gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY -d $O/sq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $O/sq.log 2>&1
echo rc=$?
