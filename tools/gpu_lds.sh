#!/bin/bash
# LDS counters of the default bench's kernels (one --pmc pass) -> gpurun_out/$1
set -o pipefail
R=${1:-lds}
O=$GRAFT_REPO_ROOT/gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_THREAD_CYCLES_VALU -d $O/lds -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-legs > $O/lds.log 2>&1
echo rc=$?
