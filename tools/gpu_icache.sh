#!/bin/bash
# Instruction-fetch counters of the default bench's kernels -> gpurun_out/$1:
# the box's counter list, then one --pmc pass (SQ wave-state buckets + SQC
# instruction-cache hits / misses).
set -o pipefail
R=${1:-icache}
O=$GRAFT_REPO_ROOT/gpurun_out/$R
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_WAIT[A-Z_]*\|SQ_INST_CYCLES[A-Z_]*\|SQ_ACTIVE[A-Z_]*" $O/avail.txt | sort -u > $O/names.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU SQC_ICACHE_HITS SQC_ICACHE_MISSES -d $O/ic -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-legs > $O/ic.log 2>&1
echo rc=$?
