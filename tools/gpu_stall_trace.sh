#!/bin/bash
# HIP + HSA API trace of a short default bench with a device sync every 10 timed
# steps: which HSA calls run inside the post-sync frame-upload stalls.
set -e -o pipefail
ROOT=$(pwd)
O=$ROOT/gpurun_out/stall_hsa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --hip-trace --hsa-trace -d $O -o run --output-format csv -- python3 $ROOT/bench.py --no-cpu-baseline --no-secondary --no-legs --no-isolated --step-profile --steps 30 --warmup 5 --measure-steps 0 --diag-sync-every 10 > $O/bench.json 2> $O/bench.err
echo done
