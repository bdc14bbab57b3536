#!/bin/bash
# Post-sync upload stall: host-buffer kind A/B with a device sync every 10 timed
# steps (bench --diag-sync-every 10); slow steps and per-call host ms of each.
set -e -o pipefail
O=gpurun_out/stall
mkdir -p $O
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated --step-profile --steps 60 --warmup 10 --diag-sync-every 10"
for A in ${ALLOCS:-torch hip register torch}; do
  timeout -k 10 150 python bench.py $Q --host-alloc $A > $O/b_$A.json 2> $O/b_$A.err
  echo "alloc $A done"
done
