#!/bin/bash
# Post-sync upload stall vs hardware queues per process (GPU_MAX_HW_QUEUES), a
# device sync every 10 timed steps; plus a HIP API trace of the default count.
set -e -o pipefail
O=gpurun_out/stallq
mkdir -p $O
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated --step-profile --steps 60 --warmup 10 --diag-sync-every 10"
for N in 4 8 16 4; do
  GPU_MAX_HW_QUEUES=$N timeout -k 10 150 python bench.py $Q > $O/q$N.json 2> $O/q$N.err
  echo "queues $N done"
done
