#!/bin/bash
# Workgroup-size sweep of the single-tile LK kernel on the bench workload.
set -e
mkdir -p gpurun_out/exp
for nt in 256 128 64; do
  PSN_LK_THREADS=$nt timeout -k 10 240 python bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/exp/threads_$nt.json
done
