#!/bin/bash
# Workgroup-size comparison: bench + stamps breakdown per PSN_LK_THREADS value.
set -e -o pipefail
mkdir -p gpurun_out/exp
for nt in 256 512; do
  PSN_LK_THREADS=$nt timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/exp/nt_$nt.json
  PSN_LK_THREADS=$nt PSN_LK_LIB=mcmtt_opticalflow_amd/lib/libpsn_lk_stamps.so timeout -k 10 120 python tools/lk_stamps.py > gpurun_out/exp/stamps_$nt.json
done
