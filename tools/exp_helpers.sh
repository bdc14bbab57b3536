#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --overlap off > gpurun_out/exp/helpers_off.json
for hlp in 0 128 512; do
  PSN_LK_FUSED_HELPERS=$hlp timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/exp/helpers_$hlp.json
done
