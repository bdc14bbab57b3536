#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out/exp
for m in fused off; do
  timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline --overlap $m > gpurun_out/exp/mode_$m.json
done
