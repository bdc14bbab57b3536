#!/bin/bash
# lk_kernel_st overlapped A phase: parity (single-tile tests), then configs[1]
# kernel-mode lines with the overlap on / off (PSN_LK_VARIANT_ST_OVL), alternating.
set -e -o pipefail
O=gpurun_out/st_ovl
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu \
  -k "variants or overlapped or config or fused or counted" > $O/test.log 2>&1
for r in 1 2 3; do
  for V in 1 0; do
    timeout -k 10 200 python bench.py --mode kernel --steps 300 --no-cpu-baseline --no-secondary --no-legs \
      --lk-variant st_ovl=$V > $O/k_${V}_$r.json 2>$O/k_${V}_$r.err
    echo "ovl=$V run $r: $(python -c "import json;d=json.loads(open('$O/k_${V}_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline'].get('avg_launch_us'))")"
  done
done
