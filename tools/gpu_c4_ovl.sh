#!/bin/bash
# configs[4] leg with the single-tile overlapped A phase on / off (PSN_LK_VARIANT_ST_OVL), alternating.
set -e -o pipefail
O=gpurun_out/c4ovl
mkdir -p $O
for r in 1 2; do
  for V in 1 0; do
    timeout -k 10 300 python bench.py --mode config4 --steps 20 --no-cpu-baseline --no-secondary --no-legs \
      --lk-variant st_ovl=$V > $O/c4_${V}_$r.json 2>$O/c4_${V}_$r.err
    echo "ovl=$V run $r: $(python -c "import json;d=json.loads(open('$O/c4_${V}_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline'].get('avg_launch_us'))")"
  done
done
