#!/bin/bash
# configs[1] kernel-mode A/B of this tree's libpsn_lk.so against var_libs/$1 (tree copies
# in /tmp), alternating three times; parity tests of the single-tile kernel first.
set -e -o pipefail
B=${1:-ovl}
R=$(pwd)
O=gpurun_out/kab
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu \
  -k "variants or overlapped or config or fused or counted" > $O/test.log 2>&1
for V in new $B; do
  D=/tmp/v_$V; rm -rf $D; mkdir -p $D
  tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
  [ $V != new ] && cp var_libs/$V/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
done
for r in 1 2 3; do
  for V in new $B; do
    (cd /tmp/v_$V && timeout -k 10 200 python bench.py --mode kernel --steps 300 --no-cpu-baseline --no-secondary \
      --no-legs > $R/$O/k_${V}_$r.json 2>$R/$O/k_${V}_$r.err)
    echo "$V run $r: $(python -c "import json;d=json.loads(open('$O/k_${V}_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline'].get('avg_launch_us'))")"
  done
done
