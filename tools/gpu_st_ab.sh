#!/bin/bash
# lk_kernel_st A/B: parity tests of the small-window kernel, then kernel-mode
# (configs[1]) and configs[4] lines for this tree and var_libs/st0.
set -e -o pipefail
R=$(pwd)
O=gpurun_out/st_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu -k "not large and not box" > $O/test.log 2>&1
for V in new st0 new st0; do
  D=/tmp/v_$V; rm -rf $D; mkdir -p $D
  tar --exclude=./gpurun_out --exclude=./build -cf - . | tar -xf - -C $D
  [ $V != new ] && cp var_libs/$V/*.so $D/mcmtt_opticalflow_amd/lib/
  (cd $D && timeout -k 10 200 python bench.py --mode kernel --steps 300 --no-cpu-baseline --no-secondary --no-legs > $R/$O/k_$V.json 2>/dev/null && timeout -k 10 200 python bench.py --mode config4 --steps 20 --no-cpu-baseline --no-secondary --no-legs > $R/$O/c4_$V.json 2>/dev/null)
  echo "variant $V"
done
