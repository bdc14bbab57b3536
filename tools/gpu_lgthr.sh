#!/bin/bash
# lk_kernel_lg ordered chains from the first failing thread (vs half wave):
# bit-exact large-window tests, then isolated launches / PETS / 4K of this build
# against var_libs/prev.
set -e -o pipefail
R=$(pwd)
O=gpurun_out/${OUT:-lgthr}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_headline_gpu.py tests/test_lk_gpu.py tests/test_tracker2d_group.py -m gpu -k "mixed or realistic or large or 4k or errors" > $O/t.log 2>&1
echo tests ok
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated"
for V in base prev base prev; do
  D=/tmp/v_$V; rm -rf $D; mkdir -p $D
  tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
  [ $V != base ] && cp var_libs/$V/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
  (cd $D && timeout -k 10 200 python tools/bx_time.py --points 512 --reps 8 --shapes 100x250,130x130,150x375,140x357 >> $R/$O/t_$V.json)
  (cd $D && timeout -k 10 200 python bench.py --steps 40 --box-dist pets $Q >> $R/$O/pets_$V.json 2>/dev/null)
  (cd $D && timeout -k 10 300 python bench.py --width 3840 --height 2160 --cameras 8 --points 4096 --boxes 64 --steps 6 --warmup 2 --measure-steps 2 $Q >> $R/$O/uhd_$V.json 2>/dev/null)
  echo "variant $V done"
done
