#!/bin/bash
# Large-window kernel build variants (var_libs/<name>/): isolated launches of
# PETS-scale windows at 128 and 512 points, then the PETS-box bench line.
set -e -o pipefail
R=$(pwd)
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated"
O=gpurun_out/lg_ab
mkdir -p $O
for V in base ${VARIANTS:-jr100 tq192 tq64}; do
  L=mcmtt_opticalflow_amd/lib/libpsn_lk.so
  [ $V != base ] && L=var_libs/$V/libpsn_lk.so
  for P in 128 512; do
    timeout -k 10 200 python tools/bx_time.py --points $P --reps 8 --shapes 100x250,130x130,150x375,140x357 --lib $L > $O/t_${V}_$P.json
  done
  echo "variant $V timed"
done
for V in base ${VARIANTS:-jr100 tq192 tq64}; do
  D=/tmp/v_$V; rm -rf $D; mkdir -p $D
  tar --exclude=./gpurun_out --exclude=./build -cf - . | tar -xf - -C $D
  [ $V != base ] && cp var_libs/$V/*.so $D/mcmtt_opticalflow_amd/lib/
  (cd $D && timeout -k 10 200 python bench.py --steps 40 --box-dist pets $Q > $R/$O/pets_$V.json 2>/dev/null)
  echo "variant $V benched"
done
echo done
