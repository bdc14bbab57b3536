#!/bin/bash
# Large-window kernel occupancy A/B (var_libs/<name>/libpsn_lk.so builds): the
# PETS-box bench line and the 4K Tracker2D line per build, isolated launches.
set -e -o pipefail
R=$(pwd)
O=gpurun_out/lg_occ
mkdir -p $O
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated"
for V in base ${VARIANTS:-nojr nojr4 w3}; do
  D=/tmp/v_$V; rm -rf $D; mkdir -p $D
  tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
  [ $V != base ] && cp var_libs/$V/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
  (cd $D && timeout -k 10 200 python bench.py --steps 40 --box-dist pets $Q > $R/$O/pets_$V.json 2>/dev/null)
  (cd $D && timeout -k 10 300 python bench.py --width 3840 --height 2160 --cameras 8 --points 4096 --boxes 64 --steps 6 --warmup 2 --measure-steps 2 $Q > $R/$O/uhd_$V.json 2>/dev/null)
  (cd $D && timeout -k 10 200 python tools/bx_time.py --points 512 --reps 8 --shapes 100x250,150x375 > $R/$O/t_$V.json)
  echo "variant $V done"
done
