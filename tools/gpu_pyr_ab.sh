#!/bin/bash
# A/B of build variants (var_libs/<name>/ holds libpsn_lk.so + libpsn_tracker2d.so):
# parity tests touching the variant, uniform and PETS-box bench lines, kernel
# stats and FETCH_SIZE of the uniform line. Results under gpurun_out/pyr_ab/.
set -e -o pipefail
R=$(pwd)
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated"
mkdir -p gpurun_out/pyr_ab
if [ -f mcmtt_opticalflow_amd/lib/libpsn_lk_ab.so ]; then
  timeout -k 10 200 python tools/bx_time.py --reps 20 > gpurun_out/pyr_ab/bxt_head.json
  timeout -k 10 200 python tools/bx_time.py --reps 20 --lib mcmtt_opticalflow_amd/lib/libpsn_lk_ab.so > gpurun_out/pyr_ab/bxt_r03.json
fi
timeout -k 10 120 python tools/lk_stamps.py > gpurun_out/pyr_ab/st_stamps.json
for V in base ${VARIANTS:-t12 t16 jr100}; do
  D=/tmp/v_$V; rm -rf $D; mkdir -p $D
  tar --exclude=./gpurun_out --exclude=./build -cf - . | tar -xf - -C $D
  if [ $V != base ]; then cp var_libs/$V/*.so $D/mcmtt_opticalflow_amd/lib/; fi
  cd $D
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu -k "pyramid or bgr or large" > $R/gpurun_out/pyr_ab/test_$V.log 2>&1
  timeout -k 10 200 python bench.py --steps 100 $Q > $R/gpurun_out/pyr_ab/bench_$V.json 2>/dev/null
  timeout -k 10 200 python bench.py --steps 40 --box-dist pets $Q > $R/gpurun_out/pyr_ab/pets_$V.json 2>/dev/null
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pyr_ab/tr_$V -o run --output-format csv -- python3 $D/bench.py --steps 50 $Q > /dev/null 2>&1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $R/gpurun_out/pyr_ab/f_$V -o run --output-format csv -- python3 $D/bench.py --steps 20 $Q > /dev/null 2>&1
  cd $R
  echo "variant $V done"
done
echo done
