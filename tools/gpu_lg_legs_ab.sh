#!/bin/bash
# large-window kernel A/B: this tree vs var_libs/$1 on isolated launches and the PETS, realistic and
# 4K tracker legs (alternating twice), after the large-window parity tests
set -e -o pipefail
B=${1:-head}
R=$(pwd)
O=gpurun_out/lglegs
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_headline_gpu.py -m gpu \
  -k "mixed or realistic" > $O/test_h.log 2>&1
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lk_gpu.py -m gpu \
  -k "large or unwritten" > $O/test.log 2>&1
tail -n 1 $O/test_h.log $O/test.log
D=/tmp/v_$B; rm -rf $D; mkdir -p $D
tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
cp var_libs/$B/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated"
for r in 1 2; do
  for V in new $B; do
    if [ $V = new ]; then W=$R; else W=$D; fi
    (cd $W && timeout -k 10 200 python tools/bx_time.py --points 512 --reps 8 --shapes 100x250,130x130,150x375,140x357 > $R/$O/t_${V}_$r.json 2>$R/$O/t_${V}_$r.err)
    echo "$V run $r: lg $(python -c "import json;d=json.load(open('$O/t_${V}_$r.json'));print({k:v['median_us'] for k,v in d.items() if isinstance(v,dict) and 'median_us' in v})")"
    (cd $W && timeout -k 10 300 python bench.py --box-dist pets --steps 40 --warmup 5 $Q > $R/$O/p_${V}_$r.json 2>$R/$O/p_${V}_$r.err)
    (cd $W && timeout -k 10 300 python bench.py --features gridfast --box-dist pets --steps 40 --warmup 5 $Q > $R/$O/r_${V}_$r.json 2>$R/$O/r_${V}_$r.err)
    (cd $W && timeout -k 10 300 python bench.py --width 3840 --height 2160 --cameras 8 --points 4096 --boxes 64 --steps 6 --warmup 2 $Q > $R/$O/k_${V}_$r.json 2>$R/$O/k_${V}_$r.err)
    echo "$V run $r: pets $(python -c "import json;print(json.loads(open('$O/p_${V}_$r.json').read().strip().splitlines()[-1])['value'])") realistic $(python -c "import json;print(json.loads(open('$O/r_${V}_$r.json').read().strip().splitlines()[-1])['value'])") 4k $(python -c "import json;print(json.loads(open('$O/k_${V}_$r.json').read().strip().splitlines()[-1])['value'])")"
  done
done
