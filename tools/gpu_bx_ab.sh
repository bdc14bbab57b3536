#!/bin/bash
# box-kernel A/B: parity (random sweep + box / poison tests), isolated box launches
# (tools/bx_time.py) and the headline frame-set of this tree vs var_libs/$1, alternating
set -e -o pipefail
B=${1:-head}
R=$(pwd)
O=gpurun_out/bxab
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_headline_gpu.py \
  tests/test_lk_sweep_gpu.py > $O/test_sweep.log 2>&1
tail -n 1 $O/test_sweep.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_lk_gpu.py -m gpu \
  -k "box or unwritten or configs2 or 1080p or batched or variants" > $O/test.log 2>&1
tail -n 1 $O/test.log
D=/tmp/v_$B; rm -rf $D; mkdir -p $D
tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
cp var_libs/$B/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
for r in 1 2 3; do
  for V in new $B; do
    if [ $V = new ]; then W=$R; else W=$D; fi
    (cd $W && timeout -k 10 200 python tools/bx_time.py --points 2048 --reps 20 --shapes 64x64,64x160 > $R/$O/t_${V}_$r.json 2>$R/$O/t_${V}_$r.err)
    (cd $W && timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-secondary --no-legs --no-isolated > $R/$O/h_${V}_$r.json 2>$R/$O/h_${V}_$r.err)
    echo "$V run $r: headline $(python -c "import json;d=json.loads(open('$O/h_${V}_$r.json').read().strip().splitlines()[-1]);print(d['value'])") bx $(python -c "import json;d=json.load(open('$O/t_${V}_$r.json'));print({k:v['median_us'] for k,v in d.items() if isinstance(v,dict) and 'median_us' in v})")"
  done
done
