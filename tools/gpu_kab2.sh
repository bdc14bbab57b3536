#!/bin/bash
# single-tile kernel A/B (this tree vs var_libs/$1): parity + poison tests, stamps of both
# (class / chain path fractions), configs[1] kernel-mode lines alternating three times
set -e -o pipefail
B=${1:-head}
R=$(pwd)
O=gpurun_out/kab2
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu \
  -k "variants or overlapped or config or fused or counted or unwritten" > $O/test.log 2>&1
timeout -k 10 120 python tools/lk_stamps.py > $O/stamps_new.json 2>&1
D=/tmp/v_$B; rm -rf $D; mkdir -p $D
tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
cp var_libs/$B/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
for r in 1 2 3; do
  for V in new $B; do
    if [ $V = new ]; then W=$R; else W=$D; fi
    (cd $W && timeout -k 10 200 python bench.py --mode kernel --steps 300 --no-cpu-baseline --no-secondary \
      --no-legs > $R/$O/k_${V}_$r.json 2>$R/$O/k_${V}_$r.err)
    echo "$V run $r: $(python -c "import json;d=json.loads(open('$O/k_${V}_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['roofline'].get('avg_launch_us'))")"
  done
done
tail -1 $O/test.log
python -c "import json;d=json.load(open('$O/stamps_new.json'));print(d['iteration_phases_cycles_per_iter'], d['wg_cycles_max'])"
