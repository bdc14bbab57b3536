#!/bin/bash
# bench.py harness A/B: this tree's bench.py vs bench_prev.py (copy an earlier bench.py there first), same library.
set -e -o pipefail
O=gpurun_out/bab
mkdir -p $O
test -f bench_prev.py
for r in 1 2 3; do
  for V in bench bench_prev; do
    timeout -k 10 200 python $V.py --mode kernel --steps 300 --no-cpu-baseline --no-secondary --no-legs > $O/${V}_$r.json 2>$O/${V}_$r.err
    echo "$V run $r: $(python -c "import json;d=json.loads(open('$O/${V}_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_us'))")"
  done
done
timeout -k 10 300 python bench.py --mode config4 --steps 20 --no-cpu-baseline --no-secondary --no-legs > $O/c4_new.json 2>$O/c4_new.err
timeout -k 10 300 python bench_prev.py --mode config4 --steps 20 --no-cpu-baseline --no-secondary --no-legs > $O/c4_prev.json 2>$O/c4_prev.err
python -c "import json;[print(f, json.loads(open('$O/'+f).read().strip().splitlines()[-1])['value']) for f in ('c4_new.json','c4_prev.json')]"
