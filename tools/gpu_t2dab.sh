#!/bin/bash
# A/B of libpsn_tracker2d.so builds on the default bench line (no CPU legs):
# base, variant, base, variant -> gpurun_out/$1 (the variant replaces the
# product file on the box for its runs only)
set -o pipefail
R=${1:-t2dab}
V=$2
O=gpurun_out/$R
mkdir -p $O
L=mcmtt_opticalflow_amd/lib
cp $L/libpsn_tracker2d.so $O/base.so
for rep in 1 2; do
  for which in base var; do
    if [ $which = var ]; then cp $V $L/libpsn_tracker2d.so; else cp $O/base.so $L/libpsn_tracker2d.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-legs --steps 100 > $O/$which.json 2> $O/$which.err || exit 1
    echo "$which $(python -c "import json;d=json.loads(open('$O/$which.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['roofline']['per_kernel_us'].items()})")"
  done
done
cp $O/base.so $L/libpsn_tracker2d.so
