#!/bin/bash
# A/B of two builds of the product libraries on the default bench line (no CPU
# legs): directories A and B each hold libpsn_lk.so + libpsn_tracker2d.so;
# they are copied over mcmtt_opticalflow_amd/lib on the box in turn (A, B, A, B)
# -> gpurun_out/$1, $4 rounds (default 2). The product files are restored from A at the end.
set -o pipefail
R=${1:-libab}
DA=$2
DB=$3
O=gpurun_out/$R
mkdir -p $O
L=mcmtt_opticalflow_amd/lib
for rep in $(seq ${4:-2}); do
  for which in A B; do
    D=$DA; [ $which = B ] && D=$DB
    cp $D/libpsn_lk.so $D/libpsn_tracker2d.so $L/
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-legs --steps 100 > $O/$which.json 2> $O/$which.err || exit 1
    echo "$which $(python -c "import json;d=json.loads(open('$O/$which.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],{k:v['avg_us'] for k,v in d['roofline']['per_kernel_us'].items()})")"
  done
done
cp $DA/libpsn_lk.so $DA/libpsn_tracker2d.so $L/
