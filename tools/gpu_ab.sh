#!/bin/bash
# Same-box A/B of two builds (ab/A, ab/B: libpsn_lk.so + libpsn_tracker2d.so):
# bench.py lines alternated A, B, A, B, ... (VARIANTS="A B C": more builds)
# Usage: tools/gpu_ab.sh TAG ROUNDS BENCH-ARGS...
set -o pipefail
R=$1; N=$2; shift 2
O=gpurun_out/$R
mkdir -p $O
for i in $(seq 1 $N); do
  for v in ${VARIANTS:-A B}; do
    timeout -k 10 240 python bench.py --lib-dir ab/$v "$@" > $O/$v$i.json 2> $O/$v$i.err || exit 1
    python -c "import json,sys; d=json.load(open('$O/$v$i.json')); print('$v$i', d['value'], d['ms_per_step'])"
  done
done
