#!/bin/bash
# the driver's default bench line (N = 1) -> gpurun_out/bench_full/$1.json
set -e -o pipefail
O=gpurun_out/bench_full
mkdir -p $O
timeout -k 10 900 python bench.py > $O/${1:-b}.json 2> $O/${1:-b}.err
tail -c 600 $O/${1:-b}.json
