#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out/exp
timeout -k 10 120 python bench.py --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/exp/v5_bench.json
PSN_LK_LIB=mcmtt_opticalflow_amd/lib/libpsn_lk_stamps.so timeout -k 10 120 python tools/lk_stamps.py > gpurun_out/exp/v5_stamps.json
