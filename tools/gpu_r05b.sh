#!/bin/bash
# r05b: the SDMA warm-up (post-sync stall), driver-like default line and a
# device sync every 10 steps; large-window isolated launches (xb off = r04 code)
set -e -o pipefail
O=gpurun_out/r05b
mkdir -p $O
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated"
timeout -k 10 150 python bench.py $Q --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err
timeout -k 10 150 python bench.py $Q --step-profile --steps 60 --warmup 10 --diag-sync-every 10 > $O/bsync.json 2> $O/bsync.err
timeout -k 10 150 python bench.py $Q --steps 100 > $O/b100.json 2> $O/b100.err
timeout -k 10 200 python tools/bx_time.py --points 512 --reps 8 --shapes 100x250,130x130,150x375,140x357 > $O/t_lg.json
timeout -k 10 200 python tools/bx_time.py --reps 20 > $O/t_bx.json
echo done
