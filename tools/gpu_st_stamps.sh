#!/bin/bash
# lk_kernel_st stamps (configs[1]: 512 points, 21x21, 4 levels) with the overlapped A phase on / off.
set -e -o pipefail
O=gpurun_out/st_stamps
mkdir -p $O
for V in 1 0; do
  ST_OVL=$V timeout -k 10 120 python tools/lk_stamps.py > $O/st_ovl$V.json 2> $O/st_ovl$V.err
done
