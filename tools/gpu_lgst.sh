#!/bin/bash
# Phase clocks of lk_kernel_lg (stamps build) on PETS-scale and 4K windows, and
# isolated launch times of the product build on the same shapes.
set -e -o pipefail
O=gpurun_out/${OUT:-lgst}
mkdir -p $O
for S in ${SHAPES:-100x250 150x375}; do
  W=${S%x*}; H=${S#*x}
  WIN=$W WINH=$H NPTS=512 timeout -k 10 120 python tools/lg_stamps.py > $O/st_$S.json
done
UHD=1 WIN=128 WINH=320 NPTS=512 timeout -k 10 120 python tools/lg_stamps.py > $O/st_uhd_128x320.json
timeout -k 10 200 python tools/bx_time.py --points 512 --reps 8 --shapes 100x250,130x130,150x375,140x357 > $O/time_512.json
echo done
