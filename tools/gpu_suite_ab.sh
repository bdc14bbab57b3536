#!/bin/bash
# the whole -m gpu suite: this tree's library, var_libs/$1, this tree again (failures listed)
set -o pipefail
B=${1:-noovl}
R=$(pwd)
O=gpurun_out/suiteab
mkdir -p $O
D=/tmp/v_$B; rm -rf $D; mkdir -p $D
tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
cp var_libs/$B/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/new1.log 2>&1; echo "new1 rc=$?"
(cd $D && timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $R/$O/$B.log 2>&1); echo "$B rc=$?"
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/new2.log 2>&1; echo "new2 rc=$?"
for f in new1 $B new2; do echo "== $f"; grep -E "^FAILED|passed|failed" $O/$f.log; done
