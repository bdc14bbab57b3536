#!/bin/bash
# the merged host-chain Tracker2D sequence test with this tree's library (twice) and var_libs/noovl
set -o pipefail
R=$(pwd)
O=gpurun_out/t2dovl
mkdir -p $O
D=/tmp/v_noovl; rm -rf $D; mkdir -p $D
tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
cp var_libs/noovl/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
K="test_tracker2d_sequence_matches_oracle"
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_tracker2d.py -m gpu -k "$K" > $O/new1.log 2>&1; echo "new1 rc=$?"
(cd $D && timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_tracker2d.py -m gpu -k "$K" > $R/$O/noovl.log 2>&1); echo "noovl rc=$?"
timeout -k 10 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_tracker2d.py -m gpu -k "$K" > $O/new2.log 2>&1; echo "new2 rc=$?"
tail -3 $O/new1.log $O/noovl.log $O/new2.log
