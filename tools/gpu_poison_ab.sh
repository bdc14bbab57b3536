#!/bin/bash
# LDS-poison tests of the single-tile kernel: this tree (fixed) and var_libs/prefix (before
# the class-3 publish fix), then the whole -m gpu suite on this tree.
set -o pipefail
R=$(pwd)
O=gpurun_out/poison
mkdir -p $O
D=/tmp/v_prefix; rm -rf $D; mkdir -p $D
tar --exclude=./gpurun_out --exclude=./build --exclude=./var_libs -cf - . | tar -xf - -C $D
cp var_libs/prefix/libpsn_lk.so $D/mcmtt_opticalflow_amd/lib/
K="unwritten_lds or overlapped or variants"
(cd $D && timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu -k "$K" > $R/$O/prefix.log 2>&1); echo "prefix rc=$?"
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu -k "$K" > $O/fixed.log 2>&1; echo "fixed rc=$?"
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/suite.log 2>&1; echo "suite rc=$?"
for f in prefix fixed suite; do echo "== $f"; grep -E "^FAILED|passed|failed" $O/$f.log | head -12; done
