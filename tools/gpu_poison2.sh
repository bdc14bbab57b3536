#!/bin/bash
# LDS-poison tests of every LK kernel, then the whole -m gpu suite
set -o pipefail
O=gpurun_out/poison2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_lk_gpu.py -m gpu -k "unwritten_lds" > $O/poison.log 2>&1; echo "poison rc=$?"
grep -E "^FAILED|passed|failed" $O/poison.log | head -12
