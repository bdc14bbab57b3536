#!/bin/bash
# One kernel-iteration check on the GPU box: the LK / Tracker2D GPU parity tests,
# the box-window kernel's phase stamps (64x64 and 64x160 windows, 2048 points)
# and a short default bench line. Usage: tools/iter_check.sh <out-subdir>
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/${1:-iter}
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 300 python -u -m pytest tests/test_lk_gpu.py tests/test_tracker2d.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
STAMPS=$ROOT/mcmtt_opticalflow_amd/lib/libpsn_lk_stamps.so
WIN=64 WINH=64 NPTS=2048 timeout -k 10 120 python tools/bx_stamps.py > "$OUT/st64.json" 2>&1
WIN=64 WINH=160 NPTS=2048 timeout -k 10 120 python tools/bx_stamps.py > "$OUT/st160.json" 2>&1
timeout -k 10 300 python bench.py --steps 60 --warmup 5 --no-cpu-baseline --no-secondary > "$OUT/bench.json" 2> "$OUT/bench.err"
echo "iter_check done"
