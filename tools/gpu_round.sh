#!/bin/bash
# One GPU-box validation pass (tools for the builder; results under gpurun_out/$1):
# the -m gpu suite, the default bench line, phase stamps of both box-window
# kernels, and a WRITE_SIZE pass of the Tracker2D bench (scratch-spill check).
set -o pipefail
R=${1:-g}
O=gpurun_out/$R
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err && \
WIN=64 WINH=64 NPTS=2048 timeout -k 10 120 python tools/bx_stamps.py > $O/st64.json 2>&1 && \
WIN=64 WINH=160 NPTS=2048 timeout -k 10 120 python tools/bx_stamps.py > $O/st160.json 2>&1 && \
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$O/write -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $GRAFT_REPO_ROOT/$O/write.log 2>&1)
echo rc=$?
