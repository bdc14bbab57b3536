#!/bin/bash
# Kernel trace of the bench (default fused ingest) for launch-gap analysis.
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/trace_${1:-fused}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --overlap ${1:-fused} > "$OUT/bench.json" 2> "$OUT/trace.log"
