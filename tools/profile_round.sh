#!/bin/bash
# Round profile on the GPU box: kernel trace + stats of the default bench, and
# separate --pmc passes (FETCH_SIZE, WRITE_SIZE) of the bench and of the
# HBM-counter calibration probe. Usage: tools/profile_round.sh r01
set -e -o pipefail
R=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$B" --steps 200 --warmup 10 --no-cpu-baseline > "$OUT/trace_bench.json" 2> "$OUT/trace.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "$B" --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 "$B" --steps 50 --warmup 5 --no-cpu-baseline > "$OUT/write.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/cfetch" -o run --output-format csv -- "$ROOT/tools/probes/probe_hbm_calib" > "$OUT/cfetch.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/cwrite" -o run --output-format csv -- "$ROOT/tools/probes/probe_hbm_calib" > "$OUT/cwrite.log" 2>&1
python3 "$ROOT/tools/pmc_summary.py" "$OUT/fetch" "$OUT/write" "$OUT/cfetch" "$OUT/cwrite" "$OUT/pmc_summary.json" > /dev/null
echo "profile $R done"
