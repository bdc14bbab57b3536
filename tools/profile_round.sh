#!/bin/bash
# Round profile on the GPU box: kernel trace + stats of the default bench
# (Tracker2D mode, configs[2]) and of the kernel mode (configs[1]), and separate
# --pmc passes (FETCH_SIZE, WRITE_SIZE) of both and of the HBM-counter
# calibration probe. Usage: tools/profile_round.sh r02
set -e -o pipefail
R=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py"
Q="--no-cpu-baseline --no-secondary"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$B" --steps 100 --warmup 5 $Q > "$OUT/trace_bench.json" 2> "$OUT/trace.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace" -o run --output-format csv -- python3 "$B" --mode kernel --steps 200 --warmup 10 $Q > "$OUT/ktrace_bench.json" 2> "$OUT/ktrace.log"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "$B" --steps 30 --warmup 3 $Q > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 "$B" --steps 30 --warmup 3 $Q > "$OUT/write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/kfetch" -o run --output-format csv -- python3 "$B" --mode kernel --steps 50 --warmup 5 $Q > "$OUT/kfetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/kwrite" -o run --output-format csv -- python3 "$B" --mode kernel --steps 50 --warmup 5 $Q > "$OUT/kwrite.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/cfetch" -o run --output-format csv -- "$ROOT/tools/probes/probe_hbm_calib" > "$OUT/cfetch.log" 2>&1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/cwrite" -o run --output-format csv -- "$ROOT/tools/probes/probe_hbm_calib" > "$OUT/cwrite.log" 2>&1
python3 "$ROOT/tools/pmc_summary.py" "$OUT/fetch" "$OUT/write" "$OUT/cfetch" "$OUT/cwrite" "$OUT/pmc_summary.json" > /dev/null
python3 "$ROOT/tools/pmc_summary.py" "$OUT/kfetch" "$OUT/kwrite" "$OUT/cfetch" "$OUT/cwrite" "$OUT/kpmc_summary.json" > /dev/null
echo "profile $R done"
