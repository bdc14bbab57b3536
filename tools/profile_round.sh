#!/bin/bash
# Round profile of the benched binary on the GPU box -> gpurun_out/prof_<tag>/:
# kernel trace + stats of the default bench line (configs[2] per GPU) and of
# the kernel mode (configs[1]); separate --pmc passes (FETCH_SIZE, WRITE_SIZE,
# SQ counters) of the default line and of the HBM-counter calibration probe;
# then tools/profile_summary.py -> profile.json (copy it to
# profiles/<tag>_tracker_profile.json; bench.py --profile reads it).
# Usage: tools/profile_round.sh r03a
set -e -o pipefail
R=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$R
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$ROOT/bench.py"
Q="--no-cpu-baseline --no-secondary --no-legs --no-isolated"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$B" --steps 100 --warmup 5 $Q > "$OUT/trace_bench.json" 2> "$OUT/trace.log"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace" -o run --output-format csv -- python3 "$B" --mode kernel --steps 200 --warmup 10 $Q > "$OUT/ktrace_bench.json" 2> "$OUT/ktrace.log"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "$B" --steps 30 --warmup 3 $Q > "$OUT/fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 "$B" --steps 30 --warmup 3 $Q > "$OUT/write.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY -d "$OUT/sq" -o run --output-format csv -- python3 "$B" --steps 30 --warmup 3 $Q > "$OUT/sq.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY -d "$OUT/sq2" -o run --output-format csv -- python3 "$B" --steps 30 --warmup 3 $Q > "$OUT/sq2.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$OUT/cfetch" -o run --output-format csv -- "$ROOT/tools/probes/probe_hbm_calib" > "$OUT/cfetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d "$OUT/cwrite" -o run --output-format csv -- "$ROOT/tools/probes/probe_hbm_calib" > "$OUT/cwrite.log" 2>&1
# isolated launches of the frame-set's windows (roofline.isolated) and the PETS-like
# mixed-box leg (legs.mixed_boxes.roofline): kernel traces, PMC bytes, SQ_WAIT_ANY
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/iso" -o run --output-format csv -- python3 "$B" --mode isolated > "$OUT/iso_time.json" 2> "$OUT/iso.log"
P="--box-dist pets --no-cpu-baseline --no-secondary --no-legs --no-isolated"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/pets" -o run --output-format csv -- python3 "$B" --steps 40 --warmup 5 $P > "$OUT/pets_bench.json" 2> "$OUT/pets.log"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pets_fetch" -o run --output-format csv -- python3 "$B" --steps 20 --warmup 3 $P > "$OUT/pets_fetch.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pets_write" -o run --output-format csv -- python3 "$B" --steps 20 --warmup 3 $P > "$OUT/pets_write.log" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY -d "$OUT/pets_sq2" -o run --output-format csv -- python3 "$B" --steps 20 --warmup 3 $P > "$OUT/pets_sq2.log" 2>&1
# the 4K Tracker2D Run (configs[4] shape: 8 x 4K cameras, 4096 points, 128 x 320 boxes): kernel trace and HBM bytes
K="--width 3840 --height 2160 --cameras 8 --points 4096 --boxes 64 --no-cpu-baseline --no-secondary --no-legs --no-isolated --steps 6 --warmup 2 --measure-steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/k4" -o run --output-format csv -- python3 "$B" $K > "$OUT/k4_bench.json" 2> "$OUT/k4.log"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/k4_fetch" -o run --output-format csv -- python3 "$B" $K > "$OUT/k4_fetch.log" 2>&1
python3 "$ROOT/tools/profile_summary.py" "$OUT" "$ROOT/mcmtt_opticalflow_amd/lib/libpsn_lk.so" "$OUT/profile.json" > "$OUT/profile_summary.log"
find "$OUT/trace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_stats.csv" \;
find "$OUT/ktrace" -name '*kernel_stats.csv' -exec cp {} "$OUT/kernel_mode_kernel_stats.csv" \;
find "$OUT/iso" -name '*kernel_stats.csv' -exec cp {} "$OUT/isolated_kernel_stats.csv" \;
find "$OUT/pets" -name '*kernel_stats.csv' -exec cp {} "$OUT/pets_kernel_stats.csv" \;
find "$OUT/k4" -name '*kernel_stats.csv' -exec cp {} "$OUT/k4_kernel_stats.csv" \;
echo "profile $R done"
