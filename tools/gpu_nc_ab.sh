# coherent vs default pinned staging of the Tracker2D pass copies: headline A/B + copy kernel time
set -e
mkdir -p gpurun_out
ENVAB_CFGS="PSN_T2D_AB_NC=1 X=1 PSN_T2D_AB_NC=1 X=1" bash tools/gpu_envab.sh
cd /tmp && export TMPDIR=/tmp
for cfg in NC CO; do
  if [ $cfg = NC ]; then export PSN_T2D_AB_NC=1; else unset PSN_T2D_AB_NC; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/nc_$cfg -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-secondary --no-legs --no-isolated --steps 50 > $GRAFT_REPO_ROOT/gpurun_out/nc_$cfg.json 2>/dev/null
done
