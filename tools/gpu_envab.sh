# A/B of runtime settings on the Tracker2D headline (value, median segment, slowest steps)
set -e
mkdir -p gpurun_out
: > gpurun_out/envab.log
for cfg in ${ENVAB_CFGS:-"X=1"}; do
  env $cfg timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-legs --no-isolated --step-profile > gpurun_out/envab.json 2> gpurun_out/envab.err
  python3 -c "
import json,sys;d=json.loads(open('gpurun_out/envab.json').read().strip().splitlines()[-1]);s=d['segments'];print(sys.argv[1],d['value'],s['median'],s['slowest_steps'],[round(x,1) for x in s['warmup_step_ms']][:6])" "$cfg" >> gpurun_out/envab.log
done
