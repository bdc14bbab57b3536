# frame pushes before vs after complete_next in the bench step (headline A/B, 3 pairs)
set -e
mkdir -p gpurun_out
: > gpurun_out/pushab.log
for i in 1 2 3; do
  for o in "" "--push-last"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-secondary --no-legs --no-isolated $o > gpurun_out/pushab.json 2> gpurun_out/pushab.err
    python3 -c "
import json,sys;d=json.loads(open('gpurun_out/pushab.json').read().strip().splitlines()[-1]);s=d['segments'];print(sys.argv[1] or 'before',d['value'],s['median'],s['slowest_steps'])" "$o" >> gpurun_out/pushab.log
  done
done
