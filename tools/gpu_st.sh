mkdir -p gpurun_out/st1
timeout -k 10 120 python tools/bx_time.py --reps 40 > gpurun_out/st1/time.json 2>&1 && \
WIN=64 WINH=64 NPTS=2048 timeout -k 10 120 python tools/bx_stamps.py > gpurun_out/st1/st64.json 2>&1 && \
WIN=64 WINH=160 NPTS=2048 timeout -k 10 120 python tools/bx_stamps.py > gpurun_out/st1/st160.json 2>&1
