timeout -k 10 300 python -u -m pytest tests/test_lk_gpu.py -k "merged_counted or counted_launch or box_kernel_16" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06g_new.log 2>&1; tail -3 gpurun_out/r06g_new.log
VARIANTS="A B" tools/gpu_ab.sh ab_merge3 2 --total-cameras 8 --points 2048 --boxes 32 --no-legs --no-secondary --no-cpu-baseline --no-isolated --steps 40 --warmup 3 > gpurun_out/ab_merge.txt 2>&1
VARIANTS="A B" tools/gpu_ab.sh ab_merge4k 2 --width 3840 --height 2160 --cameras 8 --points 4096 --boxes 64 --no-legs --no-secondary --no-cpu-baseline --no-isolated --steps 6 --warmup 2 --measure-steps 2 >> gpurun_out/ab_merge.txt 2>&1
VARIANTS="A B" tools/gpu_ab.sh ab_mergeh 2 --no-legs --no-secondary --no-cpu-baseline --no-isolated >> gpurun_out/ab_merge.txt 2>&1
cat gpurun_out/ab_merge.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06g_pytest.log 2>&1; tail -3 gpurun_out/r06g_pytest.log
