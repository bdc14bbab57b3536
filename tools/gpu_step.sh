tools/gpu_ab.sh ab_pets 3 --box-dist pets --no-legs --no-secondary --no-cpu-baseline --no-isolated --steps 60 --warmup 5 > gpurun_out/ab_pets.txt 2>&1
tools/gpu_ab.sh ab_4k 2 --width 3840 --height 2160 --cameras 8 --points 4096 --boxes 64 --no-legs --no-secondary --no-cpu-baseline --no-isolated --steps 6 --warmup 2 --measure-steps 2 > gpurun_out/ab_4k.txt 2>&1
cat gpurun_out/ab_pets.txt gpurun_out/ab_4k.txt
timeout -k 10 300 python -u -m pytest tests/test_lk_gpu.py -k "box_kernel_16 or empty_query" -x -q --timeout 120 --timeout-method thread > gpurun_out/r06c_new.log 2>&1; tail -3 gpurun_out/r06c_new.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06c_pytest.log 2>&1; tail -3 gpurun_out/r06c_pytest.log
