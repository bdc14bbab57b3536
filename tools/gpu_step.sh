VARIANTS="PIPE0 PIPE1 CH2 P1CH2" tools/gpu_ab.sh ab_lgpets 2 --box-dist pets --no-legs --no-secondary --no-cpu-baseline --no-isolated --steps 60 --warmup 5 > gpurun_out/ab_lg.txt 2>&1
VARIANTS="PIPE0 PIPE1 CH2 P1CH2" tools/gpu_ab.sh ab_lg4k 2 --width 3840 --height 2160 --cameras 8 --points 4096 --boxes 64 --no-legs --no-secondary --no-cpu-baseline --no-isolated --steps 6 --warmup 2 --measure-steps 2 >> gpurun_out/ab_lg.txt 2>&1
cat gpurun_out/ab_lg.txt
