#!/bin/bash
# r05a: new GPU tests (wide 4K windows, unsupported backward window, realistic Run)
# then the large-window phase clocks and isolated launch times.
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_lk_gpu.py tests/test_tracker2d_group.py tests/test_headline_gpu.py -m gpu -k "4k_wide or unsupported or realistic" > gpurun_out/r05a_t.log 2>&1
OUT=lgst bash tools/gpu_lgst.sh
