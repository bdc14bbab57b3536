#!/bin/bash
# r05h: whole -m gpu suite, smoke(), round profile of the final binary
set -e -o pipefail
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/profile_round.sh r05h
