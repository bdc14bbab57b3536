#!/bin/bash
# r05f round validation of the final binary: the whole -m gpu suite (one process),
# smoke(), then the round profile (tools/profile_round.sh r05f).
set -e -o pipefail
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
bash tools/profile_round.sh r05f
