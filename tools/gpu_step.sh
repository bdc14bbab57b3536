timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06h_pytest.log 2>&1; tail -2 gpurun_out/r06h_pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06h_smoke.log 2>&1; cat gpurun_out/r06h_smoke.log
bash tools/profile_round.sh r06b > gpurun_out/prof_r06b.log 2>&1; tail -2 gpurun_out/prof_r06b.log
