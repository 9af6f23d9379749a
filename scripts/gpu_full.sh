# the whole GPU suite, smoke(), then the drop-in host measurements
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "[smoke $rc]"; tail -2 gpurun_out/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/host_costs.py > gpurun_out/host_costs.txt 2>&1 && tail -2 gpurun_out/host_costs.txt | cut -c1-600 &&
timeout -k 10 300 python tools/run_mode.py dropin --k 10 > gpurun_out/dropin_glue.txt 2>&1 && tail -1 gpurun_out/dropin_glue.txt | cut -c1-900 &&
timeout -k 10 300 python tools/run_mode.py pomo --k 10 > gpurun_out/pomo.txt 2>&1 && tail -1 gpurun_out/pomo.txt | cut -c1-300
