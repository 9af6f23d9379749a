# drop-in host cost: GPU tests of the step glue, the host cost breakdown, the drop-in modes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TESTS:-"tests/test_gpu_torchstep.py tests/test_gpu_dropin.py tests/test_gpu_policy.py tests/test_gpu_envs.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python tools/host_costs.py > gpurun_out/host_costs.txt 2>&1 && tail -2 gpurun_out/host_costs.txt &&
timeout -k 10 300 python tools/run_mode.py dropin --k 10 > gpurun_out/dropin_glue.txt 2>&1 && tail -1 gpurun_out/dropin_glue.txt | cut -c1-900 &&
timeout -k 10 300 python tools/run_mode.py dropin_cvrp --k 10 > gpurun_out/dropin_cvrp.txt 2>&1 && tail -1 gpurun_out/dropin_cvrp.txt | cut -c1-900
