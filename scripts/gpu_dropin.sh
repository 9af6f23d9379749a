# drop-in path: GPU tests, then host cost per step with and without the step glue
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${TESTS:-"tests/test_gpu_torchstep.py tests/test_gpu_dropin.py tests/test_gpu_decode_certified.py tests/test_gpu_policy.py tests/test_gpu_envs.py tests/test_gpu_rollout.py tests/test_gpu_pomo.py"}
timeout -k 10 600 python -u -m pytest $T -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/run_mode.py dropin --k 10 > gpurun_out/dropin_glue.txt 2>&1 && tail -1 gpurun_out/dropin_glue.txt | cut -c1-900 &&
CO_NO_TORCHSTEP=1 timeout -k 10 300 python tools/run_mode.py dropin --k 10 > gpurun_out/dropin_py.txt 2>&1 && tail -1 gpurun_out/dropin_py.txt | cut -c1-900 &&
timeout -k 10 300 python tools/run_mode.py dropin_cvrp --k 10 > gpurun_out/dropin_cvrp.txt 2>&1 && tail -1 gpurun_out/dropin_cvrp.txt | cut -c1-900 &&
CO_NO_TORCHSTEP=1 timeout -k 10 300 python tools/run_mode.py dropin_cvrp --k 10 > gpurun_out/dropin_cvrp_py.txt 2>&1 && tail -1 gpurun_out/dropin_cvrp_py.txt | cut -c1-900 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-modes --no-cpu > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-900
