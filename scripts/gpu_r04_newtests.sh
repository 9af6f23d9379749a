# Round 4: the new drop-in SLAP / fused decode+env tests and the layout tests, then the
# SQ counter passes (scripts/gpu_pmc_sq_r04.sh).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dropin_slap.py "tests/test_gpu_rollout.py::test_tsp_reward_row_kernel_layouts" \
  "tests/test_gpu_ops.py::test_gather_out_of_range_outside_env_raises" \
  > gpurun_out/r04_newtests.log 2>&1
rc=$?; tail -30 gpurun_out/r04_newtests.log; echo "[$rc] new tests"
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$WITH_SQ" ]; then bash scripts/gpu_pmc_sq_r04.sh > gpurun_out/pmcsq_r04.log 2>&1; rc=$?; tail -14 gpurun_out/pmcsq_r04.log; exit $rc; fi
