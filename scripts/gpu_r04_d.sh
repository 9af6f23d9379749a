# Round 4 pass d: env-kernel tests after the CVRP merged stores, step timings, host profile
# of the drop-in loops.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_envs.py tests/test_gpu_fullsize.py tests/test_gpu_large_n.py tests/test_gpu_golden.py \
  tests/test_gpu_dropin.py tests/test_gpu_dropin_slap.py > gpurun_out/r04_gputests_d.log 2>&1
rc=$?; tail -3 gpurun_out/r04_gputests_d.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r04_gputests_d.log | head -20; exit $rc; fi
for p in 1 2; do timeout -k 10 120 python3 tools/run_mode.py steps; done || exit 1
for e in tsp cvrp slap; do CO_ENV=$e timeout -k 10 180 python3 tools/prof_dropin_host.py > gpurun_out/prof_host_$e.txt 2>&1 || exit 1; tail -1 gpurun_out/prof_host_$e.txt; done
