# step-kernel iteration: the env-step parity tests (TESTS), then the step kernels beside
# a same-byte copy (twice) and the stepwise CVRP episodes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_envs.py} -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  timeout -k 10 120 python tools/run_mode.py steps > gpurun_out/steps_$i.txt 2>&1 || exit $?
  tail -1 gpurun_out/steps_$i.txt
done
for m in ${MODES:-cvrp}; do
  timeout -k 10 200 python tools/run_mode.py $m --k 10 > gpurun_out/mode_$m.txt 2>&1 || exit $?
  tail -1 gpurun_out/mode_$m.txt | cut -c1-1200
done
