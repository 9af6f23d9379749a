# CVRP step parity tests + step timings of the base library and variants (VARIANTS)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_envs.py} -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread ${PYK:+-k "$PYK"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for v in ${VARIANTS:-base}; do
  echo "== $v $(CO_LIB=tools/_variants/libco_env_$v.so timeout -k 10 120 python tools/run_mode.py steps 2>/dev/null | tail -1 | cut -c1-600)" || exit 1
done
done
for m in ${MODES}; do
  timeout -k 10 200 python tools/run_mode.py $m --k 10 > gpurun_out/mode_$m.txt 2>&1 || exit $?
  tail -1 gpurun_out/mode_$m.txt | cut -c1-1200
done
