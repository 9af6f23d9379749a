# Round 4 pass p: the fused CVRP transition reading its staged row as float4 demand + aligned
# visited dwords: the drop-in / fused-step GPU tests, then A/B against the previous library.
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dropin_slap.py tests/test_gpu_dropin.py tests/test_gpu_golden.py > gpurun_out/p_tests.log 2>&1
rc=$?; tail -3 gpurun_out/p_tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/p_tests.log | head -20; exit $rc; fi
for p in 1 2 3; do
  timeout -k 10 120 python3 tools/diag_cvrp_fused.py || exit 1
  CO_LIB=tools/_variants/libco_env_prev.so timeout -k 10 120 python3 tools/diag_cvrp_fused.py | sed 's/^/prev: /' || exit 1
done
timeout -k 10 300 python3 tools/run_mode.py dropin_cvrp --k 5 > gpurun_out/p_dropin_cvrp.json 2>/dev/null && head -c 300 gpurun_out/p_dropin_cvrp.json
