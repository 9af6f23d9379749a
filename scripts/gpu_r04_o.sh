# Round 4 pass o: the fused env decode steps' certified picks against the exact path on
# adversarial near-ties (new test), and the fused CVRP step with only the unconditional
# staged-row reads (A/B against the product, interleaved).
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_dropin_slap.py tests/test_gpu_decode_certified.py > gpurun_out/o_tests.log 2>&1
rc=$?; tail -3 gpurun_out/o_tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/o_tests.log | head -20; exit $rc; fi
for p in 1 2 3; do
  timeout -k 10 120 python3 tools/diag_cvrp_fused.py || exit 1
  CO_LIB=tools/_variants/libco_env_cvrplds.so timeout -k 10 120 python3 tools/diag_cvrp_fused.py | sed 's/^/lds: /' || exit 1
done
