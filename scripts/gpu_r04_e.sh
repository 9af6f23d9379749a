# Round 4 pass e: SLAP host-known done (tests + drop-in bench), TSP step row-group
# unrolling variants, certified decode without its fallback (timing diagnostic).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_dropin_slap.py tests/test_gpu_envs.py > gpurun_out/r04_gputests_e.log 2>&1
rc=$?; tail -3 gpurun_out/r04_gputests_e.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r04_gputests_e.log | head -20; exit $rc; fi
timeout -k 10 300 python3 tools/run_mode.py dropin_slap --k 10 > gpurun_out/r04_dropin_slap_e.json || exit 1
tail -c 1500 gpurun_out/r04_dropin_slap_e.json; echo
VARIANTS="tsp_unr2 tsp_unr4" bash scripts/gpu_step_variants.sh || exit 1
VARIANTS="nofb" bash scripts/gpu_decode_variants.sh || exit 1
