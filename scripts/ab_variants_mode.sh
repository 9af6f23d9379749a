# GPU tests (TESTS=...) then A/B timing of one tools/run_mode.py mode (MODE) against
# diagnostic variant libraries (tools/build_variants.sh): VARIANTS="base name ...", 3 rounds.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider $TESTS -m gpu > gpurun_out/pt_ab.log 2>&1; rc=$?; tail -3 gpurun_out/pt_ab.log; [ $rc -ne 0 ] && exit $rc
fi
for r in 1 2 3; do
  for v in ${VARIANTS:-base}; do
    # a variant "NAME@steps" runs NAME with the step-major TSP layout (CO_TSP_LAYOUT)
    lay=rows; vv=$v; case $v in *@*) lay=${v#*@}; vv=${v%@*};; esac
    if [ $vv = base ]; then L=rl4co_slap_amd/_lib/libco_env.so; else L=tools/_variants/libco_env_$vv.so; fi
    echo "$v $(CO_TSP_LAYOUT=$lay CO_LIB=$L timeout -k 10 120 python tools/run_mode.py ${MODE:-tsp} --k ${K:-5} 2>/dev/null | tail -1 | cut -c1-400)" || exit 1
  done
done
