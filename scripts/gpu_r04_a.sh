# Round 4 first GPU pass: new tests, certified-decode variants, SQ counters.
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r04_newtests.sh || exit $?
VARIANTS="w8 w8max w8both max" bash scripts/gpu_decode_variants.sh > gpurun_out/dvar.log 2>&1; rc=$?; cat gpurun_out/dvar.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_pmc_sq_r04.sh > gpurun_out/pmcsq_r04.log 2>&1; rc=$?; tail -14 gpurun_out/pmcsq_r04.log; exit $rc
