# Round 4 pass h: the round profile (bench line + rocprofv3 kernel-trace summary of the same
# invocation), PMC HBM traffic for the headline / drop-in / POMO kernels, SQ passes for the
# fused CVRP / SLAP decode + env step kernels.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
STEPS=20 PMC_KERNELS="tsp_fused_teacher dropin_cvrp dropin_slap pomo_tsp100" bash scripts/gpu_round_profiles.sh || exit 1
PMC_KERNELS="dropin_cvrp dropin_slap" bash scripts/gpu_pmc_sq_r04.sh || exit 1
