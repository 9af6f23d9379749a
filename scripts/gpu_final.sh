# round-end evidence in one call: the whole GPU suite + smoke(), then the bench under
# rocprofv3 with PMC traffic passes (scripts/gpu_round_profiles.sh)
cd $GRAFT_REPO_ROOT
bash scripts/gpu_full.sh || exit $?
STEPS=${STEPS:-20} PMC_KERNELS="${PMC_KERNELS:-tsp_fused_teacher pomo_tsp100 cvrp_stepwise_pair slap_fused_closest_b65536}" bash scripts/gpu_round_profiles.sh
