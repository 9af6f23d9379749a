# Round 4 final B: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes) for the bench's roofline
# kernels, the POMO decode step and the drop-in fused decode + env steps; SQ passes for the
# fused SLAP decode step.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
PMC_KERNELS="tsp_fused_teacher slap_fused_closest_b65536 pomo_tsp100 dropin_cvrp dropin_slap" bash scripts/gpu_pmc.sh || exit 1
PMC_KERNELS="dropin_slap" bash scripts/gpu_pmc_sq_r04.sh || exit 1
