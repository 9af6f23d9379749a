# Round 4 pass l: is it the LDS stash? (decode / POMO timings per variant), then the SQ
# counters of the fused CVRP decode + env step (the drop-in loop).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VARIANTS="nostash stashonly trivial" bash scripts/gpu_decode_variants.sh || exit 1
PMC_KERNELS="dropin_cvrp" bash scripts/gpu_pmc_sq_r04.sh || exit 1
