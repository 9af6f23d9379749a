# Round 4 final (2): after the fused CVRP transition's vector staged reads -- the suite,
# smoke, bench lines, the kernel-trace profile, and the drop-in CVRP PMC traffic again.
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r04_final_a.sh && PMC_KERNELS="dropin_cvrp" bash scripts/gpu_pmc.sh
