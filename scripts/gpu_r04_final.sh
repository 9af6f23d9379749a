# Round 4 final: A (suite, smoke, bench lines, kernel-trace profile) then B (PMC traffic, SQ).
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r04_final_a.sh && bash scripts/gpu_r04_final_b.sh
