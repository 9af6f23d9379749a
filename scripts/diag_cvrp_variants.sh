# time co_cvrp_reward per variant library (tools/build_variants.sh), then the CVRP tests
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  CO_LIB=tools/_variants/libco_env_$v.so timeout -k 10 60 python tools/diag_cvrp_reward.py 2>/dev/null || exit 1
done
