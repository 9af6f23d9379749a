# co_cvrp_reward per variant library: HIP-event timing, then a FETCH_SIZE PMC pass
# (tools/diag_cvrp_reward.py; the reward kernel's mean per check mode is read offline)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/rv
export TMPDIR=/tmp
for v in ${VARIANTS:-base}; do
  L=tools/_variants/libco_env_$v.so; [ "$v" = base ] && L=rl4co_slap_amd/_lib/libco_env.so
  CO_LIB=$L timeout -k 10 60 python tools/diag_cvrp_reward.py 2>/dev/null || exit 1
  CO_LIB=$L timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/rv/$v -o run -- python3 tools/diag_cvrp_reward.py > gpurun_out/rv/$v.log 2>&1 || exit 1
done
