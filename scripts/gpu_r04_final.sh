# Round 4 final: A (suite, smoke, bench lines, kernel-trace profile) then B (PMC traffic, SQ),
# then the drop-in CVRP loop with the product and a variant library (unconditional LDS reads
# in the fused CVRP transition).
cd $GRAFT_REPO_ROOT
bash scripts/gpu_r04_final_a.sh && bash scripts/gpu_r04_final_b.sh || exit 1
mkdir -p gpurun_out/fv
for pass in 1 2; do
  for V in product cvrpnb; do
    if [ "$V" = product ]; then LIB=""; else LIB=tools/_variants/libco_env_$V.so; fi
    CO_LIB=$LIB timeout -k 10 300 python3 tools/run_mode.py dropin_cvrp --k 5 > gpurun_out/fv/$V.$pass.json 2> gpurun_out/fv/$V.$pass.err
    rc=$?; echo "[$rc] $pass $V $(head -c 300 gpurun_out/fv/$V.$pass.json)"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
