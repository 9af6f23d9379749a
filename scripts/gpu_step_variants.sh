# Step-kernel variants (tools/build_variants.sh -s tsp|cvrp ...): step_kernels_vs_copy per
# library, interleaved twice so box drift shows.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/svar
for pass in 1 2; do
  for V in product ${VARIANTS}; do
    if [ "$V" = product ]; then LIB=""; else LIB=tools/_variants/libco_env_$V.so; fi
    CO_LIB=$LIB timeout -k 10 120 python3 tools/run_mode.py steps > gpurun_out/svar/$V.$pass.json 2> gpurun_out/svar/$V.$pass.err
    rc=$?; echo "[$rc] $pass $V $(tail -c 400 gpurun_out/svar/$V.$pass.json)"
    if [ $rc -ne 0 ]; then tail -3 gpurun_out/svar/$V.$pass.err; exit $rc; fi
  done
done
