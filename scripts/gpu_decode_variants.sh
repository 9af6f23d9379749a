# Round 4: certified decode variants (tools/build_variants.sh -s decode_tsp ...), each timed
# as the fused TSP decode step alone (102,400 x 100, clip 10) and as the POMO episode.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dvar
for V in product ${VARIANTS}; do
  if [ "$V" = product ]; then LIB=""; else LIB=tools/_variants/libco_env_$V.so; fi
  for M in decode_kernels pomo_cert; do
    CO_LIB=$LIB timeout -k 10 240 python3 tools/run_mode.py $M --k 5 > gpurun_out/dvar/$V.$M.json 2> gpurun_out/dvar/$V.$M.err
    rc=$?; echo "[$rc] $V $M $(tail -c 300 gpurun_out/dvar/$V.$M.json)"
    if [ $rc -ne 0 ]; then tail -3 gpurun_out/dvar/$V.$M.err; exit $rc; fi
  done
done
