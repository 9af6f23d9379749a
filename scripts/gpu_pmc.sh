# HBM traffic of the engine kernels from PMC counters: FETCH_SIZE and WRITE_SIZE in
# separate passes (TCC slot budget; MI355X_MICROARCH.md HBM section), kernel-trace only.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for K in ${PMC_KERNELS:-tsp_fused_teacher}; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc/$K.$C -o run -- python3 tools/pmc_target.py --kernel $K --k 5 ${PMC_ARGS} > gpurun_out/pmc/$K.$C.log 2>&1
    rc=$?; echo "[$rc] $K $C"; if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
find gpurun_out/pmc -name "*counter_collection*.csv" | head
