# SQ stall breakdown of the engine kernels (kernel-trace PMC pass only):
#   PMC_KERNELS="pomo_tsp100" bash scripts/gpu_pmc_sq.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsq
for K in ${PMC_KERNELS:-pomo_tsp100}; do
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES --output-format csv -d gpurun_out/pmcsq/$K -o run -- python3 tools/pmc_target.py --kernel $K --k 3 > gpurun_out/pmcsq/$K.log 2>&1
  rc=$?; echo "[$rc] $K"; if [ $rc -ne 0 ]; then exit $rc; fi
done
