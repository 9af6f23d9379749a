# SQ stall / instruction-mix breakdown of the step and decode kernels (round 4): three
# kernel-trace-free PMC passes per target, each its own rocprofv3 run under a hard
# timeout (counter budget per pass: 8 SQ, 2 GRBM):
#   A: wave cycles split into waiting (s_waitcnt) / issue-stalled / issuing + VALU/SALU
#   B: memory-instruction mix and the average VMEM level (outstanding loads)
#   C: issue-stall causes (VALU / SALU / LDS / VMEM active) + TA FIFO full + clocks
#   PMC_KERNELS="tsp_stepwise cvrp_stepwise_pair" bash scripts/gpu_pmc_sq_r04.sh
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcsq
A="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"
B="SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL GRBM_GUI_ACTIVE GRBM_COUNT"
for K in ${PMC_KERNELS:-tsp_stepwise cvrp_stepwise_pair slap_stepwise_closest pomo_tsp100 slap_fused_closest_b65536}; do
  for P in A B C; do
    eval CTRS=\$$P
    timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/pmcsq/$K.$P -o run -- python3 tools/pmc_target.py --kernel $K --k 3 ${PMC_ARGS} > gpurun_out/pmcsq/$K.$P.log 2>&1
    rc=$?; echo "[$rc] $K $P"; if [ $rc -ne 0 ]; then tail -3 gpurun_out/pmcsq/$K.$P.log; exit $rc; fi
  done
done
