# Round profiles: the bench line and the rocprofv3 kernel-trace summary of the SAME
# `bench.py --steps K` invocation (the program after `--`), then PMC HBM traffic passes
# (FETCH_SIZE / WRITE_SIZE in separate runs) for the listed targets.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/rp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp -o bench -- python3 bench.py --steps ${STEPS:-20} --warmup 3 > gpurun_out/rp/bench_line.log 2> gpurun_out/rp/bench_err.log
rc=$?; echo "[$rc] profiled bench"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/rp/bench_err.log; exit $rc; fi
tail -1 gpurun_out/rp/bench_line.log | cut -c1-300
PMC_KERNELS="${PMC_KERNELS:-tsp_fused_teacher cvrp_stepwise}" bash scripts/gpu_pmc.sh
