# Round 4 pass c: the GPU suite on the loop-free decode kernels, their timings, the TSP
# step variants, then the bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r04_gputests.log 2>&1
rc=$?; tail -3 gpurun_out/r04_gputests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r04_gputests.log | head -20; exit $rc; fi
timeout -k 10 120 python3 tools/run_mode.py decode_kernels > gpurun_out/r04_decode_kernels.json && cat gpurun_out/r04_decode_kernels.json || exit 1
VARIANTS="flat16 flat32" bash scripts/gpu_step_variants.sh > gpurun_out/svar.log 2>&1; rc=$?; cat gpurun_out/svar.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
rc=$?; echo "[$rc] bench"; tail -3 gpurun_out/r04_bench.err; exit $rc
