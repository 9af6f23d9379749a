# Round 4 pass m: branch-free GreedyRow loads on rows of any N (no divergent partial-chunk
# path, so no waits on every outstanding load -- the fused env steps' LDS-DMA included),
# unconditional staged-row reads in the fused CVRP transition: the GPU suite, decode /
# POMO timings, the drop-in loops, a bench line.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/m
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/m/tests.log 2>&1
rc=$?; tail -3 gpurun_out/m/tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/m/tests.log | head -20; exit $rc; fi
VARIANTS="" bash scripts/gpu_decode_variants.sh || exit 1
for m in dropin_cvrp dropin_slap; do timeout -k 10 300 python3 tools/run_mode.py $m --k 5 > gpurun_out/m/$m.json 2> gpurun_out/m/$m.err || exit 1; echo "$m $(head -c 400 gpurun_out/m/$m.json)"; done
timeout -k 10 400 python3 bench.py > gpurun_out/m/bench_noprof.json 2> gpurun_out/m/bench_noprof.err
rc=$?; echo "[$rc] bench"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/m/bench_noprof.err; exit $rc; fi
