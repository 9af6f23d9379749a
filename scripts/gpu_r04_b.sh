# Round 4: the whole GPU suite, then the default bench line.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/r04_gputests.log 2>&1
rc=$?; tail -5 gpurun_out/r04_gputests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/r04_gputests.log | head -20; exit $rc; fi
timeout -k 10 600 python3 bench.py > gpurun_out/r04_bench.json 2> gpurun_out/r04_bench.err
rc=$?; echo "[$rc] bench"; tail -c 3000 gpurun_out/r04_bench.json; tail -3 gpurun_out/r04_bench.err; exit $rc
