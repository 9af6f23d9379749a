# Round 4 final A: the whole GPU suite, smoke(), a bench line without the profiler, then
# the round profile (bench line + rocprofv3 kernel-trace summary of the same invocation).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/fa gpurun_out/rp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/fa/tests.log 2>&1
rc=$?; tail -3 gpurun_out/fa/tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/fa/tests.log | head -20; exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fa/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/fa/smoke.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python3 bench.py > gpurun_out/fa/bench_noprof.json 2> gpurun_out/fa/bench_noprof.err
rc=$?; echo "[$rc] bench"; tail -c 400 gpurun_out/fa/bench_noprof.json; if [ $rc -ne 0 ]; then tail -5 gpurun_out/fa/bench_noprof.err; exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp -o bench -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/rp/bench_line.log 2> gpurun_out/rp/bench_err.log
rc=$?; echo "[$rc] profiled bench"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/rp/bench_err.log; exit $rc; fi
