# GPU check: parity tests, smoke, short bench. Stops at the first crash/timeout
# (rc >= 124); ordinary test failures (rc 1) do not stop the later steps.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ge 124 ]; then exit $rc; fi; }
step timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider --maxfail=20 -o addopts="" ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
tail -5 gpurun_out/pytest_gpu.log
step timeout -k 10 300 python __graft_entry__.py > gpurun_out/smoke.log 2>&1
tail -3 gpurun_out/smoke.log
step timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
tail -3 gpurun_out/bench.log
if [ -n "$WITH_PROF" ]; then
  step bash scripts/gpu_prof.sh
  cat gpurun_out/prof/run_kernel_stats.csv | cut -c1-200
fi
