# quick iteration: selected GPU tests, the phase diagnostic and the bench
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ge 124 ]; then exit $rc; fi; }
step timeout -k 10 600 python -m pytest ${TESTS:-tests} -m gpu -q -p no:cacheprovider --maxfail=10 > gpurun_out/pytest_gpu.log 2>&1
tail -3 gpurun_out/pytest_gpu.log
if [ -x tools/diag_rollout ]; then step timeout -k 10 120 ./tools/diag_rollout > gpurun_out/diag.log 2>&1; cat gpurun_out/diag.log; fi
step timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log | cut -c1-600
