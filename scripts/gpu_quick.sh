# quick iteration: selected GPU tests (TESTS) then the headline bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
step() { "$@"; rc=$?; echo "[$rc] $*"; if [ $rc -ge 124 ]; then exit $rc; fi; }
step timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -q -x -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
tail -15 gpurun_out/pytest_gpu.log
step timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-modes --no-cpu > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log | cut -c1-1500
