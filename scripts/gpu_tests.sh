# run the GPU tests named in TESTS (default: all), log to gpurun_out/pytest_gpu.log
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 ${TLIMIT:-600} python -u -m pytest ${TESTS:-tests} -m gpu -q ${PYX:--x} -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -${TAILN:-8} gpurun_out/pytest_gpu.log
exit $rc
