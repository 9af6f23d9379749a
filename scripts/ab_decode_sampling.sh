cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_decode_exact.py tests/test_gpu_decode_certified.py tests/test_gpu_golden.py tests/test_gpu_pomo.py tests/test_gpu_dropin.py tests/test_gpu_policy.py tests/test_gpu_ops.py tests/test_gpu_provenance.py tests/test_gpu_host_vs_device.py -m gpu > gpurun_out/pt_dd.log 2>&1; rc=$?; tail -3 gpurun_out/pt_dd.log; [ $rc -ne 0 ] && exit $rc
for v in base nocompact base nocompact; do
  if [ $v = base ]; then L=rl4co_slap_amd/_lib/libco_env.so; else L=tools/_variants/libco_env_$v.so; fi
  DIAG_LIB=$L DIAG_DECODE_MODE=1 DIAG_SIZES=tsp100 timeout -k 10 120 python tools/diag_decode.py 2>/dev/null | grep "clip=10" | sed "s/^/$v /" || exit 1
done
