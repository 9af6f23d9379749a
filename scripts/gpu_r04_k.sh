# Round 4 pass k: the certified fallback laid out after the hot path (branch hint): decode
# GPU tests, then decode / POMO timings against the certification-only and no-fallback bounds.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/k
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_decode_certified.py tests/test_gpu_decode_exact.py tests/test_gpu_pomo.py \
  tests/test_gpu_dropin.py tests/test_gpu_dropin_slap.py tests/test_gpu_golden.py > gpurun_out/k/tests.log 2>&1
rc=$?; tail -3 gpurun_out/k/tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/k/tests.log | head -20; exit $rc; fi
VARIANTS="trivial nofb" bash scripts/gpu_decode_variants.sh || exit 1
for m in dropin_cvrp dropin_slap; do timeout -k 10 300 python3 tools/run_mode.py $m --k 5 > gpurun_out/k/$m.json 2> gpurun_out/k/$m.err || exit 1; echo "$m $(head -c 600 gpurun_out/k/$m.json)"; done
