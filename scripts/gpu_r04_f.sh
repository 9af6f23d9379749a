# Round 4 pass f: SLAP fused kernel (int16 LDS picklist, assignment copy not unrolled) tests
# and LATE variants at B = 65,536; certified-decode fallback diagnostics.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/f
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_rollout.py tests/test_gpu_golden.py > gpurun_out/f/tests.log 2>&1
rc=$?; tail -3 gpurun_out/f/tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/f/tests.log | head -20; exit $rc; fi
CO_LIB=tools/_variants/libco_env_fbcnt.so timeout -k 10 120 python3 tools/diag_cert_count.py || exit 1
for pass in 1 2; do
  for V in product slap_l1 slap_l2; do
    if [ "$V" = product ]; then LIB=""; else LIB=tools/_variants/libco_env_$V.so; fi
    CO_LIB=$LIB timeout -k 10 200 python3 tools/run_mode.py slap65k --k 5 > gpurun_out/f/$V.$pass.json 2> gpurun_out/f/$V.$pass.err
    rc=$?; echo "[$rc] $pass $V"; python3 -c "
import json,sys; d=json.load(open('gpurun_out/f/$V.$pass.json'))
print({k: d[k] for k in d if not isinstance(d[k], (dict, list))})
print('roofline', d.get('roofline')); print('stepwise', {k: v for k, v in d.get('stepwise', {}).items() if not isinstance(v, (dict, list))})" || true
    if [ $rc -ne 0 ]; then tail -3 gpurun_out/f/$V.$pass.err; exit $rc; fi
  done
done
VARIANTS="fbnever" bash scripts/gpu_decode_variants.sh || exit 1
