# Round 4 pass g: the two-tier certified fallback (full GPU suite), fallback counts,
# decode / POMO timings against the no-fallback bound, SLAP late-coordinate variant.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/g
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/g/tests.log 2>&1
rc=$?; tail -3 gpurun_out/g/tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/g/tests.log | head -20; exit $rc; fi
CO_LIB=tools/_variants/libco_env_fbcnt.so timeout -k 10 120 python3 tools/diag_cert_count.py || exit 1
VARIANTS="nofb" bash scripts/gpu_decode_variants.sh || exit 1
for pass in 1 2; do
  for V in product slap_l1 slap_l1w8; do
    if [ "$V" = product ]; then LIB=""; else LIB=tools/_variants/libco_env_$V.so; fi
    CO_LIB=$LIB timeout -k 10 200 python3 tools/run_mode.py slap65k --k 5 > gpurun_out/g/$V.$pass.json 2> gpurun_out/g/$V.$pass.err
    rc=$?; echo "[$rc] $pass $V $(head -c 700 gpurun_out/g/$V.$pass.json)"
    if [ $rc -ne 0 ]; then tail -3 gpurun_out/g/$V.$pass.err; exit $rc; fi
  done
done
VARIANTS="tsp_nt1 tsp_nt3 tsp_nt7" bash scripts/gpu_step_variants.sh || exit 1
