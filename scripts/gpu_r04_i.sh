# Round 4 pass i: the lean certified fast pass (full GPU suite), fallback counts (decode
# shape + POMO episode), decode / POMO timings, then the round profile (bench line +
# rocprofv3 kernel-trace summary, PMC traffic) and SQ passes for the fused env decode steps.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/i
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
  > gpurun_out/i/tests.log 2>&1
rc=$?; tail -3 gpurun_out/i/tests.log; echo "[$rc] gpu tests"
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" gpurun_out/i/tests.log | head -20; exit $rc; fi
CO_LIB=tools/_variants/libco_env_fbcnt.so timeout -k 10 180 python3 tools/diag_cert_count.py || exit 1
VARIANTS="nofb" bash scripts/gpu_decode_variants.sh || exit 1

