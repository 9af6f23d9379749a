# time one bench mode (tools/run_mode.py MODE) per variant library (tools/build_variants.sh)
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for v in ${VARIANTS:-base}; do
  echo "== $v"
  CO_LIB=tools/_variants/libco_env_$v.so timeout -k 10 120 python tools/run_mode.py ${MODE:-pomo} --k ${K:-5} 2>/dev/null | tail -1 | cut -c1-400 || exit 1
done
