cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-base}; do
  for m in pomo pomo_cert; do
    echo "== $v $m $(CO_LIB=tools/_variants/libco_env_$v.so timeout -k 10 120 python tools/run_mode.py $m --k 4 2>/dev/null | tail -1 | cut -c1-80)" || exit 1
  done
done
