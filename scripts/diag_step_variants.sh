cd $GRAFT_REPO_ROOT
for v in ${VARIANTS:-base}; do
  echo "== $v $(CO_LIB=tools/_variants/libco_env_$v.so timeout -k 10 120 python tools/run_mode.py steps 2>/dev/null | tail -1 | cut -c1-600)" || exit 1
done
