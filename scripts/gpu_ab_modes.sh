# A/B of tools/run_mode.py modes (MODES) over variant libraries (VARIANTS, tools/_variants),
# then an optional rocprofv3 kernel trace of one mode with one variant (PROF="mode variant")
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for r in 1 2; do
  for v in ${VARIANTS:-base}; do
    for m in ${MODES:-slap65k}; do
      CO_LIB=tools/_variants/libco_env_$v.so timeout -k 10 200 python tools/run_mode.py $m --k ${K:-5} > gpurun_out/ab/$m.$v.$r.txt 2>&1 || exit $?
      echo "== $v $m $(tail -1 gpurun_out/ab/$m.$v.$r.txt | cut -c1-900)"
    done
  done
done
if [ -n "$PROF" ]; then
  set -- $PROF
  CO_LIB=tools/_variants/libco_env_$2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/prof -o run -- python3 tools/run_mode.py $1 --k 3 > gpurun_out/ab/prof.log 2>&1 || exit $?
  python3 tools/ktrace_grid.py gpurun_out/ab/prof/run_kernel_trace.csv ${PROFK:-slap}
fi
