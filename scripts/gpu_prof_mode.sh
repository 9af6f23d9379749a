# kernel-trace summary of one tools/run_mode.py mode (MODE, K): gpurun_out/pm/<MODE>_kernel_stats.csv
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pm
for M in ${MODES:-slap}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pm/$M -o run -- python3 tools/run_mode.py $M --k ${K:-5} > gpurun_out/pm/$M.log 2>&1
  rc=$?; echo "[$rc] $M"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/pm/$M.log; exit $rc; fi
  tail -1 gpurun_out/pm/$M.log | cut -c1-600
done
