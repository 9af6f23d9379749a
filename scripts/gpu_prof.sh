# rocprofv3 kernel trace + stats of a short bench run (no counters: --pmc runs separately)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/prof_bench.log 2>&1
rc=$?; echo "rc=$rc"
find gpurun_out/prof -name "*stats*" | head
