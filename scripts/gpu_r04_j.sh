# Round 4 pass j: where the certified fallback's cost comes from (decode kernel + POMO per
# variant), then the round profile: the bench line and the rocprofv3 kernel-trace summary
# of the same invocation.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VARIANTS="never trivial t2never nofb" bash scripts/gpu_decode_variants.sh || exit 1
mkdir -p gpurun_out/rp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rp -o bench -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/rp/bench_line.log 2> gpurun_out/rp/bench_err.log
rc=$?; echo "[$rc] profiled bench"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/rp/bench_err.log; exit $rc; fi
tail -1 gpurun_out/rp/bench_line.log | cut -c1-300
