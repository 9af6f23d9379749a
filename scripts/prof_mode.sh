# rocprofv3 kernel trace + stats of one bench mode: MODE=cvrp bash scripts/prof_mode.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pm
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pm -o $MODE -- python3 tools/run_mode.py $MODE --k ${K:-5} > gpurun_out/pm/$MODE.log 2>&1
rc=$?; echo "rc=$rc"; tail -1 gpurun_out/pm/$MODE.log
python3 - <<PY
import csv
for r in csv.DictReader(open("gpurun_out/pm/${MODE}_kernel_stats.csv")):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5} {float(r['AverageNs'])/1e3:9.2f} us  min {float(r['MinNs'])/1e3:8.2f}")
PY
