"""Per-(kernel, grid size) launch statistics from a rocprofv3 kernel_trace.csv
(diagnostic): the same kernel launched at different batch sizes is split by its grid,
so e.g. the POMO decode step (B = 102,400) and the drop-in one (B = 65,536) are told
apart.  Usage: python tools/ktrace_grid.py trace.csv [name-substring ...]"""
import collections
import csv
import statistics
import sys

path, pats = sys.argv[1], sys.argv[2:]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    if pats and not any(p in name for p in pats):
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[(name, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]))].append(dur)
for (name, grid, wg), v in sorted(agg.items()):
    print(f"{name[:60]:60s} grid={grid:>9d} wg={wg:>4d} n={len(v):>5d} "
          f"median_us={statistics.median(v):8.2f} mean_us={statistics.fmean(v):8.2f}")
