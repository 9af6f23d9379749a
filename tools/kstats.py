"""Print a rocprofv3 kernel_stats.csv compactly: name, calls, average us (diagnostic)."""
import csv
import sys

for f in sys.argv[1:]:
    print(f)
    for r in csv.DictReader(open(f)):
        name = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0][:70]
        print(f"  {name:70s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs']) / 1e3:9.2f}")
