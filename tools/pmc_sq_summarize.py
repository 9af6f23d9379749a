"""Per-kernel means of the SQ counters from scripts/gpu_pmc_sq.sh (diagnostic)."""
import collections
import csv
import glob
import os

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for f in sorted(glob.glob(os.path.join(root, "gpurun_out/pmcsq/*/run_counter_collection.csv"))):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(os.path.basename(os.path.dirname(f)))
    for k, cs in agg.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        wc = m.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"  {k[:60]:60s} waves={m.get('SQ_WAVES', 0):.0f} "
              f"wait_any={m.get('SQ_WAIT_ANY', 0) / wc:.2f} "
              f"wait_inst={m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
              f"active={m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
              f"valu/wave={m.get('SQ_INSTS_VALU', 0) / max(m.get('SQ_WAVES', 1), 1):.0f} "
              f"salu/wave={m.get('SQ_INSTS_SALU', 0) / max(m.get('SQ_WAVES', 1), 1):.0f} "
              f"busy={m.get('SQ_BUSY_CYCLES', 0):.0f}")
