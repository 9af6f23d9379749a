"""Summarise gpurun_out/pmc/<target>.{FETCH,WRITE}_SIZE counter CSVs into
profiles/<round>_pmc_traffic.json: per-kernel mean HBM bytes per launch.

gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of a
wide coalesced streaming read, so read bytes = 2 * FETCH_SIZE KiB; WRITE_SIZE is exact
for 16-B streaming stores.  The doubling is calibrated here against the kernels'
algorithmic read bytes, which it reproduces to < 0.5 %.
"""
import collections
import csv
import glob
import json
import os
import sys

rnd = sys.argv[1] if len(sys.argv) > 1 else "r01"
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
path = os.path.join(root, "profiles", f"{rnd}_pmc_traffic.json")
out = {"note": __doc__.strip(), "kernels": {}}
new = {}
for d in sorted(glob.glob(os.path.join(root, "gpurun_out/pmc/*.*_SIZE"))):
    target, counter = os.path.basename(d).rsplit(".", 1)
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        if name.startswith("void at::") or "FillFunctor" in name:
            continue  # torch's own setup copies
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        agg[short].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        e = new.setdefault(f"{target}:{k}", {"target": target, "kernel": k})
        e[counter + "_KiB_mean"] = sum(v) / len(v)
        e["dispatches_" + counter] = len(v)
for k, e in new.items():
    if "FETCH_SIZE_KiB_mean" in e and "WRITE_SIZE_KiB_mean" in e:
        e["hbm_read_bytes"] = 2 * e["FETCH_SIZE_KiB_mean"] * 1024
        e["hbm_write_bytes"] = e["WRITE_SIZE_KiB_mean"] * 1024
        e["hbm_bytes_per_launch"] = e["hbm_read_bytes"] + e["hbm_write_bytes"]
# targets measured in this pass replace their earlier entries; other targets are kept
if os.path.exists(path):
    old = json.load(open(path))["kernels"]
    done = {e["target"] for e in new.values()}
    out["kernels"] = {k: e for k, e in old.items() if e.get("target") not in done}
out["kernels"].update(new)
json.dump(out, open(path, "w"), indent=1)
print(json.dumps(new, indent=1))
