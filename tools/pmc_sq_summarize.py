"""Per-kernel SQ counter summary of scripts/gpu_pmc_sq.sh (passes A / B / C per target)
-> profiles/<round>_pmc_sq.txt (diagnostic).  Fractions of wave cycles: waiting (s_waitcnt /
barrier), issue-stalled, issuing (SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~
SQ_WAVE_CYCLES); per-wave instruction counts; vmem_latency = SQ_INST_LEVEL_VMEM /
SQ_INSTS_VMEM (average cycles a vector memory instruction is outstanding; level counters
and wave cycles are in quad-cycles: MI355X_MICROARCH.md)."""
import collections
import csv
import glob
import os
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd = sys.argv[1] if len(sys.argv) > 1 else "r04"
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "gpurun_out/pmcsq/*.[ABC]/run_counter_collection.csv"))):
    target = os.path.basename(os.path.dirname(f)).rsplit(".", 1)[0]
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        name = name.split("(")[0]
        if name.startswith("at::") or "rocclr" in name or "elementwise" in name:
            continue
        agg[(target, name)][r["Counter_Name"]].append(float(r["Counter_Value"]))
lines = [__doc__.strip(), ""]
for (target, name), cs in agg.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    waves = max(m.get("SQ_WAVES", 1), 1)
    wc = m.get("SQ_WAVE_CYCLES", 0) or 1
    vm = m.get("SQ_INSTS_VMEM_RD", 0) + m.get("SQ_INSTS_VMEM_WR", 0)
    rec = {
        "waves": waves,
        "wave_cycles/wave": wc / waves,
        "wait_any": m.get("SQ_WAIT_ANY", 0) / wc, "wait_inst": m.get("SQ_WAIT_INST_ANY", 0) / wc,
        "active": m.get("SQ_ACTIVE_INST_ANY", 0) / wc,
        "valu/wave": m.get("SQ_INSTS_VALU", 0) / waves, "salu/wave": m.get("SQ_INSTS_SALU", 0) / waves,
        "vmem_rd/wave": m.get("SQ_INSTS_VMEM_RD", 0) / waves,
        "vmem_wr/wave": m.get("SQ_INSTS_VMEM_WR", 0) / waves,
        "lds/wave": m.get("SQ_INSTS_LDS", 0) / waves, "smem/wave": m.get("SQ_INSTS_SMEM", 0) / waves,
        "branch/wave": m.get("SQ_INSTS_BRANCH", 0) / waves,
        "vmem_latency": m.get("SQ_INST_LEVEL_VMEM", 0) / vm if vm else None,
        "active_valu": m.get("SQ_ACTIVE_INST_VALU", 0) / wc, "active_sca": m.get("SQ_ACTIVE_INST_SCA", 0) / wc,
        "active_lds": m.get("SQ_ACTIVE_INST_LDS", 0) / wc, "wait_inst_lds": m.get("SQ_WAIT_INST_LDS", 0) / wc,
        "active_vmem": m.get("SQ_ACTIVE_INST_VMEM", 0) / max(m.get("SQ_WAVE_CYCLES", 0), 1),
        "ta_addr_full": m.get("SQ_VMEM_TA_ADDR_FIFO_FULL"), "ta_cmd_full": m.get("SQ_VMEM_TA_CMD_FIFO_FULL"),
        "grbm_gui_active": m.get("GRBM_GUI_ACTIVE"),
    }
    s = " ".join(f"{k}={v:.3g}" if isinstance(v, float) else f"{k}={v}" for k, v in rec.items()
                  if v is not None)
    lines.append(f"{target:28s} {name[:48]:48s}\n    {s}")
out = "\n".join(lines) + "\n"
open(os.path.join(root, "profiles", f"{rnd}_pmc_sq.txt"), "w").write(out)
print(out)
