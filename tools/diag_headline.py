"""Diagnostic: GPU time of the headline launch (co_tsp_rollout_ex, teacher-forced TSP-100
episode on row-major actions) at B = 65,536, HIP events over 100 launches, 4 input batches
cycled so each launch reads HBM (as bench.py does).  CO_LIB picks a variant library
(tools/build_variants.sh); prints one JSON line.  Also returns a checksum of the outputs
so two libraries can be compared for identical results."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rl4co_slap_amd import _native  # noqa: E402
from rl4co_slap_amd.rollout import engine  # noqa: E402

if os.environ.get("CO_LIB"):
    _native.LIB_PATH = os.environ["CO_LIB"]
_native.load()
dev = torch.device("cuda:0")
b = int(os.environ.get("DIAG_B", 65536))
n = int(os.environ.get("DIAG_N", 100))
eps = []
for salt in range(4):
    locs, acts = bench.tsp_inputs(b, n, 0, salt)
    eps.append(engine.TSPFusedEpisode(locs.to(dev), acts.to(dev)))
sh = torch.cuda.current_stream(dev).cuda_stream
it = [0]


def run():  # the bench's launch: the bound C-ABI call on the current stream
    eps[it[0] % 4]._bound(sh)
    it[0] += 1


res = []
for _ in range(5):
    _, ev = bench.timed(run, 100, 8, 1, dev)
    res.append(ev / 100 * 1e6)
res.sort()
fs = eps[0].final_state()
h = 0
for k in ("action_mask", "i", "first_node", "current_node", "done", "reward"):
    h = (h * 1000003 + int(fs[k].view(-1).to(torch.float64).mul(1.0 + torch.arange(
        fs[k].numel(), device=dev, dtype=torch.float64) % 7).sum().item() * 1e3)) % (1 << 61)
byt = (17 * n + 30) * b
print(json.dumps({"lib": os.environ.get("CO_LIB", "base"), "B": b, "N": n,
                  "us_median": round(res[2], 3), "us_all": [round(x, 2) for x in res],
                  "TBps": round(byt / res[2] / 1e6, 3), "frac": round(byt / res[2] / 8e6, 4),
                  "checksum": h, "status": int(eps[0].status.item())}))
