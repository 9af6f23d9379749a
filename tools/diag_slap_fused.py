"""Diagnostic: GPU time of the fused SLAP closest-free episode (co_slap_rollout) at
B = 16,384 and 65,536, HIP events over 60 launches with input batches cycled past the
Infinity Cache (as bench.py), plus an output checksum so two libraries can be compared.
CO_LIB picks a variant library; DIAG_POLICY=teacher for the random-feasible policy."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from rl4co_slap_amd import _native as nat  # noqa: E402

if os.environ.get("CO_LIB"):
    nat.LIB_PATH = os.environ["CO_LIB"]
nat.load()
from rl4co_slap_amd.envs.slap import SLAPGenerator  # noqa: E402
from rl4co_slap_amd.rollout.engine import SLAPFusedEpisode  # noqa: E402

dev = torch.device("cuda:0")
pol = os.environ.get("DIAG_POLICY", "closest")
out = {"lib": os.environ.get("CO_LIB", "base"), "policy": pol}
for b in (16384, 65536):
    nrot = bench.rotation(b * 2754)
    eps = []
    for r in range(nrot):
        torch.manual_seed(1234 + r)
        np.random.seed(1234 + r)
        td = SLAPGenerator(materialize_dist_mat=False)(b).to(dev)
        acts = None
        if pol == "teacher":
            acts = (torch.rand(b, 99).argsort(1)[:, :20] + 1).t().contiguous().to(dev)
        eps.append(SLAPFusedEpisode(td, actions=acts, policy=pol))
    sh = torch.cuda.current_stream(dev).cuda_stream
    it = [0]

    def run():
        eps[it[0] % nrot]._launch(sh)
        it[0] += 1

    res = sorted(bench.timed(run, 60, 6, 1, dev)[1] / 60 * 1e6 for _ in range(3))
    e = eps[0]
    chk = float(e.reward.double().sum()) + float(e.assign.double().sum() if hasattr(e, "assign") else 0)
    out[f"b{b}"] = {"us": round(res[1], 2), "frac": round(b * 2754 / res[1] / 8e6, 4),
                    "batches": nrot, "checksum": chk, "status": int(e.status.item())}
print(json.dumps(out))
