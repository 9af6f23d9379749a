"""Fused nearest-policy TSP-100 / CVRP-100 episodes at several batch sizes (diagnostic, not
part of the product): ms per episode by HIP events, to tell a throughput bound (time
proportional to B) from a residency bound (time flat while every wave fits at once).
Usage: python tools/nearest_scaling.py -> one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rl4co_slap_amd import _native as nat  # noqa: E402
from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode, TSPFusedEpisode  # noqa: E402

dev = torch.device("cuda:0")
nat.load()
sh = torch.cuda.current_stream(dev).cuda_stream
out = {}
for b in (4096, 8192, 16384, 32768, 49152, 65536, 98304, 131072):
    locs, _ = bench.tsp_inputs(b, 100, 0)
    ep = TSPFusedEpisode(locs.to(dev), None, policy="nearest", check=True)
    _, ev = bench.timed(lambda: ep._launch(sh), 5, 2, 1, dev)
    out[f"tsp_b{b}"] = round(ev / 5 * 1e3, 4)
    del ep, locs
for b in (8192, 16384, 32768, 49152, 65536):
    g = torch.Generator().manual_seed(1)
    la = torch.rand(b, 101, 2, generator=g)
    data = {"depot": la[:, 0].contiguous().to(dev), "locs": la[:, 1:].contiguous().to(dev),
            "demand": (((torch.rand(b, 100, generator=g) * 9).int() + 1).float() / 50).to(dev)}
    ep = CVRPFusedEpisode(data, vehicle_capacity=1.0)
    _, ev = bench.timed(lambda: ep.run_eager(), 5, 2, 1, dev)
    out[f"cvrp_b{b}"] = round(ev / 5 * 1e3, 4)
    del ep, data
print(json.dumps(out), flush=True)
