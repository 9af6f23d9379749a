"""Diagnostic timing of the fused SLAP episode (not part of the product):
graph-replayed launches at B = 16384 and 65536; DIAG_LIB selects a variant library."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rl4co_slap_amd import _native as nat  # noqa: E402

if os.environ.get("DIAG_LIB"):
    nat.LIB_PATH = os.environ["DIAG_LIB"]
print("lib:", nat.LIB_PATH)
nat.load()
from rl4co_slap_amd.envs.slap import SLAPGenerator  # noqa: E402
from rl4co_slap_amd.rollout.engine import SLAPFusedEpisode  # noqa: E402

dev = torch.device("cuda:0")
for b in (16384, 65536):
    torch.manual_seed(1234)
    np.random.seed(1234)
    td = SLAPGenerator(materialize_dist_mat=False)(b).to(dev)
    pol = os.environ.get("DIAG_POLICY", "closest")
    acts = None
    if pol == "teacher":
        torch.manual_seed(4321)
        acts = (torch.rand(b, 99).argsort(1)[:, :20] + 1).to(dev)
    fu = SLAPFusedEpisode(td, actions=acts, policy=pol)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fu._launch(side.cuda_stream)
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s = torch.cuda.current_stream().cuda_stream
        for _ in range(20):
            fu._launch(s)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    print(f"SLAP fused {pol} B={b}: {us:.1f} us  {b * 2754 / us / 1e3:.0f} GB/s "
          f"status={int(fu.status.item())} reward_sum={float(fu.reward.sum()):.3f}")
