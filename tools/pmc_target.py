"""Small driver for PMC passes: launches one engine kernel K times on the bench workload
(diagnostic tool, not part of the product)."""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

ap = argparse.ArgumentParser()
ap.add_argument("--kernel", default="tsp_fused_teacher")
ap.add_argument("--k", type=int, default=5)
ap.add_argument("--cycle", type=int, default=1,
                help="distinct input batches run in turn (4: the fused modes read HBM, not MALL)")
args = ap.parse_args()
dev = torch.device("cuda:0")
from rl4co_slap_amd import _native  # noqa: E402
from rl4co_slap_amd.rollout import engine  # noqa: E402

_native.load()


class _Loop:
    """A drop-in decode loop (ConstructivePolicy + env, stub decoder, certified greedy) as
    an object with run_eager(), for the fused decode + env step kernels' counters."""

    def __init__(self, env, td, logits, name):
        from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder
        from rl4co_slap_amd.td import TensorDict

        self.env, self.td, self.TD = env, td, TensorDict
        self.pol = ConstructivePolicy(None, LogitsDecoder(lambda t: logits), env_name=name,
                                      tanh_clipping=10.0)

    def run_eager(self):
        b = next(iter(self.td.values())).shape[0]
        t = self.env.reset(self.TD(dict(self.td), [b]))
        self.pol(t, self.env, phase="test", decode_type="greedy")


if args.kernel == "dropin_cvrp":
    from rl4co_slap_amd.envs import CVRPEnv

    torch.manual_seed(1234)
    la = torch.rand(32768, 101, 2)
    td = {"depot": la[:, 0].contiguous().to(dev), "locs": la[:, 1:].contiguous().to(dev),
          "demand": (((torch.rand(32768, 100) * 9).int() + 1).float() / 50.0).to(dev)}
    ep = _Loop(CVRPEnv(generator_params=dict(num_loc=100), device=dev), td,
               torch.randn(32768, 101).to(dev), "cvrp")
elif args.kernel == "dropin_slap":
    import numpy as np

    from rl4co_slap_amd.envs import SLAPEnv
    from rl4co_slap_amd.envs.slap import SLAPGenerator

    torch.manual_seed(1234)
    np.random.seed(1234)
    td = dict(SLAPGenerator(materialize_dist_mat=False)(65536).to(dev).items())
    ep = _Loop(SLAPEnv(device=dev), td, torch.randn(65536, 100).to(dev), "slap")
elif args.kernel.startswith("tsp"):
    torch.manual_seed(1234)
    locs = torch.rand(65536, 100, 2)
    torch.manual_seed(4321)
    acts = torch.rand(65536, 100).argsort(1)
    if args.kernel == "tsp_fused_teacher":
        ep = engine.TSPFusedEpisode(locs.to(dev), acts.to(dev))
        if args.cycle > 1:
            eps = [ep] + [engine.TSPFusedEpisode(torch.rand(65536, 100, 2, device=dev),
                                                 torch.rand(65536, 100, device=dev).argsort(1))
                          for _ in range(args.cycle - 1)]
    elif args.kernel == "tsp_fused_nearest":
        ep = engine.TSPFusedEpisode(locs.to(dev), None, policy="nearest")
    elif args.kernel == "tsp_stepwise_chunked":
        ep = engine.TSPStepwiseEpisode(locs.to(dev), acts.to(dev), chunk=10)
    else:
        ep = engine.TSPStepwiseEpisode(locs.to(dev), acts.to(dev))
elif args.kernel.startswith("cvrp"):
    torch.manual_seed(1234)
    locs_all = torch.rand(32768, 101, 2)
    demand = ((torch.rand(32768, 100) * 9).int() + 1).float() / 50.0
    td = {"depot": locs_all[:, 0].contiguous().to(dev),
          "locs": locs_all[:, 1:].contiguous().to(dev), "demand": demand.to(dev)}
    if args.kernel == "cvrp_fused_nearest":
        ep = engine.CVRPFusedEpisode(td)
    else:  # cvrp_stepwise[_pair]: the graph-chunked reference loop (replay = one episode);
        # _pair: the policy and co_cvrp_step as two launches (the env step kernel alone)
        ep = engine.CVRPStepwiseEpisode(td, fused_policy=not args.kernel.endswith("_pair")).capture()
        ep.run_eager = ep.replay
elif args.kernel == "pomo_tsp100":
    from rl4co_slap_amd.rollout.pomo import POMOEpisode

    torch.manual_seed(1234)
    locs = torch.rand(1024, 100, 2).to(dev)
    g = torch.Generator(device=dev).manual_seed(99)
    logits = torch.randn((99, 102400, 100), generator=g, device=dev)
    ep = POMOEpisode(locs, logits, tanh_clipping=10.0)
else:
    import numpy as np

    from rl4co_slap_amd.envs.slap import SLAPGenerator

    torch.manual_seed(1234)
    np.random.seed(1234)
    b = 65536 if args.kernel.endswith("b65536") else 16384
    td = SLAPGenerator(materialize_dist_mat=False)(b).to(dev)
    if args.kernel.startswith("slap_stepwise"):  # slap_stepwise_{closest,teacher}[_b65536]
        pol = "closest" if ("closest" in args.kernel or "chunked" in args.kernel) else "teacher"
        acts = None
        if pol == "teacher":
            torch.manual_seed(4321)
            acts = (torch.rand(b, 99).argsort(1)[:, :20] + 1).to(dev)
        # slap_stepwise_chunked_b65536: the closest policy, 10 steps per co_slap_closest_steps
        ep = engine.SLAPStepwiseEpisode(td, acts, policy=pol,
                                        chunk=10 if "chunked" in args.kernel else 1)
    elif args.kernel.startswith("slap_fused_random"):
        torch.manual_seed(4321)
        acts = (torch.rand(b, 99).argsort(1)[:, :20] + 1).to(dev)
        ep = engine.SLAPFusedEpisode(td, acts, policy="teacher")
    else:
        ep = engine.SLAPFusedEpisode(td, None, policy="closest")
        if args.cycle > 1:
            eps = [ep] + [engine.SLAPFusedEpisode(SLAPGenerator(materialize_dist_mat=False)(b).to(dev),
                                                  None, policy="closest")
                          for _ in range(args.cycle - 1)]
if "eps" not in globals():
    eps = [ep]
for j in range(args.k * len(eps)):
    eps[j % len(eps)].run_eager()
torch.cuda.synchronize()
print("ok", args.kernel)
