"""Time co_cvrp_reward alone (diagnostic): the stepwise CVRP-100 episode's step-major
actions at B=32768, 30 launches, HIP events; with and without the validity check.
CO_LIB selects a variant library (tools/build_variants.sh, e.g. -DCO_CVRP_RCUT=1)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rl4co_slap_amd import _native as nat  # noqa: E402

if os.environ.get("CO_LIB"):
    nat.LIB_PATH = os.environ["CO_LIB"]
nat.load()
from rl4co_slap_amd.rollout.engine import CVRPStepwiseEpisode  # noqa: E402

dev = torch.device("cuda:0")
b, n = 32768, 100
torch.manual_seed(1234)
la = torch.rand(b, n + 1, 2)
dm = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
td = {"depot": la[:, 0].contiguous().to(dev), "locs": la[:, 1:].contiguous().to(dev),
      "demand": dm.to(dev)}
ep = CVRPStepwiseEpisode(td).capture()
ep.replay()
torch.cuda.synchronize(dev)
T = ep.T
acts = ep.acts[:T]
s = torch.cuda.current_stream(dev).cuda_stream
out = {"lib": os.environ.get("CO_LIB", "base"), "T": T}
for check in (1, 0):
    f = nat.bind("co_cvrp_reward", b, n, T, nat.ptr(ep.locs), nat.ptr(acts), 1, b,
                 nat.ptr(ep.demand), nat.ptr(ep.vcap_t), check, nat.ptr(ep.reward),
                 nat.ptr(ep.status))
    for _ in range(3):
        f(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(30):
        f(s)
    e1.record()
    torch.cuda.synchronize(dev)
    out[f"check{check}_us"] = e0.elapsed_time(e1) * 1e3 / 30
# the drop-in loop's layout: row-major [B, T] actions (cvrp_reward_kernel, wave per instance)
ref = ep.reward.clone()
acts_rm = acts.t().contiguous()
rew_rm = torch.empty_like(ep.reward)
f = nat.bind("co_cvrp_reward", b, n, T, nat.ptr(ep.locs), nat.ptr(acts_rm), T, 1,
             nat.ptr(ep.demand), nat.ptr(ep.vcap_t), 1, nat.ptr(rew_rm), nat.ptr(ep.status))
for _ in range(3):
    f(s)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(30):
    f(s)
e1.record()
torch.cuda.synchronize(dev)
out["rowmajor_check1_us"] = e0.elapsed_time(e1) * 1e3 / 30
out["rowmajor_close"] = bool(torch.allclose(rew_rm, ref, rtol=1e-6, atol=0)) and int(ep.status.item()) == 0
print(json.dumps(out))
if os.environ.get("CO_TIMING"):  # a -DCO_CVRPR_TIMING build: per-workgroup phase clocks
    f = nat.bind("co_cvrp_reward", b, n, T, nat.ptr(ep.locs), nat.ptr(acts), 1, b,
                 nat.ptr(ep.demand), nat.ptr(ep.vcap_t), 1, nat.ptr(ep.reward),
                 nat.ptr(ep.status))
    f(s)
    f(s)
    torch.cuda.synchronize(dev)
    tm = ep.reward.view(-1, 64)[:, :5].cpu().double()
    names = ["start", "staged", "scanner_done", "walkers_done", "end"]
    print(json.dumps({nm: [round(float(tm[:, i].quantile(p)), 0) for p in (0.1, 0.5, 0.9, 1.0)]
                      for i, nm in enumerate(names)}))
