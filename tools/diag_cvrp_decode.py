"""Time co_cvrp_decode_step alone (diagnostic, not part of the product): B = 32,768
CVRP-100 state after 5 steps, greedy certified decode (tanh clip 10) + env transition, 50
launches on fixed inputs, HIP events; bytes per row as the bench counts them.  CO_LIB selects
a variant library (tools/build_variants.sh)."""
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
from rl4co_slap_amd.envs import CVRPEnv  # noqa: E402
from rl4co_slap_amd.td import TensorDict  # noqa: E402

dev = torch.device("cuda:0")
b, n = int(os.environ.get("B", 32768)), int(os.environ.get("N", 100))
torch.manual_seed(1)
la = torch.rand(b, n + 1, 2)
dm = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
env = CVRPEnv(generator_params={"num_loc": n}, device=dev)
td = env.reset(TensorDict({"depot": la[:, 0].to(dev), "locs": la[:, 1:].contiguous().to(dev),
                           "demand": dm.to(dev)}, batch_size=[b]))
for t in range(5):
    td.set("action", torch.full((b,), 1 + t, dtype=torch.int64, device=dev))
    td = env.step(td)["next"]
LS = int(os.environ.get("LSTRIDE", n + 1))
logits = torch.randn(b, LS, device=dev)[:, : n + 1]
out = dict(act=torch.empty(b, dtype=torch.int64, device=dev), lp=torch.empty(b, device=dev),
           used=torch.empty_like(td["used_capacity"]), vis=torch.empty_like(td["visited"]),
           cur=torch.empty((b, 1), dtype=torch.int64, device=dev),
           done=torch.empty(b, dtype=torch.bool, device=dev),
           rew=torch.empty(b, dtype=torch.bool, device=dev),
           mask=torch.empty_like(td["action_mask"]))
status = torch.zeros(1, dtype=torch.int32, device=dev)
p = nat.ptr
f = nat.bind("co_cvrp_decode_step", b, n, p(logits), LS, p(td["action_mask"]), 10.0, 1.0,
             nat.DECODE_CERTIFIED, None, p(out["act"]), p(out["lp"]), 0, 0, p(td["demand"]),
             p(td["used_capacity"]), p(out["used"]), p(td["vehicle_capacity"]), p(td["visited"]),
             p(out["vis"]), p(out["cur"]), p(out["done"]), p(out["rew"]), p(out["mask"]), None,
             p(status))
s = torch.cuda.current_stream(dev).cuda_stream
for _ in range(5):
    f(s)
torch.cuda.synchronize(dev)
res = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        f(s)
    e1.record()
    torch.cuda.synchronize(dev)
    res.append(e0.elapsed_time(e1) * 1e3 / 50)
us = sorted(res)[2]
row = 4 * (n + 1) + (n + 1) + 4 * n + (n + 1) + 12 + 2 * (n + 1) + 4 + 8 + 2 + 8 + 4
print(json.dumps({"lib": os.environ.get("CO_LIB", "base"), "B": b, "lstride": LS, "decode_step_us": round(us, 3),
                  "bytes_per_row": row, "GBps": round(b * row / us / 1e3, 1),
                  "status": int(status.item())}))
