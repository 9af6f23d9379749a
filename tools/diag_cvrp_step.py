"""Time co_cvrp_step alone (diagnostic): B=32768 CVRP-100 state after a few nearest-policy
steps, 50 launches on fixed inputs, HIP events.  CO_LIB selects a variant library
(tools/build_variants.sh, e.g. the CO_CVRP_CUT timing cuts)."""
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

dev = torch.device("cuda:0")
b, n = 32768, 100
torch.manual_seed(1)
la = torch.rand(b, n + 1, 2)
dm = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
env = CVRPEnv(generator_params={"num_loc": n}, device=dev)
from rl4co_slap_amd.td import TensorDict  # noqa: E402

td = env.reset(TensorDict({"depot": la[:, 0].to(dev), "locs": la[:, 1:].contiguous().to(dev),
                           "demand": dm.to(dev)}, batch_size=[b]))
for t in range(5):
    act = torch.full((b,), 1 + t, dtype=torch.int64, device=dev)
    td.set("action", act)
    td = env.step(td)["next"]
action = torch.full((b,), 7, dtype=torch.int64, device=dev)
used_out = torch.empty_like(td["used_capacity"])
vis_out = torch.empty_like(td["visited"])
mask = torch.empty_like(td["action_mask"])
cur = torch.empty((b, 1), dtype=torch.int64, device=dev)
done = torch.empty(b, dtype=torch.bool, device=dev)
rew = torch.empty(b, dtype=torch.bool, device=dev)
status = torch.zeros(1, dtype=torch.int32, device=dev)
f = nat.bind("co_cvrp_step", b, n, nat.ptr(action), nat.ptr(td["demand"]),
             nat.ptr(td["used_capacity"]), nat.ptr(used_out), nat.ptr(td["vehicle_capacity"]),
             nat.ptr(td["visited"]), nat.ptr(vis_out), nat.ptr(cur), nat.ptr(done), nat.ptr(rew),
             nat.ptr(mask), nat.ptr(status), None)
s = torch.cuda.current_stream(dev).cuda_stream
for _ in range(5):
    f(s)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    f(s)
e1.record()
torch.cuda.synchronize(dev)
us = e0.elapsed_time(e1) * 1e3 / 50
print(json.dumps({"lib": os.environ.get("CO_LIB", "base"), "step_us": us,
                  "GBps": b * (7 * n + 33) / us / 1e3}))
