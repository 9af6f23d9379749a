"""Time co_episode_stack alone (diagnostic, not part of the product): the drop-in loop's
epilogue on step-major action / log-probability rows, HIP events over back-to-back
launches on fixed inputs.  Shapes: SLAP B = 16,384 / 65,536 with T = 20, CVRP-100 B = 32,768
with T = 199.  CO_LIB selects a variant library (tools/build_variants.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rl4co_slap_amd import _native as nat  # noqa: E402

if os.environ.get("CO_LIB"):
    nat.LIB_PATH = os.environ["CO_LIB"]
nat.load()
dev = torch.device("cuda:0")
out = {"lib": os.environ.get("CO_LIB", "base")}
for b, t in ((16384, 20), (65536, 20), (32768, 199)):
    act = torch.randint(0, 100, (t, b), dtype=torch.int64, device=dev)
    lp = -torch.rand(t, b, device=dev)
    acts = torch.empty(b, t, dtype=torch.int64, device=dev)
    lps = torch.empty(b, t, device=dev)
    ll = torch.empty(b, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    p = nat.ptr
    f = nat.bind("co_episode_stack", b, t, p(act), b, p(lp), b, p(acts), p(lps), p(ll), p(st))
    s = torch.cuda.current_stream(dev).cuda_stream
    _, ev = bench.timed(lambda: f(s), 50, 5, 1, dev)
    us = ev / 50 * 1e6
    ok = torch.equal(acts, act.t()) and torch.equal(lps, lp.t())
    out[f"b{b}_t{t}_us"] = round(us, 2)
    out[f"b{b}_t{t}_TBps"] = round(2 * 12 * b * t / us / 1e6, 2)
    out[f"b{b}_t{t}_ok"] = ok
print(json.dumps(out))
