"""Diagnostic: GPU time of one co_cvrp_decode_step launch (certified greedy, no clip -- the
drop-in bench's settings) at B = 32,768, N = 100 on a mid-episode state, HIP events over
100 launches; inputs cycled over 4 copies so the launch reads HBM.  CO_LIB picks a
variant library (tools/build_variants.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rl4co_slap_amd import _native  # noqa: E402

if os.environ.get("CO_LIB"):
    _native.LIB_PATH = os.environ["CO_LIB"]
_native.load()
dev = torch.device("cuda:0")
b, n = 32768, 100
g = torch.Generator().manual_seed(5)
sets = []
for _ in range(4):
    vis = (torch.rand(b, n + 1, generator=g) < 0.5).to(torch.uint8)
    vis[:, 0] = 1
    st = {"logits": torch.randn(b, n + 1, generator=g), "mask": (vis == 0),
          "demand": ((torch.rand(b, n, generator=g) * 9).int() + 1).float() / 50.0,
          "used": torch.rand(b, 1, generator=g) * 0.5, "cap": torch.ones(b, 1), "vis": vis}
    st["mask"][:, 0] = True
    sets.append({k: v.to(dev) for k, v in st.items()})
outs = dict(act=torch.empty(b, dtype=torch.int64, device=dev), lp=torch.empty(b, device=dev),
            used=torch.empty(b, 1, device=dev), vis=torch.empty(b, n + 1, dtype=torch.uint8, device=dev),
            cur=torch.empty(b, 1, dtype=torch.int64, device=dev), done=torch.empty(b, dtype=torch.bool, device=dev),
            rew=torch.empty(b, dtype=torch.bool, device=dev), mask=torch.empty(b, n + 1, dtype=torch.bool, device=dev))
status = torch.zeros(1, dtype=torch.int32, device=dev)
sh = torch.cuda.current_stream(dev).cuda_stream
launches = [_native.bind("co_cvrp_decode_step", b, n, s["logits"].data_ptr(), n + 1, s["mask"].data_ptr(),
                         0.0, 1.0, _native.DECODE_CERTIFIED, None, outs["act"].data_ptr(),
                         outs["lp"].data_ptr(), 0, 0, s["demand"].data_ptr(), s["used"].data_ptr(),
                         outs["used"].data_ptr(), s["cap"].data_ptr(), s["vis"].data_ptr(),
                         outs["vis"].data_ptr(), outs["cur"].data_ptr(), outs["done"].data_ptr(),
                         outs["rew"].data_ptr(), outs["mask"].data_ptr(), None, status.data_ptr())
            for s in sets]
it = [0]


def run():
    launches[it[0] % 4](sh)
    it[0] += 1


_, ev = bench.timed(run, 100, 8, 1, dev)
print(f"co_cvrp_decode_step B={b} N={n}: {ev / 100 * 1e6:.2f} us per launch")
