"""co_cvrp_step at B = 32,768, N = 100 with and without the not-done counter (diagnostic:
the cost of the counter's one-atomic-per-workgroup path), HIP events, alternating."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from rl4co_slap_amd import _native as nat  # noqa: E402

d = torch.device("cuda:0")
if os.environ.get("CO_LIB"):  # a variant library (tools/build_variants.sh)
    nat.LIB_PATH = os.environ["CO_LIB"]
nat.load()
b, n = 32768, 100
act = torch.randint(0, n + 1, (b,), device=d)
dem = torch.rand(b, n, device=d) * 0.1
used, used2 = torch.zeros(b, 1, device=d), torch.zeros(b, 1, device=d)
vcap = torch.ones(b, 1, device=d)
vis = torch.zeros(b, n + 1, dtype=torch.uint8, device=d)
cur = torch.empty(b, dtype=torch.int64, device=d)
done, rw = torch.empty(b, dtype=torch.bool, device=d), torch.empty(b, dtype=torch.bool, device=d)
m = torch.empty(b, n + 1, dtype=torch.bool, device=d)
st = torch.zeros(1, dtype=torch.int32, device=d)
nd = torch.zeros(1, dtype=torch.int32, device=d)
out = {}
for rep in range(3):
    for name, ndp in (("no_counter", None), ("counter", nat.ptr(nd))):
        f = nat.bind("co_cvrp_step", b, n, nat.ptr(act), nat.ptr(dem), nat.ptr(used), nat.ptr(used2),
                     nat.ptr(vcap), nat.ptr(vis), nat.ptr(vis), nat.ptr(cur), nat.ptr(done),
                     nat.ptr(rw), nat.ptr(m), nat.ptr(st), ndp)
        out.setdefault(name, []).append(round(bench.time_bound(f, d) * 1e6, 2))
print(out)
