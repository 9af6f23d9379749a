"""Host-side cost (us per call) of the pieces of the drop-in decode step at B = 64, where
the device work is negligible (diagnostic, not part of the product)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rl4co_slap_amd import _native as nat  # noqa: E402
from rl4co_slap_amd.envs import TSPEnv  # noqa: E402
from rl4co_slap_amd.td import TensorDict  # noqa: E402

dev = torch.device("cuda:0")
b, n = 64, 100
nat.load()


def us(f, reps=2000):
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    t = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    return round(t, 3)


out = {}
out["torch.empty"] = us(lambda: torch.empty((b, n), dtype=torch.bool, device=dev))
buf = torch.empty(b * n + 8 * b * 4, dtype=torch.uint8, device=dev)
out["view_slice"] = us(lambda: buf[: b * n].view(b, n))
env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
out["pool.empty"] = us(lambda: env._out((b, n), torch.bool, dev, 0))
out["stream_of"] = us(lambda: nat.stream_of(buf))
td = env.reset(TensorDict({"locs": torch.rand(b, n, 2, device=dev)}, [b]))
out["td[key]"] = us(lambda: td["action_mask"])
out["td.update6"] = us(lambda: td.update({"a": buf, "b": buf, "c": buf, "d": buf, "e": buf,
                                          "f": buf}))
logits = torch.randn(b, n, device=dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
mask = td["action_mask"]
i = td["i"]
act = torch.empty(b, dtype=torch.int64, device=dev)
lp = torch.empty(b, device=dev)
mo = torch.empty((b, n), dtype=torch.bool, device=dev)
io = torch.empty((b, 1), dtype=torch.int64, device=dev)
fo = torch.empty(b, dtype=torch.int64, device=dev)
dn = torch.empty(b, dtype=torch.bool, device=dev)
rw = torch.empty(b, dtype=torch.bool, device=dev)
s = nat.stream_of(mask)
args = (b, n, logits.data_ptr(), n, mask.data_ptr(), 10.0, 1.0, nat.DECODE_CERTIFIED, None,
        act.data_ptr(), lp.data_ptr(), 0, 0, mo.data_ptr(), i.data_ptr(), io.data_ptr(), None,
        fo.data_ptr(), 1, dn.data_ptr(), rw.data_ptr(), None, st.data_ptr(), s)
out["nat.call(co_tsp_decode_step)"] = us(lambda: nat.call("co_tsp_decode_step", *args))
out["data_ptr"] = us(lambda: logits.data_ptr())


def one_episode_step():
    t = env.reset(TensorDict({"locs": td["locs"]}, [b]))
    return env.decode_and_step(t, logits, nat.DECODE_CERTIFIED, 1.0, 10.0, None, 0, 0, st)


out["reset+decode_and_step"] = us(one_episode_step, 500)
out["reset"] = us(lambda: env.reset(TensorDict({"locs": td["locs"]}, [b])), 500)
print(out)
