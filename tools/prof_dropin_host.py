"""Host-side cost of the drop-in decode loop (diagnostic): cProfile of
ConstructivePolicy.forward on TSPEnv / CVRPEnv / SLAPEnv (CO_ENV) at B=64 (device work
negligible), top entries, then the plain wall time per episode."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rl4co_slap_amd.envs import CVRPEnv, SLAPEnv, TSPEnv  # noqa: E402
from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder  # noqa: E402
from rl4co_slap_amd.td import TensorDict  # noqa: E402

dev = torch.device(os.environ.get("CO_DEV", "cuda:0"))  # CO_DEV=cpu: the host build
name = os.environ.get("CO_ENV", "tsp")
b, n = 64, 100
if name == "tsp":
    data = {"locs": torch.rand(b, n, 2, device=dev)}
    env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
    na = n
elif name == "cvrp":
    la = torch.rand(b, n + 1, 2, device=dev)
    data = {"depot": la[:, 0].contiguous(), "locs": la[:, 1:].contiguous(),
            "demand": ((torch.rand(b, n, device=dev) * 9).int() + 1).float() / 50.0}
    env = CVRPEnv(generator_params=dict(num_loc=n), device=dev)
    na = n + 1
else:
    from rl4co_slap_amd.envs.slap import SLAPGenerator

    data = dict(SLAPGenerator(materialize_dist_mat=False)(b).to(dev).items())
    env = SLAPEnv(device=dev)
    na = 100
logits = torch.randn(b, na, device=dev)
pol = ConstructivePolicy(None, LogitsDecoder(lambda td: logits), env_name=name)


def run(k):
    for _ in range(k):
        pol(env.reset(TensorDict(dict(data), [b])), env, phase="test", decode_type="greedy")
    if dev.type == "cuda":
        torch.cuda.synchronize()


run(3)
pr = cProfile.Profile()
pr.enable()
run(10)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
import time  # noqa: E402

t0 = time.perf_counter()
run(20)
print(name, "wall ms per episode", (time.perf_counter() - t0) / 20 * 1e3)
