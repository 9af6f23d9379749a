"""Host-side cost of the drop-in decode loop (diagnostic): cProfile of
ConstructivePolicy.forward on TSPEnv at B=64 (device work negligible), top entries."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rl4co_slap_amd.envs import TSPEnv  # noqa: E402
from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder  # noqa: E402
from rl4co_slap_amd.td import TensorDict  # noqa: E402

dev = torch.device(os.environ.get("CO_DEV", "cuda:0"))  # CO_DEV=cpu: the host build
b, n = 64, 100
locs = torch.rand(b, n, 2, device=dev)
logits = torch.randn(b, n, device=dev)
env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
pol = ConstructivePolicy(None, LogitsDecoder(lambda td: logits), env_name="tsp")


def run(k):
    for _ in range(k):
        pol(env.reset(TensorDict({"locs": locs}, [b])), env, phase="test", decode_type="greedy")
    if dev.type == "cuda":
        torch.cuda.synchronize()


run(3)
pr = cProfile.Profile()
pr.enable()
run(10)
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
