"""The two builds of the C ABI against each other: the host library (CPU TensorDicts,
csrc/host) and the gfx950 library on identical inputs through the same env classes --
every step's state bit-equal, rewards within 1e-5, decode log-probabilities bit-equal
(both restate ATen's F.log_softmax), greedy actions equal."""
import numpy as np
import pytest
import torch

from rl4co_slap_amd import TensorDict
from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.envs import CVRPEnv, SLAPEnv, TSPEnv
from rl4co_slap_amd.utils.decoding import decode_step

pytestmark = pytest.mark.gpu


def _close(a, b):
    assert ((a - b).abs() <= 1e-5 * b.abs().clamp(min=1)).all()


@pytest.mark.parametrize("name,b,n", [("tsp", 200, 50), ("cvrp", 150, 30)])
def test_env_steps_host_equals_device(dev, name, b, n):
    nat.load_host()
    cls = TSPEnv if name == "tsp" else CVRPEnv
    env_h, env_d = cls(generator_params=dict(num_loc=n), device="cpu"), \
        cls(generator_params=dict(num_loc=n), device=dev)
    gen = env_h.generator(batch_size=[b])
    td_h = env_h.reset(TensorDict({k: v.clone() for k, v in gen.items()}, [b]))
    td_d = env_d.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()}, [b]))
    g = torch.Generator().manual_seed(n)
    acts = []
    while not td_h["done"].all():
        m = td_h["action_mask"]
        a = torch.where(m.any(1), (torch.rand(m.shape, generator=g) * m).argmax(1),
                        torch.zeros(b, dtype=torch.int64))
        acts.append(a)
        td_h["action"] = a
        td_d["action"] = a.to(dev)
        td_h = env_h.step(td_h)["next"]
        td_d = env_d.step(td_d)["next"]
        for k in td_h.keys():
            if k in ("locs", "demand", "depot", "capacity"):
                continue
            assert torch.equal(td_h[k], td_d[k].cpu()), k
    acts = torch.stack(acts, 1)
    _close(env_d.get_reward(td_d, acts.to(dev)).cpu(), env_h.get_reward(td_h, acts))


def test_slap_host_equals_device(dev):
    b = 64
    env_h, env_d = SLAPEnv(device="cpu"), SLAPEnv(device=dev)
    np.random.seed(3)
    gen = env_h.generator(batch_size=[b])
    td_h = env_h.reset(TensorDict({k: v.clone() for k, v in gen.items()}, [b]))
    td_d = env_d.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()}, [b]))
    g = torch.Generator().manual_seed(1)
    for _ in range(20):
        a = (torch.rand(td_h["action_mask"].shape, generator=g) * td_h["action_mask"]).argmax(1)
        td_h["action"], td_d["action"] = a, a.to(dev)
        td_h, td_d = env_h.step(td_h)["next"], env_d.step(td_d)["next"]
        for k in ("action_mask", "assignment", "i", "done", "to_choose"):
            assert torch.equal(td_h[k], td_d[k].cpu()), k
    _close(env_d.get_reward(td_d, None).cpu(), env_h.get_reward(td_h, None))


@pytest.mark.parametrize("n", [10, 37, 100, 200])
@pytest.mark.parametrize("clip,temp", [(0.0, 1.0), (10.0, 1.0), (10.0, 0.8)])
def test_decode_host_equals_device(dev, n, clip, temp):
    b = 300
    g = torch.Generator().manual_seed(n)
    x = torch.randn(b, n, generator=g) * 4
    mask = torch.rand(b, n, generator=g) > 0.25
    mask[:, -1] = True
    ah, lh, fh = decode_step(x, mask, "greedy", temp, clip, return_full=True)
    ad, ld, fd = decode_step(x.to(dev), mask.to(dev), "greedy", temp, clip, return_full=True)
    assert torch.equal(ah, ad.cpu())
    assert torch.equal(lh, ld.cpu())
    assert torch.equal(fh, fd.cpu())
