"""The committed golden fixtures (tests/golden/*.npz, made by the oracle) through the
HIP path: stepwise env API every step, fused episodes, the decode step and the POMO
episode.  Masks / indices / bool state bit-exact; rewards 1e-5 relative."""
import os

import numpy as np
import pytest
import torch

from rl4co_slap_amd import TensorDict
from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.envs import CVRPEnv, SLAPEnv, TSPEnv
from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode, SLAPFusedEpisode, TSPFusedEpisode
from rl4co_slap_amd.rollout.pomo import POMOEpisode
from rl4co_slap_amd.utils.decoding import decode_step

pytestmark = pytest.mark.gpu
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    f = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    return {k: f[k] for k in f.files}


def masks(f, n):
    return np.unpackbits(f["masks"], axis=-1, count=n).astype(bool)


def close(got, want, rel=1e-5):
    got, want = np.asarray(got), np.asarray(want)
    assert (np.abs(got - want) <= rel * np.maximum(1.0, np.abs(want))).all()


@pytest.mark.parametrize("name", ["tsp20_b128_teacher", "tsp20_b128_nearest",
                                  "tsp100_b64_teacher", "tsp100_b64_nearest"])
def test_tsp_golden(dev, name):
    f = load(name)
    b, n = f["actions"].shape
    m = masks(f, n)
    env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
    td = env.reset(TensorDict({"locs": torch.from_numpy(f["locs"]).to(dev)}, [b]))
    acts = torch.from_numpy(f["actions"]).to(dev)
    for t in range(n):
        td["action"] = acts[:, t].contiguous()
        td = env.step(td)["next"]
        assert np.array_equal(td["action_mask"].cpu().numpy(), m[t]), t
        assert np.array_equal(td["first_node"].cpu().numpy(), f["first_node"][t])
        assert np.array_equal(td["done"].cpu().numpy(), f["done"][t])
    close(env.get_reward(td, acts).cpu(), f["reward"])
    policy = "nearest" if name.endswith("nearest") else "teacher"
    ep = TSPFusedEpisode(torch.from_numpy(f["locs"]).to(dev),
                         acts if policy == "teacher" else None, policy=policy)
    ep.run_eager()
    torch.cuda.synchronize()
    st = ep.final_state()
    assert int(ep.status.item()) == 0
    assert np.array_equal(st["actions"].cpu().numpy(), f["actions"])
    assert np.array_equal(st["action_mask"].cpu().numpy(), m[-1])
    close(st["reward"].cpu(), f["reward"])


@pytest.mark.parametrize("name", ["cvrp20_b64_nearest", "cvrp100_b64_nearest"])
def test_cvrp_golden(dev, name):
    f = load(name)
    b, T = f["actions"].shape
    n = f["locs"].shape[1]
    m = masks(f, n + 1)
    gen = {k: torch.from_numpy(f[k]).to(dev) for k in ("depot", "locs", "demand")}
    gen["capacity"] = torch.ones(b, 1, device=dev)
    env = CVRPEnv(generator_params=dict(num_loc=n), device=dev)
    td = env.reset(TensorDict(dict(gen), [b]))
    acts = torch.from_numpy(f["actions"]).to(dev)
    for t in range(T):
        td["action"] = acts[:, t].contiguous()
        td = env.step(td)["next"]
        assert np.array_equal(td["action_mask"].cpu().numpy(), m[t]), t
        assert np.array_equal(td["used_capacity"].cpu().numpy().reshape(-1), f["used_capacity"][t])
        assert np.array_equal(td["done"].cpu().numpy().reshape(-1), f["done"][t])
    close(env.get_reward(td, acts).cpu(), f["reward"])
    ep = CVRPFusedEpisode(gen, vehicle_capacity=float(f["vehicle_capacity"]))
    ep.run_eager()
    torch.cuda.synchronize()
    st = ep.final_state()
    assert np.array_equal(st["actions"].cpu().numpy(), f["actions"])
    assert np.array_equal(st["visited"].cpu().numpy(), f["visited"])
    assert np.array_equal(st["action_mask"].cpu().numpy(), m[-1])
    close(st["reward"].cpu(), f["reward"])


@pytest.mark.parametrize("name", ["slap_b32_closest", "slap_b32_random"])
def test_slap_golden(dev, name):
    f = load(name)
    b, P = f["actions"].shape
    L = f["locs"].shape[1]
    m = masks(f, L)
    gen = {"freq": f["freq"], "locs": f["locs"], "picklist": f["picklist"],
           "depot_loc_dist": f["depot_loc_dist"], "assignment": f["assignment0"]}
    gen = {k: torch.from_numpy(v).to(dev) for k, v in gen.items()}
    env = SLAPEnv(device=dev)
    td = env.reset(TensorDict({k: v.clone() for k, v in gen.items()}, [b]))
    acts = torch.from_numpy(f["actions"]).to(dev)
    for t in range(P):
        td["action"] = acts[:, t].contiguous()
        td = env.step(td)["next"]
        assert np.array_equal(td["action_mask"].cpu().numpy(), m[t]), t
    assert np.array_equal(td["assignment"].cpu().numpy(), f["assignment"])
    close(env.get_reward(td, acts).cpu(), f["reward"])
    closest = name.endswith("closest")
    ep = SLAPFusedEpisode(gen, None if closest else acts, policy="closest" if closest else "teacher")
    ep.run_eager()
    torch.cuda.synchronize()
    st = ep.final_state()
    assert np.array_equal(st["actions"].cpu().numpy(), f["actions"])
    assert np.array_equal(st["assignment"].cpu().numpy(), f["assignment"])
    assert np.array_equal(st["action_mask"].cpu().numpy(), m[-1])
    close(st["reward"].cpu(), f["reward"])


@pytest.mark.parametrize("name", ["decode_b256_n100_noclip", "decode_b256_n100_clip10"])
def test_decode_golden(dev, name):
    """Greedy decode of the fixture rows: bit-exact actions and log-probabilities.  The
    clip-10 fixture is decoded from the oracle's post-clip logits (torch.tanh is MKL's on
    the CPU; the kernel's own tanh is tested in test_gpu_decode_exact.py)."""
    f = load(name)
    clip = float(f["clip"])
    logits = torch.from_numpy(f["logits_clipped"] if clip > 0 else f["logits"]).to(dev)
    mask = torch.from_numpy(f["mask"]).to(dev)
    sel, logp, _ = decode_step(logits, mask, "greedy", 1.0, 0.0)
    assert np.array_equal(sel.cpu().numpy(), f["action"])
    assert np.array_equal(logp.cpu().numpy().view(np.uint32), f["logp_sel"].view(np.uint32))


def test_pomo_golden(dev):
    """The POMO TSP-20 fixture episode from the oracle's post-clip logits: actions and
    the per-instance baseline / max reward / loss unconditionally."""
    f = load("pomo_tsp20_b8")
    locs = torch.from_numpy(f["locs"]).to(dev)
    ep = POMOEpisode(locs, torch.from_numpy(f["logits_clipped"]).to(dev), tanh_clipping=0.0)
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) == 0
    st = ep.final_state()
    assert np.array_equal(st["actions"].cpu().numpy(), f["actions"])
    close(st["reward"].cpu().numpy(), f["reward"])
    close(st["log_likelihood"].cpu().numpy(), f["log_likelihood"], rel=1e-5)
    close(st["bl_val"].cpu().numpy(), f["bl_val"])
    close(st["max_reward"].cpu().numpy(), f["max_reward"])
    s = f["actions"].shape[0] // f["locs"].shape[0]
    loss = -st["loss_terms"].cpu().sum().item() / f["actions"].shape[0]
    assert abs(loss - float(f["loss"])) <= 1e-5 * max(1.0, abs(float(f["loss"]))) + 1e-6, s
