"""Golden fixtures for the hot path, produced by the oracle -- the CPU
restatement of the reference's env / decode / POMO code (``oracle/``).  The reference
itself may not be executed here, so these vectors pin the HIP path and
guard the oracle against drift; they are data only (inputs and expected outputs).

    python tests/golden/make_golden.py          # rewrite the .npz files
    build_all()                                  # the same dicts, for the tests

Per-step masks are stored bit-packed along the last axis (``np.packbits``).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import decoding as odec  # noqa: E402
from oracle.envs import (CVRPOracle, SLAPOracle, TSPOracle, cvrp_nearest_action,  # noqa: E402
                         slap_closest_free_action, tsp_nearest_action)
from oracle.rollout import constructive_forward, pomo_loss  # noqa: E402
from oracle.td import TD  # noqa: E402


def _pack(masks):  # [T, B, n] bool -> packed uint8
    return np.packbits(masks.numpy().astype(np.uint8), axis=-1)


def _episode(env, td, policy, keys=()):
    """Step until every instance is done; record each step's mask (and `keys`)."""
    acts, masks, rec = [], [], {k: [] for k in keys}
    while not td["done"].all():
        a = policy(td)
        acts.append(a.clone())
        td["action"] = a
        td = env.step(td)["next"]
        masks.append(td["action_mask"].clone())
        for k in keys:
            rec[k].append(td[k].clone().reshape(td[k].shape[0]))
    acts = torch.stack(acts, 1)
    reward = env.get_reward(td, acts)
    return acts, torch.stack(masks), {k: torch.stack(v) for k, v in rec.items()}, reward, td


def tsp(b, n, policy):
    env = TSPOracle(num_loc=n, seed=1234)
    td = env.reset(batch_size=[b])
    locs = td["locs"].clone()
    if policy == "teacher":
        g = torch.Generator().manual_seed(4321)
        perm = torch.rand(b, n, generator=g).argsort(1)
        it = iter(range(n))
        pol = lambda t: perm[:, next(it)]  # noqa: E731
    else:
        pol = tsp_nearest_action
    acts, masks, rec, reward, td = _episode(env, td, pol, keys=("first_node", "done"))
    return {"locs": locs.numpy(), "actions": acts.numpy(), "masks": _pack(masks),
            "first_node": rec["first_node"].numpy(), "done": rec["done"].numpy(),
            "reward": reward.numpy()}


def cvrp(b, n):
    env = CVRPOracle(num_loc=n, seed=1234)
    gen = env.generate([b])
    td = env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    acts, masks, rec, reward, td = _episode(env, td, cvrp_nearest_action,
                                            keys=("used_capacity", "done"))
    return {"depot": gen["depot"].numpy(), "locs": gen["locs"].numpy(),
            "demand": gen["demand"].numpy(), "vehicle_capacity": np.float32(env.vehicle_capacity),
            "actions": acts.numpy(), "masks": _pack(masks),
            "used_capacity": rec["used_capacity"].numpy(), "done": rec["done"].numpy(),
            "visited": td["visited"].numpy(), "reward": reward.numpy()}


def slap(b, policy):
    env = SLAPOracle(seed=1234)
    np.random.seed(1234)
    gen = env.generate([b])
    td = env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    if policy == "closest":
        pol = slap_closest_free_action
    else:  # random free location, seeded (the reference's random-feasible bench policy)
        g = torch.Generator().manual_seed(99)
        pol = lambda t: torch.multinomial(t["action_mask"].float(), 1, generator=g).squeeze(-1)  # noqa: E731
    acts, masks, _, reward, td = _episode(env, td, pol)
    return {"freq": gen["freq"].numpy(), "locs": gen["locs"].numpy(),
            "picklist": gen["picklist"].numpy(), "depot_loc_dist": gen["depot_loc_dist"].numpy(),
            "assignment0": gen["assignment"].numpy(), "actions": acts.numpy(),
            "masks": _pack(masks), "assignment": td["assignment"].numpy(),
            "reward": reward.numpy()}


def decode(b, n, clip):
    g = torch.Generator().manual_seed(7 + int(clip))
    logits = torch.randn(b, n, generator=g) * 3
    mask = torch.rand(b, n, generator=g) > 0.4
    mask[torch.arange(b), torch.randint(0, n, (b,), generator=g)] = True
    logp = odec.process_logits(logits, mask, temperature=1.0, tanh_clipping=clip)
    act = logp.argmax(-1)
    out = {"logits": logits.numpy(), "mask": mask.numpy(), "clip": np.float32(clip),
           "action": act.numpy(), "logp_sel": logp.gather(1, act[:, None]).squeeze(1).numpy()}
    if clip > 0:  # the oracle's post-clip logits (decoding.py:172-173, torch.tanh on the CPU)
        out["logits_clipped"] = (torch.tanh(logits) * clip).numpy()
    return out


def pomo(b, n):
    env = TSPOracle(num_loc=n, seed=n)
    td = env.reset(batch_size=[b])
    locs = td["locs"].clone()
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(n - 1, n * b, n, generator=g) * 2
    step = {"t": 0}

    def logits_fn(_):
        lg = logits[step["t"]]
        step["t"] += 1
        return lg.clone()

    out = constructive_forward(td, env, logits_fn, decode_type="multistart_greedy",
                               tanh_clipping=10.0)
    ref = pomo_loss(out["reward"], out["log_likelihood"], n)
    return {"locs": locs.numpy(), "logits": logits.numpy(), "actions": out["actions"].numpy(),
            "reward": out["reward"].numpy(), "log_likelihood": out["log_likelihood"].numpy(),
            "bl_val": ref["bl_val"].squeeze(1).numpy(), "max_reward": ref["max_reward"].numpy(),
            "loss": np.float32(ref["loss"]),
            # the post-clip logits the oracle decoded (torch.tanh on the CPU, x 10)
            "logits_clipped": (torch.tanh(logits) * 10.0).numpy()}


def build_all():
    prev = torch.get_num_threads()
    torch.set_num_threads(1)  # one summation order for the float fixtures
    try:
        return _build()
    finally:
        torch.set_num_threads(prev)


def _build():
    return {
        "tsp20_b128_teacher": tsp(128, 20, "teacher"),
        "tsp20_b128_nearest": tsp(128, 20, "nearest"),
        "tsp100_b64_teacher": tsp(64, 100, "teacher"),
        "tsp100_b64_nearest": tsp(64, 100, "nearest"),
        "cvrp20_b64_nearest": cvrp(64, 20),
        "cvrp100_b64_nearest": cvrp(64, 100),
        "slap_b32_closest": slap(32, "closest"),
        "slap_b32_random": slap(32, "random"),
        "decode_b256_n100_noclip": decode(256, 100, 0.0),
        "decode_b256_n100_clip10": decode(256, 100, 10.0),
        "pomo_tsp20_b8": pomo(8, 20),
    }


if __name__ == "__main__":
    for name, arrays in build_all().items():
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **arrays)
        print(f"{name}: {os.path.getsize(path) / 1024:.1f} KiB")
