"""BASELINE configs 3 and 4 at their full batch sizes on the device (CVRP-100 B=32,768;
SLAP B=16,384 and 65,536): the fused and stepwise engines against each other and
against size-independent properties of the reference semantics, plus the oracle on a
512-instance slice of the same batch (the oracle is too slow to mirror the whole):

* CVRP: every customer visited exactly once, the batch-wide episode length T the
  reference loop runs (``constructive/base.py:230``; ``while not td["done"].all()``)
  equal between the fused and the stepwise engine, trailing depot padding after each
  instance is done, capacity respected; slice actions / rewards = the oracle's.
* SLAP: i = P, the assignment equals the step actions (product t <- step t's location),
  P distinct non-depot locations, the mask clears exactly the depot and those P
  (``slap/env.py:38-93``, the per-batch loop ``:61-62``); slice state / rewards = oracle.
"""
import numpy as np
import pytest
import torch

from oracle.rollout import rollout as ref_rollout
from oracle.td import TD

pytestmark = pytest.mark.gpu

SLICE = slice(8000, 8512)


def _close(got, want):
    assert ((got - want).abs() <= 1e-5 * want.abs().clamp(min=1)).all()


def test_cvrp100_config3_full_batch(dev):
    from oracle.envs import CVRPOracle, cvrp_nearest_action
    from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode, CVRPStepwiseEpisode

    b, n = 32768, 100
    torch.manual_seed(1234)  # SURVEY 8d config 3 recipe (cvrp/generator.py:116-143)
    locs_all = torch.rand(b, n + 1, 2)
    demand = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
    gen = {"depot": locs_all[:, 0].contiguous(), "locs": locs_all[:, 1:].contiguous(),
           "demand": demand}
    td = {k: v.to(dev) for k, v in gen.items()}
    fused = CVRPFusedEpisode(td)
    fused.run_eager()
    torch.cuda.synchronize()
    assert int(fused.status.item()) == 0
    sf = fused.final_state()
    sw = CVRPStepwiseEpisode(td).capture()
    T = sw.replay()
    torch.cuda.synchronize()
    assert int(sw.status.item()) == 0
    ss = sw.final_state()
    assert T == sf["steps"]  # the batch-wide episode length, both engines
    acts = sf["actions"].cpu()
    assert torch.equal(acts, ss["actions"].cpu())
    for k in ("visited", "action_mask", "used_capacity", "current_node", "done"):
        assert torch.equal(sf[k].cpu(), ss[k].cpu()), k
    # the two engines' reward kernels sum the edges in different orders (tolerance 1e-5)
    _close(sf["reward"].cpu(), ss["reward"].cpu())
    # every customer exactly once, depot padding after the last customer
    cust = torch.zeros(b, n + 1, dtype=torch.int64).scatter_add_(1, acts, torch.ones_like(acts))
    assert (cust[:, 1:] == 1).all()
    last = torch.where(acts > 0, torch.arange(acts.shape[1]).expand_as(acts), -1).max(1).values
    tail = torch.arange(acts.shape[1])[None, :] > last[:, None]
    assert (acts[tail] == 0).all()
    assert sf["visited"].all() and sf["done"].all()
    # per-route load <= capacity (1.0 after the /capacity normalisation)
    d = torch.cat([torch.zeros(b, 1), demand], 1).gather(1, acts)
    route = (acts == 0).cumsum(1)
    load = torch.zeros(b, int(route.max()) + 1).scatter_add_(1, route, d)
    assert (load <= 1.0 + 1e-5).all()
    # the oracle on a slice of the same batch: its own batch-wide length <= T, then depot
    env = CVRPOracle(num_loc=n, seed=1234)
    tds = env.reset(TD({k: v[SLICE].clone() for k, v in gen.items()}, [512]))
    r, tdf, a = ref_rollout(env, tds, cvrp_nearest_action)
    ts = a.shape[1]
    assert ts <= T
    assert torch.equal(acts[SLICE, :ts], a) and (acts[SLICE, ts:] == 0).all()
    _close(sf["reward"].cpu()[SLICE], r)
    # the full batch keeps stepping the slice with the depot action until T (the policy's
    # choice once nothing is feasible): continue the oracle the same way
    for _ in range(T - ts):
        tdf["action"] = torch.zeros(512, dtype=torch.int64)
        tdf = env.step(tdf)["next"]
    assert torch.equal(sf["visited"].cpu()[SLICE], tdf["visited"])
    assert torch.equal(sf["used_capacity"].cpu()[SLICE], tdf["used_capacity"].view(-1, 1))


def _slap_batch(b, seed):
    from rl4co_slap_amd.envs.slap import SLAPGenerator

    torch.manual_seed(seed)
    np.random.seed(seed)
    return SLAPGenerator(materialize_dist_mat=False)(b)


def _slap_props(st, b, p=20, l=100):
    acts = st["actions"].cpu()
    assert (st["i"].cpu() == p).all() and st["done"].all()
    assert torch.equal(st["assignment"].cpu().long(), acts)
    assert (acts > 0).all()
    srt = acts.sort(1).values
    assert (srt[:, 1:] != srt[:, :-1]).all()  # P distinct locations
    m = st["action_mask"].cpu()
    assert (m.sum(1) == l - 1 - p).all() and not m[:, 0].any()
    assert not m.gather(1, acts).any()


@pytest.mark.parametrize("b", [16384, 65536])
def test_slap_config4_full_batch(dev, b):
    from oracle.envs import SLAPOracle, slap_closest_free_action
    from rl4co_slap_amd.rollout.engine import SLAPFusedEpisode, SLAPStepwiseEpisode

    gen = _slap_batch(b, 1234)
    td = gen.to(dev)
    fc = SLAPFusedEpisode(td, policy="closest")
    fc.run_eager()
    torch.cuda.synchronize()
    assert int(fc.status.item()) == 0
    sc = fc.final_state()
    _slap_props(sc, b)
    # teacher-forced seeded permutation (SURVEY 8d config 4 random-feasible)
    g = torch.Generator().manual_seed(4321)
    acts_t = torch.rand(b, 99, generator=g).argsort(1)[:, :20] + 1
    ft = SLAPFusedEpisode(td, actions=acts_t.to(dev), policy="teacher")
    ft.run_eager()
    torch.cuda.synchronize()
    assert int(ft.status.item()) == 0
    st = ft.final_state()
    _slap_props(st, b)
    assert torch.equal(st["actions"].cpu(), acts_t)
    if b == 16384:  # the stepwise engine at config 4's size: identical state and reward
        sw = SLAPStepwiseEpisode(td, policy="closest")
        sw.run_eager()
        torch.cuda.synchronize()
        assert int(sw.status.item()) == 0
        ss = sw.final_state()
        for k in ("actions", "assignment", "action_mask", "i", "done"):
            assert torch.equal(ss[k].cpu(), sc[k].cpu()), k
        _close(ss["reward"].cpu(), sc["reward"].cpu())
    # the oracle on a slice of the same batch, both policies
    env = SLAPOracle(seed=1234)
    keys = ("locs", "picklist", "depot_loc_dist", "assignment", "freq")
    for pol, st_ in (("closest", sc), ("teacher", st)):
        tds = env.reset(TD({k: gen[k][SLICE].clone() for k in keys}, [512]))
        if pol == "closest":
            r, tdf, a = ref_rollout(env, tds, slap_closest_free_action)
        else:
            it = iter(range(20))
            r, tdf, a = ref_rollout(env, tds, lambda t: acts_t[SLICE][:, next(it)])
        assert torch.equal(st_["actions"].cpu()[SLICE], a)
        for k in ("action_mask", "assignment", "i", "done"):
            assert torch.equal(st_[k].cpu()[SLICE], tdf[k]), (pol, k)
        _close(st_["reward"].cpu()[SLICE], r)
