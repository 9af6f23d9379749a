"""GPU parity beyond the fused engines' tile sizes: the node counts of the reference's
larger configs (CVRP's capacity table runs to N = 1,000, rl4co/envs/routing/cvrp/
generator.py:15-30; nothing in the env or decode code caps N).

* TSP env steps + reward at N = 500 / 1,000 against the oracle (every step's state);
* ``co_tsp_rollout`` past its single-launch limits (teacher N > 256, nearest N > 1,024):
  the stepwise launch sequence inside the same entry point;
* a POMO TSP-500 episode (decode-fused steps, reward, shared baseline);
* CVRP-500 / -1000 env steps with the nearest-feasible policy and the episode reward;
* decode rows longer than the register row engines (N > 2,048): ATen's log_softmax bit
  for bit (greedy / evaluate / top-k), sampling by its distribution;
* a SLAP warehouse of L = 300 slots through the fused-episode API (stepwise fallback).
Same bar as the other parity tests: bit-exact state / actions, rewards within 1e-5."""
import numpy as np
import pytest
import torch

import rl4co_slap_amd as ra
from oracle import decoding as odec
from oracle.envs import CVRPOracle, SLAPOracle, TSPOracle, cvrp_nearest_action, tsp_nearest_action
from oracle.rollout import constructive_forward, pomo_loss
from oracle.td import TD
from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.envs import CVRPEnv, TSPEnv
from rl4co_slap_amd.utils.decoding import decode_step

pytestmark = pytest.mark.gpu


def _close(got, ref, rtol=1e-5):
    got, ref = got.cpu(), ref.cpu()
    assert ((got - ref).abs() <= rtol * ref.abs().clamp(min=1.0)).all(), (got - ref).abs().max()


def _bits(a, b):
    return torch.equal(a.contiguous().view(torch.int32), b.contiguous().view(torch.int32))


@pytest.mark.parametrize("b,n,every", [(24, 500, 1), (8, 1000, 25)])
def test_tsp_env_steps_and_reward_large_n(dev, b, n, every):
    ref_env = TSPOracle(num_loc=n, seed=n)
    td_ref = ref_env.reset(batch_size=[b])
    env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
    td = env.reset(ra.TensorDict({"locs": td_ref["locs"].clone()}, [b]))
    acts = torch.rand(b, n, generator=torch.Generator().manual_seed(n)).argsort(1)
    for t in range(n):
        td_ref["action"] = acts[:, t].clone()
        td_ref = ref_env.step(td_ref)["next"]
        td["action"] = acts[:, t].to(dev)
        td = env.step(td)["next"]
        if t % every == 0 or t == n - 1:
            for k in ("action_mask", "first_node", "current_node", "i", "done", "reward"):
                assert torch.equal(td[k].cpu(), td_ref[k]), (k, t)
    _close(env.get_reward(td, acts.to(dev)), ref_env.get_reward(td_ref, acts))
    # step-major actions (the stepwise engine's layout) through the same entry point
    st = acts.t().contiguous().to(dev)
    r = torch.empty(b, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    nat.call("co_tsp_reward", b, n, n, nat.ptr(td["locs"]), b, nat.ptr(st), 1, b, 1, nat.ptr(r),
             nat.ptr(status), nat.stream_of(r))
    torch.cuda.synchronize()
    assert int(status.item()) == 0
    _close(r, ref_env.get_reward(td_ref, acts))
    bad = acts.clone()
    bad[1, 7] = bad[1, 8]
    with pytest.raises(AssertionError, match="Invalid tour"):
        env.get_reward(td, bad.to(dev))


@pytest.mark.parametrize("n,policy", [(300, "teacher"), (257, "teacher"), (1100, "nearest")])
def test_tsp_rollout_beyond_single_launch_limits(dev, n, policy):
    from rl4co_slap_amd.rollout.engine import TSPFusedEpisode

    b = 70 if n < 1000 else 5
    ref_env = TSPOracle(num_loc=n, seed=3)
    td_ref = ref_env.reset(batch_size=[b])
    locs = td_ref["locs"].clone()
    if policy == "teacher":
        acts = torch.rand(b, n, generator=torch.Generator().manual_seed(1)).argsort(1)
        it = iter(range(n))
        pol = lambda td: acts[:, next(it)]  # noqa: E731
    else:
        acts = None
        pol = tsp_nearest_action
    r_ref, td_ref, acts_ref = _oracle_rollout(ref_env, td_ref, pol)
    ep = TSPFusedEpisode(locs.to(dev), None if acts is None else acts.to(dev), policy=policy)
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) == 0
    st = ep.final_state()
    assert torch.equal(st["actions"].cpu(), acts_ref)
    for k in ("action_mask", "first_node", "current_node", "i"):
        assert torch.equal(st[k].cpu().reshape(td_ref[k].shape), td_ref[k]), k
    assert torch.equal(st["done"].cpu(), td_ref["done"].reshape(-1))
    _close(st["reward"], r_ref)


def _oracle_rollout(env, td, policy):
    from oracle.rollout import rollout

    return rollout(env, td, policy)


def test_pomo_tsp500_episode(dev):
    """POMO multistart greedy on TSP-500 (16 starts per instance, 4 instances): decode-fused
    steps with tanh clipping 10 (certified math), reward, shared baseline."""
    from rl4co_slap_amd.rollout.pomo import POMOEpisode

    b, n, s = 4, 500, 16
    g = torch.Generator().manual_seed(9)
    logits = torch.randn(n - 1, s * b, n, generator=g) * 2
    env = TSPOracle(num_loc=n, seed=n)
    td = env.reset(batch_size=[b])
    locs = td["locs"].clone()
    step = {"t": 0}

    def logits_fn(_):
        lg = logits[step["t"]]
        step["t"] += 1
        return lg.clone()

    out = constructive_forward(td, env, logits_fn, decode_type="multistart_greedy",
                               tanh_clipping=10.0, tanh=odec.tanh_cr, num_starts=s)
    ref = pomo_loss(out["reward"], out["log_likelihood"], s)
    for math in ("certified", "exact"):
        ep = POMOEpisode(locs.to(dev), logits.to(dev), num_starts=s, tanh_clipping=10.0,
                         decode_math=math)
        ep.run_eager()
        torch.cuda.synchronize()
        assert int(ep.status.item()) == 0
        st = ep.final_state()
        assert torch.equal(st["actions"].cpu(), out["actions"]), math
        _close(st["reward"], out["reward"])
        _close(st["log_likelihood"], out["log_likelihood"])
        assert torch.allclose(st["bl_val"].cpu(), ref["bl_val"].squeeze(1), rtol=1e-5, atol=1e-5)
        assert st["done"].all() and not st["action_mask"].any()


@pytest.mark.parametrize("b,n,every", [(16, 500, 1), (6, 1000, 20)])
def test_cvrp_env_steps_and_reward_large_n(dev, b, n, every):
    ref_env = CVRPOracle(num_loc=n, seed=n)
    gen = ref_env.generate([b])
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    env = CVRPEnv(generator_params=dict(num_loc=n), device=dev)
    td = env.reset(ra.TensorDict({k: v.clone() for k, v in gen.items()}, [b]))
    acts, t = [], 0
    while not td_ref["done"].all():
        a = cvrp_nearest_action(td_ref)
        td_ref["action"] = a
        td_ref = ref_env.step(td_ref)["next"]
        td["action"] = a.to(dev)
        td = env.step(td)["next"]
        acts.append(a)
        if t % every == 0:
            for k in ("action_mask", "current_node", "used_capacity", "visited", "done"):
                assert torch.equal(td[k].cpu().reshape(td_ref[k].shape), td_ref[k]), (k, t)
        t += 1
        assert t < 3 * n
    assert bool(td["done"].all())
    acts = torch.stack(acts, 1)
    _close(env.get_reward(td, acts.to(dev)), ref_env.get_reward(td_ref, acts))


def _rows(b, n, seed, p_mask=0.3, scale=3.0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(b, n, generator=g) * scale
    m = torch.rand(b, n, generator=g) > p_mask
    m[torch.arange(b), torch.randint(0, n, (b,), generator=g)] = True
    return x, m


@pytest.mark.parametrize("n", [2049, 3000, 5000, 20000])
@pytest.mark.parametrize("clip,temp", [(0.0, 1.0), (10.0, 1.0), (10.0, 0.7)])
def test_decode_long_rows_bit_exact(dev, n, clip, temp):
    b = 48 if n < 10000 else 8
    x, m = _rows(b, n, n)
    want = odec.process_logits(x.clone(), m, temp, clip, tanh=odec.tanh_cr)
    for math in ("exact", "certified"):
        act, lp, full = decode_step(x.to(dev), m.to(dev), "greedy", temperature=temp,
                                    tanh_clipping=clip, return_full=True, math=math)
        assert _bits(full.cpu(), want), math
        ref_act = odec.greedy(want, m)
        assert torch.equal(act.cpu(), ref_act), math
        assert _bits(lp.cpu(), want.gather(1, ref_act[:, None]).squeeze(1))
    given = torch.multinomial(m.float(), 1, generator=torch.Generator().manual_seed(2)).squeeze(1)
    a_e, lp_e, _ = decode_step(x.to(dev), m.to(dev), "evaluate", temperature=temp,
                               tanh_clipping=clip, action=given.to(dev))
    assert torch.equal(a_e.cpu(), given)
    assert _bits(lp_e.cpu(), want.gather(1, given[:, None]).squeeze(1))


def test_decode_long_rows_degenerate_and_top_k(dev):
    n = 4096
    x, m = _rows(16, n, 5)
    x[3, 100] = float("nan")
    m[4] = False  # all masked: NaN row, action 0, infeasible
    x[5, 7] = x[5, 9] = x[5].max() + 1  # exact tie: first index
    m[5, 7] = m[5, 9] = True
    want = odec.process_logits(x.clone(), m)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    act, lp, full = decode_step(x.to(dev), m.to(dev), "greedy", return_full=True, status=status)
    got = full.cpu()
    assert torch.equal(got.isnan(), want.isnan())
    fin = ~want.isnan()
    assert _bits(got[fin], want[fin])
    assert torch.equal(act.cpu()[[0, 1, 2, 3, 5]], want.argmax(1)[[0, 1, 2, 3, 5]])
    assert int(act[4]) == 0 and int(act[5]) == 7
    assert int(status.item()) & nat.ST_INFEASIBLE
    for k in (1, 5, 37):
        wk = odec.process_logits(x[:3].clone(), m[:3], top_k=k)
        _, _, fk = decode_step(x[:3].to(dev), m[:3].to(dev), "greedy", return_full=True, top_k=k)
        assert _bits(fk.cpu(), wk), k
    with pytest.raises(RuntimeError):  # top-p is not offered for rows this long
        decode_step(x[:2].to(dev), m[:2].to(dev), "sampling", top_p=0.9, seed=1)


def test_decode_long_rows_sampling_distribution(dev):
    """Sampling over 3,000 actions: one row repeated 20,000 times, its logits concentrated
    on 6 actions; empirical frequencies within a 5-sigma binomial band of softmax, every
    draw feasible, and the draw keyed by (seed, offset, row) deterministic."""
    n, reps = 3000, 20000
    g = torch.Generator().manual_seed(0)
    row = torch.full((n,), -30.0)
    hot = torch.tensor([5, 99, 1000, 2048, 2049, 2999])
    row[hot] = torch.randn(6, generator=g)
    mask = torch.ones(n, dtype=torch.bool)
    mask[17] = False
    x = row.expand(reps, n).contiguous()
    m = mask.expand(reps, n).contiguous()
    p = torch.softmax(odec.process_logits(row[None].clone(), mask[None])[0].double(), 0)
    a1, _, _ = decode_step(x.to(dev), m.to(dev), "sampling", seed=1234, offset=3)
    a2, _, _ = decode_step(x.to(dev), m.to(dev), "sampling", seed=1234, offset=3)
    assert torch.equal(a1, a2)
    a = a1.cpu()
    assert bool(mask[a].all())
    cnt = torch.bincount(a, minlength=n).double()
    for h in hot.tolist():
        mu = reps * p[h]
        sd = (reps * p[h] * (1 - p[h])).sqrt()
        assert abs(cnt[h] - mu) <= 5 * sd + 1, (h, cnt[h], mu)


def test_slap_fused_api_large_warehouse(dev):
    """L = 300 slots (n_aisles=20, n_locs=15): SLAPFusedEpisode runs the stepwise launch
    sequence; closest-free actions, final state and reward against the oracle."""
    from oracle.envs import slap_closest_free_action
    from rl4co_slap_amd.rollout.engine import SLAPFusedEpisode

    b = 12
    ref_env = SLAPOracle(n_aisles=20, n_locs=15, seed=4)
    np.random.seed(4)
    gen = ref_env.generate([b])
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    r_ref, td_ref, acts_ref = _oracle_rollout(ref_env, td_ref, slap_closest_free_action)
    td = {k: v.clone().to(dev) for k, v in gen.items()}
    ep = SLAPFusedEpisode(td, policy="closest")
    ep.run_eager()
    torch.cuda.synchronize()
    st = ep.final_state()
    assert torch.equal(st["actions"].cpu(), acts_ref)
    assert torch.equal(st["assignment"].cpu(), td_ref["assignment"])
    assert torch.equal(st["action_mask"].cpu(), td_ref["action_mask"])
    _close(st["reward"], r_ref)
