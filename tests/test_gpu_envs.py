"""GPU parity: the HIP env kernels (through the C ABI, via the env classes) against
the CPU oracle on identical seeded instances and actions.

Bar: bit-exact for masks / indices / bool and int state and the CVRP capacity
floats; episode rewards within |gpu - ref| <= 1e-5 * max(1, |ref|) (the summation
order of 100 f32 edges differs from ATen's vectorised CPU reduction)."""
import numpy as np
import pytest
import torch

from oracle.envs import (CVRPOracle, SLAPOracle, TSPOracle, cvrp_nearest_action,
                         slap_closest_free_action, tsp_nearest_action)
from oracle.td import TD
from rl4co_slap_amd.envs import CVRPEnv, SLAPEnv, TSPEnv

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def assert_reward_close(got, ref):
    got, ref = got.cpu(), ref.cpu()
    tol = RTOL * torch.clamp(ref.abs(), min=1.0)
    assert ((got - ref).abs() <= tol).all(), (got - ref).abs().max()


def assert_same(a, b, key):
    a = a.cpu()
    assert a.dtype == b.dtype, (key, a.dtype, b.dtype)
    assert a.shape == b.shape, (key, a.shape, b.shape)
    assert torch.equal(a, b), key


def rand_perm_actions(b, n, seed):
    g = torch.Generator().manual_seed(seed)
    return torch.rand(b, n, generator=g).argsort(1)


@pytest.mark.parametrize("b,n", [(1, 5), (63, 20), (128, 20), (200, 37), (64, 100), (130, 100), (7, 3)])
def test_tsp_teacher_forced_episode(dev, b, n):
    ref_env = TSPOracle(num_loc=n, seed=1234)
    td_ref = ref_env.reset(batch_size=[b])
    env = TSPEnv(generator_params=dict(num_loc=n), seed=99, device=dev)
    import rl4co_slap_amd as ra

    td = env.reset(ra.TensorDict({"locs": td_ref["locs"].clone()}, [b]))
    for k in ("action_mask", "first_node", "current_node", "i", "done", "terminated"):
        assert_same(td[k], td_ref[k], k)
    acts = rand_perm_actions(b, n, 4321)
    for t in range(n):
        td_ref["action"] = acts[:, t].clone()
        td_ref = ref_env.step(td_ref)["next"]
        td["action"] = acts[:, t].to(dev)
        td = env.step(td)["next"]
        for k in ("action_mask", "first_node", "current_node", "i", "done", "reward"):
            assert_same(td[k], td_ref[k], f"{k}@{t}")
    r_ref = ref_env.get_reward(td_ref, acts)
    r = env.get_reward(td, acts.to(dev))
    assert_reward_close(r, r_ref)


def test_tsp_invalid_tour_raises(dev):
    env = TSPEnv(generator_params=dict(num_loc=6), seed=1, device=dev)
    td = env.reset(batch_size=[4])
    acts = torch.arange(6).repeat(4, 1)
    acts[2, 3] = 1
    with pytest.raises(AssertionError, match="Invalid tour"):
        env.get_reward(td, acts.to(dev))
    env.check_solution = False
    env.get_reward(td, acts.to(dev))  # no check -> no error


def test_tsp_first_node_unknown_i_uses_device_test(dev):
    # td["i"] of foreign provenance -> batch-wide any(i == 0) on the device (tsp/env.py:70)
    ref_env = TSPOracle(num_loc=4, seed=0)
    env = TSPEnv(generator_params=dict(num_loc=4), seed=0, device=dev)
    for ivals, expect in [([[0], [5]], [2, 0]), ([[3], [5]], [1, 1])]:
        td = env.reset(batch_size=[2])
        td["i"] = torch.tensor(ivals, device=dev)
        td["first_node"] = torch.tensor([1, 1], device=dev)
        td["action"] = torch.tensor([2, 0], device=dev)
        td = env.step(td)["next"]
        assert td["first_node"].tolist() == expect
        assert td["i"].cpu().squeeze(-1).tolist() == [v[0] + 1 for v in ivals]


def test_tsp_nearest_policy_episode(dev):
    b, n = 96, 50
    ref_env = TSPOracle(num_loc=n, seed=5)
    td_ref = ref_env.reset(batch_size=[b])
    env = TSPEnv(generator_params=dict(num_loc=n), seed=5, device=dev)
    import rl4co_slap_amd as ra
    from rl4co_slap_amd import _native as nat

    td = env.reset(ra.TensorDict({"locs": td_ref["locs"].clone()}, [b]))
    for t in range(n):
        a_ref = tsp_nearest_action(td_ref)
        out = torch.empty(b, dtype=torch.int64, device=dev)
        nat.call("co_tsp_nearest_action", b, n, nat.ptr(td["locs"]), nat.ptr(td["action_mask"]),
                 nat.ptr(td["current_node"]), int(t == 0), nat.ptr(out), nat.stream_of(out))
        assert torch.equal(out.cpu(), a_ref), t
        td_ref["action"] = a_ref
        td_ref = ref_env.step(td_ref)["next"]
        td["action"] = out
        td = env.step(td)["next"]


def _cvrp_pair(b, n, seed, dev):
    import rl4co_slap_amd as ra

    ref_env = CVRPOracle(num_loc=n, seed=seed)
    gen = ref_env.generate([b])
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    env = CVRPEnv(generator_params=dict(num_loc=n), seed=seed, device=dev)
    td = env.reset(ra.TensorDict({k: v.clone() for k, v in gen.items()}, [b]))
    return ref_env, td_ref, env, td


CVRP_KEYS = ("locs", "action_mask", "current_node", "used_capacity", "vehicle_capacity", "visited")


@pytest.mark.parametrize("b,n", [(1, 10), (64, 20), (33, 50), (128, 100)])
def test_cvrp_random_feasible_episode(dev, b, n):
    ref_env, td_ref, env, td = _cvrp_pair(b, n, 1234, dev)
    for k in CVRP_KEYS:
        assert_same(td[k], td_ref[k], k)
    g = torch.Generator().manual_seed(11)
    acts = []
    t = 0
    while not td_ref["done"].all():
        a = torch.multinomial(td_ref["action_mask"].float(), 1, generator=g).squeeze(-1)
        acts.append(a)
        td_ref["action"] = a
        td_ref = ref_env.step(td_ref)["next"]
        td["action"] = a.to(dev)
        td = env.step(td)["next"]
        for k in CVRP_KEYS + ("done", "reward"):
            assert_same(td[k], td_ref[k], f"{k}@{t}")
        t += 1
    acts = torch.stack(acts, 1)
    assert_reward_close(env.get_reward(td, acts.to(dev)), ref_env.get_reward(td_ref, acts))


def _cvrp_step_raw(td, action, offset=0, not_done=None, inplace=False):
    """co_cvrp_step on copies of the state; `offset` bytes shift the visited / mask
    buffers off 16-B alignment (4: the quad kernel still applies; 3: the per-instance
    fallback kernel); `inplace` updates the visited buffer in place."""
    from rl4co_slap_amd import _native as nat

    b, n = td["demand"].shape
    dev = td["demand"].device

    def shifted(x):
        flat = torch.empty(x.numel() + 16, dtype=torch.uint8, device=dev)
        v = flat[offset:offset + x.numel()].view(x.shape)
        v.copy_(x.view(torch.uint8) if x.dtype == torch.bool else x)
        return v

    vis_in = shifted(td["visited"])
    vis_out, mask = shifted(td["visited"]), shifted(td["action_mask"])
    if inplace:
        vis_out = vis_in
    used_out = torch.empty_like(td["used_capacity"])
    cur = torch.empty((b, 1), dtype=torch.int64, device=dev)
    done = torch.empty(b, dtype=torch.bool, device=dev)
    rew = torch.empty(b, dtype=torch.bool, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    nat.call("co_cvrp_step", b, n, nat.ptr(action), nat.ptr(td["demand"]),
             nat.ptr(td["used_capacity"]), nat.ptr(used_out), nat.ptr(td["vehicle_capacity"]),
             nat.ptr(vis_in), nat.ptr(vis_out), nat.ptr(cur), nat.ptr(done), nat.ptr(rew),
             nat.ptr(mask), nat.ptr(status),
             nat.ptr(not_done) if not_done is not None else None, nat.stream_of(action))
    return {"visited": vis_out, "action_mask": mask.view(torch.bool), "used_capacity": used_out,
            "current_node": cur, "done": done, "reward": rew, "status": status}


# 3 <= N <= 252 with 4-B-aligned byte rows and a 16-B-aligned demand block: the quad kernel
# (16 lanes per row, up to 4 dwords per lane; partial quads when B % 4 != 0); N <= 511 aligned:
# the tile kernel (R = min(64, 8192 // (N+1)) & ~15 rows); N = 600 and misaligned buffers
# take the per-instance kernel
@pytest.mark.parametrize("b,n,offset", [(70, 100, 0), (70, 100, 3), (70, 100, 4), (41, 200, 0),
                                        (19, 511, 0), (3, 256, 0), (9, 600, 0), (64, 15, 0),
                                        (5, 3, 0), (6, 4, 0), (13, 63, 0), (11, 64, 0),
                                        (9, 255, 0), (7, 252, 0), (1, 100, 0), (2, 37, 0),
                                        (5, 97, 4), (3, 98, 0), (5, 99, 0)])
def test_cvrp_step_tile_paths_and_not_done(dev, b, n, offset):
    ref_env, td_ref, env, td = _cvrp_pair(b, n, 4242 + n, dev)
    g = torch.Generator().manual_seed(5)
    t = 0
    while not td_ref["done"].all():
        a = torch.multinomial(td_ref["action_mask"].float(), 1, generator=g).squeeze(-1)
        td_ref["action"] = a
        td_ref = ref_env.step(td_ref)["next"]
        nd = torch.zeros(1, dtype=torch.int32, device=dev)
        out = _cvrp_step_raw(td, a.to(dev), offset, nd, inplace=(t % 2 == 1))
        for k in ("visited", "action_mask", "used_capacity", "current_node", "done", "reward"):
            assert_same(out[k], td_ref[k], f"{k}@{t}")
        assert int(nd.item()) == int((~td_ref["done"]).sum()), t
        assert int(out["status"].item()) == 0
        td["action"] = a.to(dev)
        td = env.step(td)["next"]
        t += 1


def test_cvrp_step_out_of_range_action_flag(dev):
    _, _, env, td = _cvrp_pair(64, 30, 3, dev)
    a = torch.zeros(64, dtype=torch.int64, device=dev)
    a[5] = 31
    out = _cvrp_step_raw(td, a)
    assert int(out["status"].item()) & 8  # CO_ST_INDEX_RANGE
    assert int(out["visited"][5].sum().item()) == 0  # no visited update for the bad row


def test_cvrp_nearest_policy_and_mask(dev):
    from rl4co_slap_amd import _native as nat

    b, n = 80, 30
    ref_env, td_ref, env, td = _cvrp_pair(b, n, 77, dev)
    acts = []
    while not td_ref["done"].all():
        a_ref = cvrp_nearest_action(td_ref)
        cur = td["current_node"].contiguous()
        out = torch.empty(b, dtype=torch.int64, device=dev)
        nat.call("co_cvrp_nearest_action", b, n, nat.ptr(td["locs"]), nat.ptr(td["action_mask"]),
                 nat.ptr(cur), nat.ptr(out), nat.stream_of(out))
        assert torch.equal(out.cpu(), a_ref)
        acts.append(a_ref)
        td_ref["action"] = a_ref
        td_ref = ref_env.step(td_ref)["next"]
        td["action"] = out
        td = env.step(td)["next"]
        assert torch.equal(CVRPEnv.get_action_mask(td).cpu(), td_ref["action_mask"])
    acts = torch.stack(acts, 1)
    assert_reward_close(env.get_reward(td, acts.to(dev)), ref_env.get_reward(td_ref, acts))


def test_cvrp_validity_errors(dev):
    import rl4co_slap_amd as ra

    env = CVRPEnv(generator_params=dict(num_loc=2), device=dev)
    td = ra.TensorDict({"locs": torch.tensor([[[0.0, 1.0], [1.0, 0.0]]]),
                        "depot": torch.tensor([[0.0, 0.0]]), "demand": torch.tensor([[0.6, 0.6]]),
                        "capacity": torch.tensor([[1.0]])}, [1])
    td = env.reset(td)
    with pytest.raises(AssertionError, match="Used more than capacity"):
        env.get_reward(td, torch.tensor([[1, 2, 0]], device=dev))
    with pytest.raises(AssertionError, match="Invalid tour"):
        env.get_reward(td, torch.tensor([[1, 1, 0]], device=dev))
    r1 = env.get_reward(td, torch.tensor([[1, 0, 2, 0]], device=dev))
    r2 = env.get_reward(td, torch.tensor([[1, 0, 2, 0, 0, 0]], device=dev))
    assert r1.item() == r2.item() == pytest.approx(-4.0)


@pytest.mark.parametrize("b", [1, 32, 100])
def test_slap_episode(dev, b):
    import rl4co_slap_amd as ra

    ref_env = SLAPOracle(seed=1234)
    np.random.seed(1234)
    gen = ref_env.generate([b])
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    env = SLAPEnv(seed=1, device=dev)
    td = env.reset(ra.TensorDict({k: v.clone() for k, v in gen.items()}, [b]))
    keys = ("action_mask", "assignment", "to_choose", "i", "ratio", "reward", "done", "terminated")
    for k in keys:
        assert_same(td[k], td_ref[k], k)
    g = torch.Generator().manual_seed(3)
    for t in range(20):
        if t % 2 == 0:
            a = torch.multinomial(td_ref["action_mask"].float(), 1, generator=g).squeeze(-1)
        else:
            a = slap_closest_free_action(td_ref)
            from rl4co_slap_amd import _native as nat

            out = torch.empty(b, dtype=torch.int64, device=dev)
            nat.call("co_slap_closest_free_action", b, 100, nat.ptr(td["depot_loc_dist"]),
                     nat.ptr(td["action_mask"]), nat.ptr(out), nat.stream_of(out))
            assert torch.equal(out.cpu(), a)
        td_ref["action"] = a
        td_ref = ref_env.step(td_ref)["next"]
        td["action"] = a.to(dev)
        td = env.step(td)["next"]
        for k in ("action_mask", "assignment", "to_choose", "i", "reward", "done"):
            assert_same(td[k], td_ref[k], f"{k}@{t}")
    assert_reward_close(env.get_reward(td, None), ref_env.get_reward(td_ref, None))


def _slap_step_raw(td, action, inplace, offset=0):
    """co_slap_step on copies of the state (`offset` bytes shift the mask buffers off 4-B
    alignment: the byte-tile kernel instead of the 16-lane group kernel)."""
    from rl4co_slap_amd import _native as nat

    b, l = td["action_mask"].shape
    p = td["assignment"].shape[1]
    dev = action.device

    def shifted(x):
        flat = torch.empty(x.numel() + 16, dtype=torch.uint8, device=dev)
        v = flat[offset:offset + x.numel()].view(x.shape)
        v.copy_(x.view(torch.uint8))
        return v

    m_in, m_out = shifted(td["action_mask"]), shifted(td["action_mask"])
    a_in = td["assignment"].clone()
    a_out = a_in if inplace else torch.full_like(a_in, 12345)
    i_out = torch.empty_like(td["i"])
    done = torch.empty((b, 1), dtype=torch.bool, device=dev)
    rew = torch.empty((b, 1), dtype=torch.bool, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    tc = td["to_choose"]
    nat.call("co_slap_step", b, l, p, nat.ptr(action), nat.ptr(tc), tc.stride(0), nat.ptr(a_in),
             nat.ptr(a_out), nat.ptr(m_in), nat.ptr(m_out), nat.ptr(td["i"]), nat.ptr(i_out),
             nat.ptr(done), nat.ptr(rew), nat.ptr(st), nat.stream_of(action))
    return {"action_mask": m_out.view(torch.bool), "assignment": a_out, "i": i_out, "done": done,
            "reward": rew, "status": st}


@pytest.mark.parametrize("offset", [0, 1])
def test_slap_step_group_and_tile_paths(dev, offset):
    # negative actions index from the end (python indexing); in- and out-of-place
    # assignment; an out-of-range action flags CO_ST_INDEX_RANGE and clears nothing
    import rl4co_slap_amd as ra

    b = 37
    ref_env = SLAPOracle(seed=5)
    np.random.seed(5)
    gen = ref_env.generate([b])
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    env = SLAPEnv(seed=1, device=dev)
    td = env.reset(ra.TensorDict({k: v.clone() for k, v in gen.items()}, [b]))
    bad = torch.ones(b, dtype=torch.int64, device=dev)
    bad[4] = 100
    out = _slap_step_raw(td, bad, inplace=False, offset=offset)
    assert int(out["status"].item()) & 8
    assert torch.equal(out["action_mask"][4].cpu(), td["action_mask"][4].cpu())
    assert not torch.equal(out["action_mask"][3].cpu(), td["action_mask"][3].cpu())
    g = torch.Generator().manual_seed(9)
    for t in range(20):
        a = torch.multinomial(td_ref["action_mask"].float(), 1, generator=g).squeeze(-1)
        a[t % 3::3] -= 100  # the same locations, written python-negative
        out = _slap_step_raw(td, a.to(dev), inplace=(t % 2 == 1), offset=offset)
        td_ref["action"] = a
        td_ref = ref_env.step(td_ref)["next"]
        for k in ("action_mask", "assignment", "i", "done", "reward"):
            assert_same(out[k], td_ref[k], f"{k}@{t}")
        assert int(out["status"].item()) == 0
        td["action"] = a.to(dev)
        td = env.step(td)["next"]


def test_slap_reward_partial_assignment_wraps(dev):
    # unassigned products (-1) index the last location, like python indexing
    import rl4co_slap_amd as ra

    ref_env = SLAPOracle(seed=2)
    np.random.seed(2)
    gen = ref_env.generate([16])
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, [16]))
    env = SLAPEnv(seed=1, device=dev)
    td = env.reset(ra.TensorDict({k: v.clone() for k, v in gen.items()}, [16]))
    assign = torch.randint(-1, 100, (16, 20), dtype=torch.int32)
    td_ref["assignment"] = assign
    td["assignment"] = assign.to(dev)
    assert_reward_close(env.get_reward(td, None), ref_env.get_reward(td_ref, None))


def test_empty_batch(dev):
    env = TSPEnv(generator_params=dict(num_loc=10), device=dev)
    td = env.reset(batch_size=[0])
    td["action"] = torch.zeros(0, dtype=torch.int64, device=dev)
    td = env.step(td)["next"]
    assert td["action_mask"].shape == (0, 10)


def _cvrp_reward_status(dev, depot_locs, actions, demand, step_major):
    """co_cvrp_reward with check=1 on [b, T] actions; returns (reward, status bits)."""
    from rl4co_slap_amd import _native as nat

    b, T = actions.shape
    n = demand.shape[1]
    acts = (actions.t() if step_major else actions).contiguous().to(dev)
    sb, st = (1, b) if step_major else (T, 1)
    lf, dm = depot_locs.contiguous().to(dev), demand.contiguous().to(dev)
    vcap = torch.ones(b, device=dev)
    reward = torch.empty(b, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    nat.call("co_cvrp_reward", b, n, T, nat.ptr(lf), nat.ptr(acts), sb, st, nat.ptr(dm),
             nat.ptr(vcap), 1, nat.ptr(reward), nat.ptr(status), nat.stream_of(acts))
    return reward.cpu(), int(status.item())


def _oracle_over(demand, actions):
    from oracle.envs import CVRPOracle

    td = TD({"demand": demand, "vehicle_capacity": torch.ones(demand.shape[0], 1)}, [demand.shape[0]])
    try:
        CVRPOracle.check_solution_validity(td, actions)
    except AssertionError as e:
        return "capacity" in str(e)
    return False


@pytest.mark.parametrize("step_major", [False, True])
def test_cvrp_reward_capacity_scan_routes(dev, step_major):
    """Both reward kernels' capacity scans equal the reference's sequential scan per row
    (row-major actions: the route-split scan, lanes over routes, repeated passes until no
    route start changes; step-major: the tile kernel's sequential scan), including routes
    that end in (cap, cap + 1e-5] and leave a residual for the next one, a chain of three
    such routes (three passes), and a row of more than 64 routes (lanes owning two routes
    each) -- rows checked one launch each (status is batch-wide)."""
    g = torch.Generator().manual_seed(17)
    rows = []
    # residual 3.8e-6 after route 1; route 2 overflows only with it / fits even with it
    for tail, want in (([0.5, 0.500008], True), ([0.5, 0.5], False)):
        dm = torch.tensor([[0.5, 0.5000038] + tail])
        rows.append((dm, torch.tensor([[1, 2, 0, 3, 4, 0, 0]]), want))
    # a chain of residual routes: 3.8e-6 left after each of routes 1 and 2, so route 3 of
    # the same demands overflows only through the chain (1 + 3 x 3.8e-6 > 1 + 1e-5) while
    # a route 3 of [0.5, 0.5] still fits
    for tail, want in (([0.5, 0.5000038], True), ([0.5, 0.5], False)):
        dm = torch.tensor([[0.5, 0.5000038, 0.5, 0.5000038] + tail])
        rows.append((dm, torch.tensor([[1, 2, 0, 3, 4, 0, 5, 6, 0, 0]]), want))
    # 140 single-customer routes (> 64 routes per row), one of them over capacity or not
    for over_at in (None, 137):
        dm = torch.full((1, 140), 0.25)
        if over_at is not None:
            dm[0, over_at] = 1.5
        acts = torch.stack([torch.arange(1, 141), torch.zeros(140, dtype=torch.int64)], 1)
        rows.append((dm, acts.reshape(1, -1), over_at is not None))
    for r in range(40):
        n = int(torch.randint(5, 40, (1,), generator=g))
        dm = (torch.randint(1, 10, (1, n), generator=g).float() / 10.0)
        perm = torch.randperm(n, generator=g) + 1
        acts, used = [], 0.0
        for c in perm.tolist():  # greedy routes; some rows deliberately overfill one route
            if used + dm[0, c - 1].item() > 1.0 and not (r % 5 == 0 and len(acts) < 4):
                acts.append(0)
                used = 0.0
            acts.append(c)
            used += dm[0, c - 1].item()
        acts += [0] * int(torch.randint(1, 4, (1,), generator=g))
        rows.append((dm, torch.tensor([acts]), None))
    n_over = 0
    for dm, acts, want in rows:
        n = dm.shape[1]
        locs = torch.rand(1, n + 1, 2, generator=g)
        _, st = _cvrp_reward_status(dev, locs, acts, dm, step_major)
        over = _oracle_over(dm, acts)
        if want is not None:
            assert over == want
        assert bool(st & 2) == over, (dm, acts)
        assert not st & 1
        n_over += over
    assert 3 <= n_over < len(rows)


def _cvrp_oracle_reward(locs, demand, actions):
    td = TD({"locs": locs, "demand": demand,
             "vehicle_capacity": torch.ones(demand.shape[0], 1)}, [demand.shape[0]])
    return CVRPOracle._get_reward(None, td, actions)


def _cvrp_random_tours(b, n, extra, seed):
    """Valid tours over n customers with `extra` additional depot visits spread through
    them (row-major [b, n + extra]) and demands that make some rows overflow."""
    g = torch.Generator().manual_seed(seed)
    T = n + extra
    acts = torch.zeros(b, T, dtype=torch.int64)
    for r in range(b):
        slots = torch.randperm(T, generator=g)[:n].sort()[0]
        acts[r, slots] = torch.randperm(n, generator=g) + 1
    dm = torch.randint(1, 10, (b, n), generator=g).float() / 30.0
    locs = torch.rand(b, n + 1, 2, generator=g)
    return locs, dm, acts


@pytest.mark.parametrize("b,n,extra", [(1, 5, 3), (70, 10, 1490), (300, 100, 12), (64, 100, 60)])
@pytest.mark.parametrize("step_major", [False, True])
def test_cvrp_reward_tile_kernel_vs_oracle(dev, b, n, extra, step_major):
    """Rewards of both layouts vs the oracle's tour length; the validity/capacity status
    of the whole batch vs the oracle's asserts.  T = 1,500 makes the step-major tile
    kernel split the episode into chunks (its LDS demand sequence holds ~290 steps at
    N = 10), carrying the capacity scan across them; B = 70 / 300 leave partial tiles."""
    locs, dm, acts = _cvrp_random_tours(b, n, extra, 1000 + b + n)
    r, st = _cvrp_reward_status(dev, locs, acts, dm, step_major)
    assert_reward_close(r, _cvrp_oracle_reward(locs, dm, acts))
    assert bool(st & 2) == _oracle_over(dm, acts)
    assert not st & 1
    # per row: the status is batch-wide, so compare row by row on a few rows
    for row in range(min(b, 6)):
        _, st1 = _cvrp_reward_status(dev, locs[row:row + 1], acts[row:row + 1],
                                     dm[row:row + 1], step_major)
        assert bool(st1 & 2) == _oracle_over(dm[row:row + 1], acts[row:row + 1]), row


@pytest.mark.parametrize("step_major", [False, True])
def test_cvrp_reward_long_episode_row_major_fallback(dev, step_major):
    """T = 5,000 steps: beyond the wave-per-instance kernel's LDS sequence (64 KB), so
    row-major actions also take the chunked tile kernel (no CO_E_INVAL)."""
    locs, dm, acts = _cvrp_random_tours(3, 12, 4988, 77)
    r, st = _cvrp_reward_status(dev, locs, acts, dm, step_major)
    assert_reward_close(r, _cvrp_oracle_reward(locs, dm, acts))
    assert bool(st & 2) == _oracle_over(dm, acts)
    assert not st & 1


@pytest.mark.parametrize("step_major", [False, True])
def test_cvrp_reward_invalid_and_range(dev, step_major):
    """Revisit, missing customer and out-of-range index through both kernels: the
    reference's "Invalid tour" (and the gather's range error) as status bits."""
    locs, dm, acts = _cvrp_random_tours(130, 20, 10, 5)
    _, st = _cvrp_reward_status(dev, locs, acts, dm, step_major)
    assert not st & 1
    bad = acts.clone()
    nz = (bad[77] != 0).nonzero()[:2, 0]
    bad[77, nz[1]] = bad[77, nz[0]]  # revisit + a missing customer
    _, st = _cvrp_reward_status(dev, locs, bad, dm, step_major)
    assert st & 1
    bad = acts.clone()
    bad[129, 3] = 21  # out of range
    _, st = _cvrp_reward_status(dev, locs, bad, dm, step_major)
    assert st & 1 and st & 8


def _slap_reward_direct(dev, locs, assign, picks):
    from rl4co_slap_amd import _native as nat

    b, l, _ = locs.shape
    p = assign.shape[1]
    o, k = picks.shape[1], picks.shape[2]
    lc, ac, pc = locs.contiguous().to(dev), assign.contiguous().to(dev), picks.contiguous().to(dev)
    out = torch.empty(b, device=dev)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    nat.call("co_slap_reward", b, l, p, o, k, nat.ptr(ac), nat.ptr(pc), nat.ptr(lc), nat.ptr(out),
             nat.ptr(st), nat.stream_of(out))
    torch.cuda.synchronize()
    return out.cpu(), int(st.item())


@pytest.mark.parametrize("b,l,p,o,k", [
    (33, 100, 20, 20, 5),     # the lane-group kernel (16 instances per workgroup, tail block)
    (5, 120, 32, 25, 5),      # its largest register slots (L <= 128, P <= 32, S <= 128)
    (9, 300, 40, 30, 7),      # the LDS-staged wave-per-instance kernel
    (3, 9000, 20, 20, 5),     # beyond the LDS staging: the global-gather kernel
])
def test_slap_reward_paths_vs_oracle(dev, b, l, p, o, k):
    """co_slap_reward on every one of its three kernels, random coordinates, a partial
    assignment (-1 wraps to the last slot) and picklists, against the oracle's
    _get_reward (slap/env.py:131-143)."""
    g = torch.Generator().manual_seed(l + p)
    locs = torch.rand(b, l, 2, generator=g) * 10
    assign = torch.randint(-1, l, (b, p), generator=g, dtype=torch.int64).to(torch.int32)
    picks = torch.randint(0, p, (b, o, k), generator=g)
    got, st = _slap_reward_direct(dev, locs, assign, picks)
    ref = SLAPOracle._get_reward(TD({"assignment": assign, "picklist": picks, "locs": locs}, [b]),
                                 None)
    assert st == 0
    assert_reward_close(got, ref)
    # an out-of-range product index in a picklist is flagged (torch raises)
    picks[0, 1, 2] = p + 3
    _, st = _slap_reward_direct(dev, locs, assign, picks)
    assert st & 8


@pytest.mark.parametrize("n", [3, 16, 20, 24, 36, 100, 128, 252, 256, 260])
@pytest.mark.parametrize("b", [1, 15, 16, 17, 33, 1000])
def test_tsp_step_kernel_paths_vs_reference(dev, b, n):
    """co_tsp_step on arbitrary (not policy-reachable) states through every kernel path
    (the flat 16-byte-chunk kernel for N % 4 == 0, 16 <= N <= 256 incl. the partial last
    wave's tail dwords; the lane-group and tile kernels otherwise): random mask bytes with
    all-zero rows, actions at chunk / row boundaries, out-of-range actions (status bit, no
    byte cleared), first_mode 0 / 1, in and out of place -- against tsp/env.py:67-93."""
    from rl4co_slap_amd import _native as nat

    g = torch.Generator().manual_seed(b * 1000 + n)
    mask = torch.rand(b, n, generator=g) < 0.6
    mask[:: 5] = False  # rows with nothing left
    act = torch.randint(0, n, (b,), generator=g)
    act[1::7] = n - 1
    act[2::11] = 0
    bad = torch.zeros(b, dtype=torch.bool)
    if b > 3:
        act[3] = n  # out of range
        bad[3] = True
    i = torch.randint(0, n, (b, 1), generator=g)
    first = torch.randint(0, n, (b,), generator=g)
    for first_mode in (0, 1):
        for inplace in (False, True):
            m_d = mask.to(dev)
            m_o = m_d if inplace else torch.empty_like(m_d)
            i_d, f_d = i.to(dev), first.to(dev)
            i_o, f_o = torch.empty_like(i_d), torch.empty_like(f_d)
            cur = torch.empty_like(f_d)
            done = torch.empty(b, dtype=torch.bool, device=dev)
            rw = torch.ones(b, dtype=torch.bool, device=dev)
            st = torch.zeros(1, dtype=torch.int32, device=dev)
            a_d = act.to(dev)
            nat.call("co_tsp_step", b, n, nat.ptr(a_d), nat.ptr(m_d), nat.ptr(m_o), nat.ptr(i_d),
                     nat.ptr(i_o), nat.ptr(f_d), nat.ptr(f_o), nat.ptr(cur), nat.ptr(done),
                     nat.ptr(rw), first_mode, None, nat.ptr(st), nat.stream_of(m_d))
            want = mask.clone()
            ok = ~bad
            want[ok.nonzero().squeeze(1), act[ok]] = False
            assert torch.equal(m_o.cpu(), want), (first_mode, inplace)
            assert torch.equal(done.cpu(), ~want.any(-1))
            assert torch.equal(i_o.cpu(), i + 1)
            assert torch.equal(f_o.cpu(), act if first_mode == 1 else first)
            assert torch.equal(cur.cpu(), act)
            assert not bool(rw.any())
            assert bool(int(st.item()) & nat.ST_INDEX_RANGE) == bool(bad.any())
