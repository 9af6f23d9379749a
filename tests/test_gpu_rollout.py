"""GPU parity for the rollout engine (stepwise HIP-graph and the fused one-launch
episode) against the oracle's env-only rollout (rl4co/utils/decoding.py:88-109)."""
import pytest
import torch

from oracle.envs import TSPOracle, tsp_nearest_action
from oracle.rollout import rollout as ref_rollout
import functools

from rl4co_slap_amd.rollout.engine import TSPFusedEpisode, TSPStepwiseEpisode

pytestmark = pytest.mark.gpu

# the fused episode on both action layouts: row-major [B, N] (lane group per instance,
# the default) and step-major [N, B] (the LDS-tile engine)
ROWS = functools.partial(TSPFusedEpisode, layout="rows")
STEPS = functools.partial(TSPFusedEpisode, layout="steps")
LAYOUTS = pytest.mark.parametrize("fused", [ROWS, STEPS], ids=["rows", "steps"])


def _ref(b, n, seed, policy):
    env = TSPOracle(num_loc=n, seed=seed)
    td = env.reset(batch_size=[b])
    locs = td["locs"].clone()
    if policy == "teacher":
        acts = torch.rand(b, n, generator=torch.Generator().manual_seed(seed + 1)).argsort(1)
        it = iter(range(n))
        r, tdf, a = ref_rollout(env, td, lambda t: acts[:, next(it)])
    else:
        r, tdf, a = ref_rollout(env, td, tsp_nearest_action)
    return locs, a, r, tdf


def _check(state, a, r, tdf, exact_reward=False):
    assert torch.equal(state["action_mask"].cpu(), tdf["action_mask"])
    assert torch.equal(state["first_node"].cpu(), tdf["first_node"])
    assert torch.equal(state["current_node"].cpu(), tdf["current_node"])
    assert torch.equal(state["i"].cpu(), tdf["i"])
    assert torch.equal(state["done"].cpu(), tdf["done"])
    assert torch.equal(state["actions"].cpu(), a)
    got = state["reward"].cpu()
    assert ((got - r).abs() <= 1e-5 * r.abs().clamp(min=1)).all()


@pytest.mark.parametrize("cls", [ROWS, STEPS, TSPStepwiseEpisode], ids=["rows", "steps", "stepwise"])
@pytest.mark.parametrize("b,n", [(1, 5), (100, 20), (256, 100), (77, 64), (65, 65), (40, 150)])
@pytest.mark.parametrize("policy", ["teacher", "nearest"])
def test_tsp_rollout_matches_oracle(dev, cls, b, n, policy):
    locs, a, r, tdf = _ref(b, n, 1234 + n, policy)
    ep = cls(locs.to(dev), a.to(dev) if policy == "teacher" else None, policy=policy)
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) == 0
    _check(ep.final_state(), a, r, tdf)
    # graph replay gives the same result
    ep.capture()
    ep.replay()
    torch.cuda.synchronize()
    _check(ep.final_state(), a, r, tdf)


@LAYOUTS
def test_tsp_fused_invalid_tour_flag(dev, fused):
    b, n = 70, 12
    locs = torch.rand(b, n, 2)
    acts = torch.arange(n).repeat(b, 1)
    acts[33, 5] = 7  # duplicate -> not a permutation
    ep = fused(locs.to(dev), acts.to(dev))
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) & 1


@LAYOUTS
def test_tsp_fused_full_size_properties(dev, fused):
    # BASELINE config 2 size: size-independent properties (oracle too slow to mirror whole)
    b, n = 65536, 100
    g = torch.Generator().manual_seed(1234)
    locs = torch.rand(b, n, 2, generator=g)
    acts = torch.rand(b, n, generator=torch.Generator().manual_seed(4321)).argsort(1)
    ep = fused(locs.to(dev), acts.to(dev))
    ep.run_eager()
    torch.cuda.synchronize()
    st = ep.final_state()
    assert int(ep.status.item()) == 0
    assert not st["action_mask"].any() and st["done"].all()
    assert (st["i"] == n).all()
    assert torch.equal(st["first_node"].cpu(), acts[:, 0])
    assert torch.equal(st["current_node"].cpu(), acts[:, -1])
    # every instance's reward against the oracle's tour length
    from oracle.ops import gather_by_index, get_tour_length

    ref = -get_tour_length(gather_by_index(locs, acts))
    got = st["reward"].cpu()
    assert ((got - ref).abs() <= 1e-5 * ref.abs().clamp(min=1)).all()
    # rotation invariance of the closed tour length
    ep2 = fused(locs.to(dev), acts.roll(37, dims=1).to(dev))
    ep2.run_eager()
    torch.cuda.synchronize()
    assert ((ep2.reward - ep.reward).abs() <= 1e-5 * ep.reward.abs()).all()


@pytest.mark.parametrize("bad", [5, 64 * 700 + 47, 64 * 700 + 48, 64 * 1000 + 63])
@LAYOUTS
def test_tsp_fused_large_batch_invalid_tour_flag(dev, bad, fused):
    """Revisit detection at the full batch (1.33 rounds of resident tiles: first-round and
    tail tiles, low and high lanes), other instances' rewards unaffected."""
    b, n = 64 * 1024, 100
    locs = torch.rand(b, n, 2, generator=torch.Generator().manual_seed(7))
    acts = torch.arange(n).repeat(b, 1)
    acts[bad, 60] = 3  # node 3 twice, node 60 never
    ep = fused(locs.to(dev), acts.to(dev))
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) & 1
    from oracle.ops import gather_by_index, get_tour_length

    ok = torch.ones(b, dtype=torch.bool)
    ok[bad] = False
    ref = -get_tour_length(gather_by_index(locs[ok], acts[ok]))
    got = ep.reward.cpu()[ok]
    assert ((got - ref).abs() <= 1e-5 * ref.abs().clamp(min=1)).all()


@pytest.mark.parametrize("b", [768 * 64 + 40, 65536, 2 * 768 * 64 + 100])
@LAYOUTS
def test_tsp_fused_split_tail_tiles_final_state(dev, b, fused):
    """Batches past one resident round (768 full 64-instance tiles on 256 CUs) end in
    split tiles (32 instances, 8 step ranges).  Every row's final state and reward against
    the reference semantics computed on the CPU: mask = nodes absent from the action row
    (rows with a revisit keep one), done = nothing left, first / current node, i = N."""
    from oracle.ops import gather_by_index, get_tour_length

    n = 100
    g = torch.Generator().manual_seed(b)
    locs = torch.rand(b, n, 2, generator=g)
    acts = torch.rand(b, n, generator=g).argsort(1)
    bad = torch.tensor([0, 49151, 49152, 49183, 49184, b - 1])
    acts[bad, 50] = acts[bad, 10]  # a revisit: the node at step 50 is never visited
    ep = fused(locs.to(dev), acts.to(dev))
    ep.run_eager()
    torch.cuda.synchronize()
    st = ep.final_state()
    assert int(ep.status.item()) & 1
    left = torch.ones(b, n, dtype=torch.bool)
    left.scatter_(1, acts, False)
    assert torch.equal(st["action_mask"].cpu(), left)
    assert torch.equal(st["done"].cpu().view(-1), ~left.any(1))
    assert (st["i"].cpu() == n).all()
    assert torch.equal(st["first_node"].cpu().view(-1), acts[:, 0])
    assert torch.equal(st["current_node"].cpu().view(-1), acts[:, -1])
    ref = -get_tour_length(gather_by_index(locs, acts))
    got = st["reward"].cpu().view(-1)
    assert ((got - ref).abs() <= 1e-5 * ref.abs().clamp(min=1)).all()


def _slap_ref(b, seed, policy):
    import numpy as np

    from oracle.envs import SLAPOracle, slap_closest_free_action
    from oracle.td import TD

    env = SLAPOracle(seed=seed)
    np.random.seed(seed)
    gen = env.generate([b])
    td = env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    if policy == "teacher":
        g = torch.Generator().manual_seed(seed)
        acts = torch.stack([torch.randperm(99, generator=g)[:20] + 1 for _ in range(b)])
        it = iter(range(20))
        r, tdf, a = ref_rollout(env, td, lambda t: acts[:, next(it)])
    else:
        r, tdf, a = ref_rollout(env, td, slap_closest_free_action)
    return gen, a, r, tdf


@pytest.mark.parametrize("cls_name", ["SLAPFusedEpisode", "SLAPStepwiseEpisode"])
@pytest.mark.parametrize("b", [1, 64, 100, 300])
@pytest.mark.parametrize("policy", ["teacher", "closest"])
def test_slap_rollout_matches_oracle(dev, cls_name, b, policy):
    import rl4co_slap_amd.rollout.engine as eng
    from rl4co_slap_amd.td import TensorDict

    gen, a, r, tdf = _slap_ref(b, 1234 + b, policy)
    td = TensorDict({k: v.clone() for k, v in gen.items()}, [b]).to(dev)
    ep = getattr(eng, cls_name)(td, a.to(dev) if policy == "teacher" else None, policy=policy)
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) == 0
    st = ep.final_state()
    for k in ("action_mask", "i", "assignment", "done"):
        assert torch.equal(st[k].cpu(), tdf[k]), k
    assert torch.equal(st["actions"].cpu(), a)
    got = st["reward"].cpu()
    assert ((got - r).abs() <= 1e-5 * r.abs().clamp(min=1)).all()


@pytest.mark.parametrize("aisles,locs,prods,orders", [(6, 8, 12, 9), (12, 15, 40, 25),
                                                      (10, 10, 20, 20), (4, 5, 19, 7),
                                                      (7, 7, 20, 9)])
@pytest.mark.parametrize("dist", ["grid", "random_ties", "zeros_inf"])
@pytest.mark.parametrize("cls_name", ["SLAPFusedEpisode", "SLAPStepwiseEpisode"])
def test_slap_fused_closest_sizes(dev, aisles, locs, prods, orders, dist, cls_name):
    """Closest-free episodes for every lane-group width of the fused kernel (L = 48 -> 8
    lanes, 100 -> 16, 180 -> 32), P close to L - 1 (a lane's sorted list runs dry), and
    depot distances with many exact ties at random positions; the stepwise engine's
    co_slap_closest_step (policy + step in one launch: 1 / 2 / 3 units of 4 locations
    per lane; L = 49 takes its two-launch fallback).  "zeros_inf": ties of -0.0 / +0.0 and
    a few +inf distances (never picked while a finite free slot is left)."""
    import numpy as np

    import rl4co_slap_amd.rollout.engine as eng
    from oracle.envs import SLAPOracle, slap_closest_free_action
    from oracle.td import TD
    from rl4co_slap_amd.td import TensorDict

    b = 77
    env = SLAPOracle(n_products=prods, n_aisles=aisles, n_locs=locs, max_orders=orders, seed=3)
    np.random.seed(3)
    gen = env.generate([b])
    if dist in ("random_ties", "zeros_inf"):
        g = torch.Generator().manual_seed(9)
        gen["depot_loc_dist"] = torch.randint(0, 6, gen["depot_loc_dist"].shape,
                                              generator=g).float() * 0.5
    if dist == "zeros_inf":
        dd = gen["depot_loc_dist"]
        sel = torch.rand(dd.shape, generator=g)
        dd[(dd == 0) & (sel < 0.5)] = -0.0
        dd[sel > 0.97] = float("inf")
    td = env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    r, tdf, a = ref_rollout(env, td, slap_closest_free_action)
    ep = getattr(eng, cls_name)(TensorDict({k: v.clone() for k, v in gen.items()}, [b]).to(dev),
                                None, policy="closest")
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) == 0
    st = ep.final_state()
    assert torch.equal(st["actions"].cpu(), a)
    for k in ("action_mask", "i", "assignment", "done"):
        assert torch.equal(st[k].cpu(), tdf[k]), k
    got = st["reward"].cpu()
    assert ((got - r).abs() <= 1e-5 * r.abs().clamp(min=1)).all()


# --------------------------------------------------------------------------- CVRP
def _cvrp_ref(b, n, seed):
    from oracle.envs import CVRPOracle, cvrp_nearest_action
    from oracle.td import TD

    env = CVRPOracle(num_loc=n, seed=seed)
    gen = env.generate([b])
    td = env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    r, tdf, a = ref_rollout(env, td, cvrp_nearest_action)
    return gen, float(env.vehicle_capacity), a, r, tdf


def _check_cvrp(state, a, r, tdf):
    assert state["steps"] == a.shape[1]
    assert torch.equal(state["actions"].cpu(), a)
    for k in ("locs", "visited", "action_mask", "vehicle_capacity"):
        assert torch.equal(state[k].cpu(), tdf[k].to(state[k].dtype)), k
    assert torch.equal(state["current_node"].cpu(), tdf["current_node"].view(-1, 1))
    assert torch.equal(state["used_capacity"].cpu(), tdf["used_capacity"].view(-1, 1))
    assert torch.equal(state["done"].cpu(), tdf["done"].view(-1))
    got = state["reward"].cpu()
    assert ((got - r).abs() <= 1e-5 * r.abs().clamp(min=1)).all()


@pytest.mark.parametrize("b,n", [(1, 5), (64, 20), (256, 100), (33, 63), (9, 127), (17, 130)])
@pytest.mark.parametrize("kind", ["fused", "stepwise", "stepwise_pair"])
def test_cvrp_rollout_matches_oracle(dev, b, n, kind):
    from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode, CVRPStepwiseEpisode

    gen, vcap, a, r, tdf = _cvrp_ref(b, n, 4321 + n)
    td = {k: v.to(dev) for k, v in gen.items()}
    if kind == "fused":
        ep = CVRPFusedEpisode(td, vehicle_capacity=vcap)
        ep.run_eager()
        torch.cuda.synchronize()
        assert int(ep.status.item()) == 0
        _check_cvrp(ep.final_state(), a, r, tdf)
        ep.capture()
        ep.replay()
        torch.cuda.synchronize()
        _check_cvrp(ep.final_state(), a, r, tdf)
    else:
        # stepwise: co_cvrp_nearest_step (policy + step in one launch); stepwise_pair: the
        # co_cvrp_nearest_action + co_cvrp_step pair
        ep = CVRPStepwiseEpisode(td, vehicle_capacity=vcap, chunk=4,
                                 fused_policy=kind == "stepwise").capture()
        for _ in range(2):  # replays are repeatable
            T = ep.replay()
            torch.cuda.synchronize()
            assert T == a.shape[1]
            assert int(ep.status.item()) == 0
            _check_cvrp(ep.final_state(), a, r, tdf)


def test_cvrp_fused_truncation_flag(dev):
    from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode

    gen, vcap, a, r, tdf = _cvrp_ref(8, 20, 5)
    ep = CVRPFusedEpisode({k: v.to(dev) for k, v in gen.items()}, vehicle_capacity=vcap,
                          max_steps=10)
    ep.run_eager()
    torch.cuda.synchronize()
    with pytest.raises(RuntimeError, match="not done"):
        ep.final_state()


def _sqrt_tie_pair(c):
    """Two points whose f32 squared distances to `c` differ while their correctly rounded
    f32 sqrt is equal (found by nudging one coordinate by single ulps)."""
    g = torch.Generator().manual_seed(0)
    for _ in range(10000):
        a = torch.rand(2, generator=g) * 0.5 + 0.25
        b = a.clone()
        for _ in range(4):
            b[0] = torch.nextafter(b[0], torch.tensor(2.0))
            da, db = a - c, b - c
            sa = da[0] * da[0] + da[1] * da[1]
            sb = db[0] * db[0] + db[1] * db[1]
            ra, rb = torch.sqrt(sa.double()).float(), torch.sqrt(sb.double()).float()
            if sa != sb and ra == rb:  # correctly rounded sqrt (see oracle/envs.py _f32_sqrt)
                return (a, b) if sa < sb else (b, a)
    raise AssertionError("no tie pair found")


@pytest.mark.parametrize("n", [8, 40, 100])
def test_nearest_sqrt_tie_lowest_index(dev, n):
    """torch.argmin over rounded distances picks the LOWER index of two nodes whose
    squared distances differ but round to the same sqrt; the kernels scan squared
    distances and must repair such ties."""
    from oracle.envs import tsp_nearest_action  # noqa: F401  (policy under test: rollout)

    c = torch.tensor([0.5, 0.5])
    near, far = _sqrt_tie_pair(c)  # |far| > |near| in squared distance, same sqrt
    b = 3
    locs = torch.rand(b, n, 2) * 0.01 + 5.0  # every other node far away
    locs[:, 0] = c
    idx_far, idx_near = 1 + (n // 3), 2 + (n // 2)  # the larger squared distance first
    locs[:, idx_far], locs[:, idx_near] = far, near
    env = TSPOracle(num_loc=n, seed=1)
    from oracle.td import TD

    td = env.reset(TD({"locs": locs.clone()}, [b]))
    r, tdf, a = ref_rollout(env, td, tsp_nearest_action)
    assert (a[:, 1] == idx_far).all()  # the reference's choice
    ep = TSPFusedEpisode(locs.to(dev), None, policy="nearest")
    ep.run_eager()
    torch.cuda.synchronize()
    _check(ep.final_state(), a, r, tdf)


@pytest.mark.parametrize("n", [97, 100, 112, 113])
@pytest.mark.parametrize("layout", ["pomo_lb3", "strided", "pomo_lb3_strided", "contiguous"])
def test_tsp_reward_row_kernel_layouts(dev, n, layout):
    """co_tsp_reward on row-major [B, N] actions through every row-kernel path: LDS-DMA
    (contiguous, instance batch a multiple of the wave's rows), 16-byte action pairs
    (16-byte aligned rows with an even stride: strided slices, POMO instance batches not a
    multiple of 4 -- TSP-100 takes 7 steps per lane there, an odd count: scalar loads) and
    scalar loads.  Reward = -tour length of locs[e % LB] (the multistart row map) within
    1e-5; invalid rows flagged."""
    from oracle.ops import gather_by_index, get_tour_length
    from rl4co_slap_amd import _native as nat

    g = torch.Generator().manual_seed(n)
    lb = 3 if layout.startswith("pomo") else 24
    b = lb * (5 if layout.startswith("pomo") else 1)
    locs = torch.rand(lb, n, 2, generator=g)
    acts = torch.stack([torch.randperm(n, generator=g) for _ in range(b)])
    acts[1, 4] = acts[1, 5]  # one invalid tour
    width = n + 2 if layout.endswith("strided") else n
    full = torch.zeros(b, width, dtype=torch.int64)
    full[:, :n] = acts
    a_dev = full.to(dev)[:, :n]
    assert a_dev.stride(0) == width
    reward = torch.empty(b, dtype=torch.float32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    l_dev = locs.to(dev)
    nat.call("co_tsp_reward", b, n, n, nat.ptr(l_dev), lb, nat.ptr(a_dev), a_dev.stride(0),
             a_dev.stride(1), 1, nat.ptr(reward), nat.ptr(status), nat.stream_of(l_dev))
    rows = torch.arange(b) % lb
    ref = -get_tour_length(gather_by_index(locs[rows], acts))
    r = reward.cpu()
    ok = torch.ones(b, dtype=torch.bool)
    ok[1] = False
    assert ((r[ok] - ref[ok]).abs() <= 1e-5 * ref[ok].abs().clamp(min=1)).all()
    assert int(status.item()) & nat.ST_INVALID_TOUR


@pytest.mark.parametrize("n", [20, 100, 112, 130])
@pytest.mark.parametrize("same_lane", [True, False])
def test_nearest_sqrt_tie_lane_layouts(dev, n, same_lane):
    """The fused nearest episodes pick on squared distances and repair ties of the rounded
    sqrt in a rare exact pass: a sqrt tie whose lower-index node sits before the winner in
    the SAME lane (node indices 16 apart: the G = 16 lane layout for N <= 128) and in
    another lane, plus an exact squared-distance tie at two indices, all through the
    oracle's argmin over rounded distances."""
    c = torch.tensor([0.5, 0.5])
    near, far = _sqrt_tie_pair(c)
    b = 4
    g = torch.Generator().manual_seed(n)
    locs = torch.rand(b, n, 2, generator=g) * 0.01 + 5.0  # every other node far away
    locs[:, 0] = c
    idx_far = 3
    idx_near = idx_far + 16 if same_lane else idx_far + 5
    locs[:, idx_far], locs[:, idx_near] = far, near
    # an exact tie further on: two nodes at one point, both nearest from the tie pair
    t1, t2 = (idx_near + 7) % n, (idx_near + 23) % n
    if t1 not in (0, idx_far, idx_near) and t2 not in (0, idx_far, idx_near, t1):
        locs[:, t1] = locs[:, t2] = c + (near - c) * 1.01  # radially beyond the pair
    env = TSPOracle(num_loc=n, seed=1)
    from oracle.td import TD

    td = env.reset(TD({"locs": locs.clone()}, [b]))
    r, tdf, a = ref_rollout(env, td, tsp_nearest_action)
    assert (a[:, 1] == idx_far).all()
    ep = TSPFusedEpisode(locs.to(dev), None, policy="nearest")
    ep.run_eager()
    torch.cuda.synchronize()
    _check(ep.final_state(), a, r, tdf)


@pytest.mark.parametrize("n", [20, 100, 111])
@pytest.mark.parametrize("same_lane", [True, False])
def test_cvrp_nearest_sqrt_tie(dev, n, same_lane):
    """CVRP's fused nearest-feasible episode on the same sqrt-tie construction (customers
    near / far from the depot whose squared distances differ but round to one f32 sqrt):
    the lower node index wins, as the oracle's argmin over rounded distances."""
    from oracle.envs import CVRPOracle, cvrp_nearest_action
    from oracle.td import TD
    from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode

    c = torch.tensor([0.5, 0.5])
    near, far = _sqrt_tie_pair(c)
    b = 4
    env = CVRPOracle(num_loc=n, seed=9)
    gen = env.generate([b])
    gen["depot"][:] = c
    gen["locs"] = gen["locs"] * 0.01 + 5.0
    # node index = customer + 1; 16 apart: one lane of the G = 16 layout
    cf = 2
    cn = cf + 16 if same_lane else cf + 5
    gen["locs"][:, cf - 1], gen["locs"][:, cn - 1] = far, near
    td = env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    r, tdf, a = ref_rollout(env, td, cvrp_nearest_action)
    assert (a[:, 0] == cf).all()
    ep = CVRPFusedEpisode({k: v.to(dev) for k, v in gen.items()},
                          vehicle_capacity=float(env.vehicle_capacity))
    ep.run_eager()
    torch.cuda.synchronize()
    _check_cvrp(ep.final_state(), a, r, tdf)


@pytest.mark.parametrize("n", [30, 100, 110])
@pytest.mark.parametrize("grid", [4, 16])
def test_nearest_on_a_grid_many_ties(dev, n, grid):
    """Coordinates on a coarse grid: exact duplicates and many equal distances every step,
    so the truncated-key ratio test sends most steps down the exact path (lowest index of
    the rounded-distance minimum) -- TSP and CVRP against the oracle's argmin."""
    from oracle.envs import CVRPOracle, cvrp_nearest_action
    from oracle.td import TD
    from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode

    b = 24
    g = torch.Generator().manual_seed(n * grid)
    locs = torch.randint(0, grid, (b, n, 2), generator=g).float() / grid
    env = TSPOracle(num_loc=n, seed=1)
    r, tdf, a = ref_rollout(env, env.reset(TD({"locs": locs.clone()}, [b])), tsp_nearest_action)
    ep = TSPFusedEpisode(locs.to(dev), None, policy="nearest")
    ep.run_eager()
    torch.cuda.synchronize()
    _check(ep.final_state(), a, r, tdf)
    cenv = CVRPOracle(num_loc=n, seed=3)
    gen = cenv.generate([b])
    gen["depot"] = torch.randint(0, grid, (b, 2), generator=g).float() / grid
    gen["locs"] = torch.randint(0, grid, (b, n, 2), generator=g).float() / grid
    r, tdf, a = ref_rollout(cenv, cenv.reset(TD({k: v.clone() for k, v in gen.items()}, [b])),
                            cvrp_nearest_action)
    ep = CVRPFusedEpisode({k: v.to(dev) for k, v in gen.items()},
                          vehicle_capacity=float(cenv.vehicle_capacity))
    ep.run_eager()
    torch.cuda.synchronize()
    _check_cvrp(ep.final_state(), a, r, tdf)


@pytest.mark.parametrize("scale", [1e-3, 1e-19, 1e-21])
def test_nearest_tiny_and_near_ratio_distances(dev, scale):
    """Clusters of points a few `scale` apart (squared distances down to the f32 subnormal
    range, where the ratio bound does not hold and the exact path runs) and pairs whose
    squared distances differ by a relative 1e-6 (inside the ratio window, distinct sqrt)."""
    from oracle.td import TD

    b, n = 16, 100
    g = torch.Generator().manual_seed(int(-torch.log10(torch.tensor(scale)).item()))
    centers = torch.rand(b, 10, 2, generator=g) * (1.0 if scale > 1e-6 else scale * 100)
    locs = (centers.repeat_interleave(10, dim=1)
            + torch.randint(-3, 4, (b, n, 2), generator=g).float() * scale)
    locs[:, 1::7] = locs[:, 0:1] + (locs[:, 1::7] - locs[:, 0:1]) * (1 + 1e-6)
    env = TSPOracle(num_loc=n, seed=1)
    r, tdf, a = ref_rollout(env, env.reset(TD({"locs": locs.clone()}, [b])), tsp_nearest_action)
    ep = TSPFusedEpisode(locs.to(dev), None, policy="nearest")
    ep.run_eager()
    torch.cuda.synchronize()
    _check(ep.final_state(), a, r, tdf)
