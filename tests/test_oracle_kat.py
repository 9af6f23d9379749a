"""Hand-derived known-answer tests pinning the CPU oracle to the reference's source
semantics (the reference holds no value fixtures)."""
import numpy as np
import pytest
import torch

from oracle.envs import CVRPOracle, SLAPOracle, TSPOracle
from oracle.ops import batchify, gather_by_index, get_tour_length, unbatchify
from oracle.rollout import rollout
from oracle.td import TD


def test_unit_square_tour_length():
    # ops.py:93-101: closed tour through the unit square corners = 4
    sq = torch.tensor([[[0.0, 0.0], [1.0, 0.0], [1.0, 1.0], [0.0, 1.0]]])
    assert get_tour_length(sq).item() == 4.0


def test_tsp_step_semantics_and_done():
    env = TSPOracle(num_loc=4, seed=0)
    locs = torch.tensor([[[0.0, 0.0], [1.0, 0.0], [1.0, 1.0], [0.0, 1.0]]])
    td = env.reset(TD({"locs": locs}, [1]))
    assert td["done"].shape == (1, 1) and td["terminated"].shape == (1, 1)
    assert td["action_mask"].all() and td["i"].item() == 0
    for k, a in enumerate([2, 0, 3, 1]):
        td["action"] = torch.tensor([a])
        td = env.step(td)["next"]
        assert td["i"].item() == k + 1
        assert td["first_node"].item() == 2  # first action sticks (tsp/env.py:70)
        assert not td["action_mask"][0, a]
        assert td["done"].item() == (k == 3)
        assert td["reward"].dtype == torch.bool  # zeros_like(done) (tsp/env.py:81)
    r = env.get_reward(td, torch.tensor([[2, 0, 3, 1]]))
    # 2->0 diag sqrt2, 0->3 1, 3->1 sqrt2, 1->2 1
    assert torch.allclose(r, torch.tensor([-(2 + 2 * 2 ** 0.5)]))


def test_tsp_first_node_batch_wide_test():
    # tsp/env.py:70: `i.all() == 0` is batch-wide -> if ANY i is 0, every row takes action
    env = TSPOracle(num_loc=3, seed=0)
    td = env.reset(batch_size=[2])
    td["i"] = torch.tensor([[0], [5]])
    td["first_node"] = torch.tensor([1, 1])
    td["action"] = torch.tensor([2, 0])
    td = env.step(td)["next"]
    assert td["first_node"].tolist() == [2, 0]


def test_tsp_invalid_tour_asserts():
    env = TSPOracle(num_loc=3, seed=0)
    td = env.reset(batch_size=[1])
    with pytest.raises(AssertionError, match="Invalid tour"):
        env.get_reward(td, torch.tensor([[0, 0, 1]]))


def test_cvrp_strict_capacity_boundary():
    # cvrp/env.py:140: strict `>`: a demand exactly equal to the remaining capacity is feasible
    env = CVRPOracle(num_loc=2, seed=0)
    td = TD({"locs": torch.tensor([[[0.1, 0.1], [0.2, 0.2]]]), "depot": torch.tensor([[0.0, 0.0]]),
             "demand": torch.tensor([[0.5, 0.5]]), "capacity": torch.tensor([[1.0]])}, [1])
    td = env.reset(td)
    # depot masked at reset while customers are feasible (cvrp/env.py:146-148)
    assert td["action_mask"].tolist() == [[False, True, True]]
    td["action"] = torch.tensor([1])
    td = env.step(td)["next"]
    assert td["used_capacity"].item() == 0.5
    assert td["action_mask"].tolist() == [[True, False, True]]  # 0.5 + 0.5 > 1.0 is False
    td["action"] = torch.tensor([2])
    td = env.step(td)["next"]
    assert td["action_mask"].tolist() == [[True, False, False]]
    assert not td["done"].item()
    td["action"] = torch.tensor([0])
    td = env.step(td)["next"]
    assert td["done"].item() and td["used_capacity"].item() == 0.0


def test_cvrp_over_capacity_and_padding():
    env = CVRPOracle(num_loc=2, seed=0)
    td = TD({"locs": torch.tensor([[[0.0, 1.0], [1.0, 0.0]]]), "depot": torch.tensor([[0.0, 0.0]]),
             "demand": torch.tensor([[0.6, 0.6]]), "capacity": torch.tensor([[1.0]])}, [1])
    td = env.reset(td)
    with pytest.raises(AssertionError, match="Used more than capacity"):
        env.get_reward(td, torch.tensor([[1, 2, 0]]))
    # zero padding after done adds zero-length depot->depot edges
    r1 = env.get_reward(td, torch.tensor([[1, 0, 2, 0]]))
    r2 = env.get_reward(td, torch.tensor([[1, 0, 2, 0, 0, 0]]))
    assert r1.item() == r2.item() == pytest.approx(-4.0)


def test_slap_grid_and_manhattan():
    env = SLAPOracle(seed=0)
    g = env.generate([2])
    locs = g["locs"]
    for i in [0, 7, 10, 55, 99]:
        assert locs[1, i, 0].item() == np.float32((i // 10) * 2.4)
        assert locs[1, i, 1].item() == float(i % 10)
    assert torch.equal(g["depot_loc_dist"], locs[..., 0] + locs[..., 1])
    assert g["assignment"].dtype == torch.int32 and (g["assignment"] == -1).all()
    assert g["picklist"].shape == (2, 20, 5) and g["picklist"].dtype == torch.int64
    assert g["freq"].shape == (2, 20, 1) and (g["freq"] >= 1).all() and (g["freq"] < 20).all()


def test_slap_reward_hand_built():
    env = SLAPOracle(n_products=3, n_aisles=1, n_locs=4, max_orders=2, max_products_in_order=3, seed=0)
    td = env.reset(env.generate([1]))
    # product p at location 1+p -> y = 1, 2, 3 ; x = 0
    td["assignment"] = torch.tensor([[1, 2, 3]], dtype=torch.int32)
    td["picklist"] = torch.tensor([[[0, 2, 1], [1, 1, 1]]])
    r = env.get_reward(td, None)
    # order 0: y 1 -> 3 -> 2 -> 1 = 2 + 1 + 1 = 4 ; order 1: duplicates -> 0
    assert r.item() == -4.0


def test_slap_done_exactly_at_p_and_shrinking_to_choose():
    env = SLAPOracle(seed=3)
    td = env.reset(batch_size=[3])
    assert not td["action_mask"][:, 0].any()
    for t in range(20):
        assert td["to_choose"].shape == (3, 20 - t)
        free = td["action_mask"].float().argmax(-1)
        td["action"] = free
        td = env.step(td)["next"]
        assert td["done"].shape == (3, 1)
        assert td["done"].all().item() == (t == 19)
    assert (td["assignment"] >= 1).all()


def test_batchify_roundtrip():
    # reference tests/test_utils.py:98-116
    x = torch.randn(5, 3, 2)
    y = batchify(x, 4)
    assert y.shape == (20, 3, 2)
    assert torch.equal(unbatchify(y, 4)[:, 2], x)
    assert torch.equal(y[2 * 5 + 3], x[3])  # layout index r*B + b


def test_gather_by_index_squeeze():
    src = torch.arange(24.0).view(2, 4, 3)
    out = gather_by_index(src, torch.tensor([1, 3]))
    assert out.shape == (2, 3) and out[1, 0].item() == 21.0


@pytest.mark.parametrize("name", ["tsp", "cvrp"])
def test_reference_shape_test(name):
    # reference tests/test_envs.py:39-59 (batch 2, size 20, random policy) -- shape only
    env = TSPOracle(num_loc=20, seed=1) if name == "tsp" else CVRPOracle(num_loc=20, seed=1)
    td = env.reset(batch_size=[2])
    r, _, _ = rollout(env, td, lambda t: torch.multinomial(t["action_mask"].float(), 1).squeeze(-1))
    assert r.shape == (2,)


# Philox-4x32-10 known-answer vectors published with the Random123 library (kat_vectors):
# (counter words, key words) -> output words.
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,want", PHILOX_KAT)
def test_philox_known_answers(ctr, key, want):
    from oracle.generate import philox4x32_10

    got = philox4x32_10(np.array([ctr], dtype=np.uint64), np.array([key], dtype=np.uint64))
    assert tuple(int(v) for v in got[0]) == want


def test_uniform_fill_oracle_grid_and_demand():
    from oracle.generate import uniform_fill

    v = uniform_fill(4099, 0.0, 1.0, seed=123)
    assert v.dtype == np.float32 and v.shape == (4099,)
    assert (v >= 0).all() and (v < 1).all()
    assert np.array_equal(v * 2.0 ** 24, np.floor(v * 2.0 ** 24))
    d = uniform_fill(20000, 0.0, 9.0, seed=7, capacity=40.0)
    k = np.rint(d * 40.0).astype(int)
    assert set(np.unique(k)) == set(range(1, 10))
    assert np.array_equal(uniform_fill(10, 0, 1, seed=5, offset=1), uniform_fill(14, 0, 1, seed=5)[4:])


def test_slap_dropin_episode_hand_known_answer():
    """The decode loop (constructive/base.py:229-251) on a hand-built SLAP instance with a
    known greedy sequence and reward -- values worked out by hand from slap/env.py:38-143
    and decoding.py:327-381, not produced by the oracle: 3 products, 4 locations on a line
    x = 0, 1, 2, 3 (location 0 the depot, masked at reset); the policy's logits favour
    location 3, then 1, then 2 (argmax over the still-free ones); to_choose = 0, 1, 2, so
    product p takes step p's location: assignment [3, 1, 2]; orders [[0, 1], [2, 2]]:
    order 0 is the closed tour 3 -> 1 -> 3 (length 4), order 1 a product picked twice
    (length 0): reward -4; done after exactly P = 3 steps, every location then masked."""
    from oracle.rollout import constructive_forward

    env = SLAPOracle(n_products=3, n_aisles=1, n_locs=4, seed=0)
    td = TD({"locs": torch.tensor([[[0.0, 0.0], [1.0, 0.0], [2.0, 0.0], [3.0, 0.0]]]),
             "freq": torch.ones(1, 3, 1), "assignment": torch.full((1, 3), -1, dtype=torch.int),
             "picklist": torch.tensor([[[0, 1], [2, 2]]]),
             "depot_loc_dist": torch.tensor([[0.0, 1.0, 2.0, 3.0]])}, [1])
    td = env.reset(td)
    assert td["action_mask"].tolist() == [[False, True, True, True]]
    table = torch.tensor([[0.0, 2.0, 1.0, 3.0]])
    steps = []
    out = constructive_forward(td, env, lambda t: steps.append(1) or table, decode_type="greedy")
    assert out["actions"].tolist() == [[3, 1, 2]]
    assert len(steps) == 3
    fin = out["td"]
    assert fin["assignment"].tolist() == [[3, 1, 2]]
    assert fin["action_mask"].tolist() == [[False, False, False, False]]
    assert bool(fin["done"].all()) and fin["i"].tolist() == [[3]]
    assert float(out["reward"][0]) == -4.0
