"""co_tsp_steps (round 6): K consecutive TSPEnv._step calls (tsp/env.py:67-93) in one launch
must leave every buffer exactly as the K single co_tsp_step launches do -- both ping-pong
state buffers (mask, i, first node), current node, done, reward and the status word --
including out-of-range actions, steps 0 with and without the first-node rule, rows the
lane-group kernel does not take (N % 4 != 0: the single-step fallback) and every group
width; and the chunked stepwise episode equals the one-launch-per-step episode."""
import pytest
import torch

from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.rollout.engine import TSPStepwiseEpisode

pytestmark = pytest.mark.gpu


def _state(b, n, dev, g):
    mask = (torch.rand(b, n, generator=g) < 0.7).to(dev)
    i = torch.randint(0, n, (b, 1), generator=g).to(dev)
    first = torch.randint(0, n, (b,), generator=g).to(dev)
    return mask, i, first


def _run(b, n, k, acts, st0, first_mode, chunked, dev):
    mask0, i0, first0 = st0
    bufs = {"mask": [mask0.clone(), torch.full_like(mask0, True)],
            "i": [i0.clone(), torch.full_like(i0, -7)],
            "first": [first0.clone(), torch.full_like(first0, -9)]}
    cur = torch.full((b,), -5, dtype=torch.int64, device=dev)
    done = torch.full((b,), True, dtype=torch.bool, device=dev)
    rew = torch.full((b,), True, dtype=torch.bool, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    s = nat.stream_of(mask0)
    if chunked:
        nat.call("co_tsp_steps", b, n, k, nat.ptr(acts), acts.stride(0),
                 nat.ptr(bufs["mask"][0]), nat.ptr(bufs["i"][0]), nat.ptr(bufs["first"][0]),
                 nat.ptr(bufs["mask"][1]), nat.ptr(bufs["i"][1]), nat.ptr(bufs["first"][1]),
                 nat.ptr(cur), nat.ptr(done), nat.ptr(rew), first_mode, nat.ptr(status), s)
    else:
        for t in range(k):
            src, dst = t & 1, (t + 1) & 1
            nat.call("co_tsp_step", b, n, nat.ptr(acts[t]), nat.ptr(bufs["mask"][src]),
                     nat.ptr(bufs["mask"][dst]), nat.ptr(bufs["i"][src]), nat.ptr(bufs["i"][dst]),
                     nat.ptr(bufs["first"][src]), nat.ptr(bufs["first"][dst]), nat.ptr(cur),
                     nat.ptr(done), nat.ptr(rew), first_mode if t == 0 else 0, None,
                     nat.ptr(status), s)
    torch.cuda.synchronize()
    return bufs, cur, done, rew, int(status.item())


@pytest.mark.parametrize("n", [100, 20, 32, 64, 128, 256, 1000, 7, 3])
@pytest.mark.parametrize("b,k", [(1, 1), (63, 2), (1000, 7), (4096, 10)])
@pytest.mark.parametrize("first_mode", [0, 1])
def test_steps_equal_single_steps(dev, n, b, k, first_mode):
    g = torch.Generator().manual_seed(n * 131 + b * 7 + k + first_mode)
    st0 = _state(b, n, dev, g)
    acts = torch.randint(0, n, (k, b), generator=g)
    if b > 1:  # a few out-of-range actions (negative / >= N): status bit, no clear
        acts[k - 1, 0] = -1
        acts[0, b - 1] = n + 3
    acts = acts.to(dev)
    x = _run(b, n, k, acts, st0, first_mode, True, dev)
    y = _run(b, n, k, acts, st0, first_mode, False, dev)
    for key in ("mask", "i", "first"):
        for j in range(2):
            assert torch.equal(x[0][key][j], y[0][key][j]), (key, j)
    for a, c in zip(x[1:4], y[1:4]):
        assert torch.equal(a, c)
    assert x[4] == y[4]
    if b > 1:
        assert x[4] & nat.ST_INDEX_RANGE


def test_steps_strided_action_rows(dev):
    """act_stride > B: action row t at action + t * stride (a [T, B'] slab, B' > B)."""
    b, n, k = 500, 100, 5
    g = torch.Generator().manual_seed(3)
    st0 = _state(b, n, dev, g)
    wide = torch.stack([torch.randperm(n, generator=g)[:k] for _ in range(b + 40)], 1).to(dev)
    x = _run(b, n, k, wide, st0, 1, True, dev)
    y = _run(b, n, k, wide[:, :b].contiguous(), st0, 1, False, dev)
    for key in ("mask", "i", "first"):
        for j in range(2):
            assert torch.equal(x[0][key][j], y[0][key][j]), (key, j)
    assert torch.equal(x[1], y[1]) and torch.equal(x[2], y[2])


def test_steps_validation(dev):
    lib = nat.load()
    # stride below B, bad first_mode, missing buffers: rejected without a launch
    assert lib.co_tsp_steps(4, 10, 2, 1, 3, 1, 1, 1, 1, 1, 1, None, 1, 1, 0, 1, None) != 0
    assert lib.co_tsp_steps(4, 10, 2, 1, 4, 1, 1, 1, 1, 1, 1, None, 1, 1, 2, 1, None) != 0
    assert lib.co_tsp_steps(4, 10, 2, 1, 4, None, 1, 1, 1, 1, 1, None, 1, 1, 0, 1, None) != 0
    assert lib.co_tsp_steps(0, 10, 2, None, 0, None, None, None, None, None, None, None, None,
                            None, 0, None, None) == 0


@pytest.mark.parametrize("chunk", [2, 10, 33, 100])
def test_chunked_stepwise_episode_equals_per_step(dev, chunk):
    b, n = 2048, 100
    g = torch.Generator().manual_seed(chunk)
    locs = torch.rand(b, n, 2, generator=g)
    acts = torch.rand(b, n, generator=g).argsort(1)
    a = TSPStepwiseEpisode(locs.to(dev), acts.to(dev)).capture()
    c = TSPStepwiseEpisode(locs.to(dev), acts.to(dev), chunk=chunk).capture()
    a.replay()
    c.replay()
    torch.cuda.synchronize()
    fa, fc = a.final_state(), c.final_state()
    for key in ("action_mask", "i", "first_node", "current_node", "done", "reward"):
        assert torch.equal(fa[key], fc[key]), key
    # both ping-pong buffers (the state of the last two steps)
    for j in range(2):
        assert torch.equal(a.mask[j], c.mask[j]) and torch.equal(a.i[j], c.i[j])
    assert int(c.status.item()) == 0
