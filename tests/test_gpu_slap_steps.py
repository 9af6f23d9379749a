"""co_slap_closest_steps (round 6): K consecutive closest-free SLAP steps (the bench policy
fused with SLAPEnv._step, slap/env.py:38-93) in one launch must leave every buffer exactly
as the K single co_slap_closest_step launches do -- both ping-pong state buffers (mask,
i), the actions, the assignment (the first step out of place from the starting one, then
in place), done, reward and the status word -- including distance ties, fully masked rows,
products out of range and negative, the uniform product (to_choose NULL), rows the lane
group kernel does not take (the single-step fallback); and the chunked stepwise episode
equals the one-launch-per-step episode."""
import pytest
import torch

from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.envs.slap import SLAPGenerator
from rl4co_slap_amd.rollout.engine import SLAPStepwiseEpisode

pytestmark = pytest.mark.gpu


def _run(b, l, p, k, dist, tc, tc_stride, st0, out_of_place, chunked, dev):
    mask0, i0, assign0 = st0
    mask = [mask0.clone(), torch.full_like(mask0, True)]
    i = [i0.clone(), torch.full_like(i0, -7)]
    assign = torch.full_like(assign0, -3) if out_of_place else assign0.clone()
    a_in = assign0 if out_of_place else assign
    acts = torch.full((k, b), -5, dtype=torch.int64, device=dev)
    done = torch.full((b,), True, dtype=torch.bool, device=dev)
    rew = torch.full((b,), True, dtype=torch.bool, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    s = nat.stream_of(mask0)
    tcp = nat.ptr(tc) if tc is not None else None
    if chunked:
        nat.call("co_slap_closest_steps", b, l, p, k, nat.ptr(dist), tcp, tc_stride, nat.ptr(a_in),
                 nat.ptr(assign), nat.ptr(mask[0]), nat.ptr(i[0]), nat.ptr(mask[1]), nat.ptr(i[1]),
                 nat.ptr(acts), b, nat.ptr(done), nat.ptr(rew), nat.ptr(status), s)
    else:
        for t in range(k):
            src, dst = t & 1, (t + 1) & 1
            nat.call("co_slap_closest_step", b, l, p, nat.ptr(dist),
                     nat.ptr(tc[:, t:]) if tc is not None else None,
                     tc_stride if tc is not None else tc_stride + t,
                     nat.ptr(a_in if t == 0 else assign), nat.ptr(assign), nat.ptr(mask[src]),
                     nat.ptr(mask[dst]), nat.ptr(acts[t]), nat.ptr(i[src]), nat.ptr(i[dst]),
                     nat.ptr(done), nat.ptr(rew), nat.ptr(status), s)
    torch.cuda.synchronize()
    return mask, i, assign, acts, done, rew, int(status.item())


@pytest.mark.parametrize("l", [100, 20, 64, 256, 36, 7, 300])
@pytest.mark.parametrize("b,k", [(1, 1), (63, 3), (1000, 7), (4096, 20)])
@pytest.mark.parametrize("out_of_place", [True, False])
def test_steps_equal_single_steps(dev, l, b, k, out_of_place):
    p = 20
    g = torch.Generator().manual_seed(l * 131 + b * 7 + k + out_of_place)
    dist = torch.randint(0, 9, (b, l), generator=g).float().to(dev)  # many ties
    mask = torch.rand(b, l, generator=g) < 0.8
    if b > 2:
        mask[1] = False  # a fully masked row: argmin of all-inf picks slot 0
    st0 = (mask.to(dev), torch.randint(0, p, (b, 1), generator=g).to(dev),
           torch.randint(-1, l, (b, p), generator=g).int().to(dev))
    tc = torch.randint(0, p, (b, p), generator=g).float()
    if b > 1:  # a negative product (python indexing) and one out of range (status bit)
        tc[0, 0] = -2
        tc[b - 1, k - 1] = p + 4
    tc = tc.to(dev)
    x = _run(b, l, p, k, dist, tc, p, st0, out_of_place, True, dev)
    y = _run(b, l, p, k, dist, tc, p, st0, out_of_place, False, dev)
    for j in range(2):
        assert torch.equal(x[0][j], y[0][j]), ("mask", j)
        assert torch.equal(x[1][j], y[1][j]), ("i", j)
    for name, a, c in zip(("assign", "acts", "done", "reward"), x[2:6], y[2:6]):
        assert torch.equal(a, c), name
    assert x[6] == y[6]
    if b > 1:
        assert x[6] & nat.ST_INDEX_RANGE


def test_steps_uniform_product(dev):
    """to_choose NULL: step t chooses product tc_stride + t for every row."""
    b, l, p, k = 777, 100, 20, 6
    g = torch.Generator().manual_seed(5)
    dist = torch.rand(b, l, generator=g).to(dev)
    st0 = ((torch.rand(b, l, generator=g) < 0.9).to(dev),
           torch.zeros(b, 1, dtype=torch.int64, device=dev),
           torch.full((b, p), -1, dtype=torch.int32, device=dev))
    x = _run(b, l, p, k, dist, None, 3, st0, True, True, dev)
    y = _run(b, l, p, k, dist, None, 3, st0, True, False, dev)
    for j in range(2):
        assert torch.equal(x[0][j], y[0][j]) and torch.equal(x[1][j], y[1][j])
    for a, c in zip(x[2:6], y[2:6]):
        assert torch.equal(a, c)
    assert x[6] == y[6] == 0
    assert torch.equal(x[2][:, 3:3 + k].long(), x[3].t())  # product 3+t holds step t's slot


def test_steps_validation(dev):
    lib = nat.load()
    # action stride below B, a uniform product past P, missing buffers: rejected
    assert lib.co_slap_closest_steps(4, 8, 5, 2, 1, 1, 5, 1, 1, 1, 1, 1, 1, 1, 3, 1, 1, 1,
                                     None) != 0
    assert lib.co_slap_closest_steps(4, 8, 5, 2, 1, None, 4, 1, 1, 1, 1, 1, 1, 1, 4, 1, 1, 1,
                                     None) != 0
    assert lib.co_slap_closest_steps(4, 8, 5, 2, 1, 1, 5, 1, 1, None, 1, 1, 1, 1, 4, 1, 1, 1,
                                     None) != 0
    assert lib.co_slap_closest_steps(0, 8, 5, 2, None, None, 0, None, None, None, None, None,
                                     None, None, 0, None, None, None, None) == 0


@pytest.mark.parametrize("chunk", [2, 7, 20])
def test_chunked_stepwise_episode_equals_per_step(dev, chunk):
    torch.manual_seed(chunk)
    td = SLAPGenerator(materialize_dist_mat=False)(2048).to(dev)
    a = SLAPStepwiseEpisode(td, policy="closest").capture()
    c = SLAPStepwiseEpisode(td, policy="closest", chunk=chunk).capture()
    a.replay()
    c.replay()
    torch.cuda.synchronize()
    fa, fc = a.final_state(), c.final_state()
    for key in ("action_mask", "i", "assignment", "done", "reward", "actions"):
        assert torch.equal(fa[key], fc[key]), key
    for j in range(2):
        assert torch.equal(a.mask[j], c.mask[j]) and torch.equal(a.i[j], c.i[j])
    assert int(c.status.item()) == 0
