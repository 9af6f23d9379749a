"""CO_DECODE_CERTIFIED: greedy picks on the fast math, certified per row by an error bound,
the exact math for any wave holding an uncertified row.  The actions must be the exact
path's (which is bit-exact with ATen, tests/test_gpu_decode_exact.py) on every row --
including adversarial near-ties at and around the certification margin, exact ties,
tanh-saturated ties, NaN / inf rows and all-masked rows -- and the selected
log-probabilities within 1e-5 of the exact ones."""
import pytest
import torch

from rl4co_slap_amd import _native as nat

pytestmark = pytest.mark.gpu


def _adversarial_logits(b, n, seed, dev):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(b, n, generator=g) * 2
    top = x.argmax(1)
    rows = torch.arange(b)
    other = (top + 1 + torch.randint(0, n - 1, (b,), generator=g)) % n
    # a runner-up at distances that straddle the certification margin (clip 10: ~4e-5)
    gaps = torch.tensor([0.0, 1e-8, 1e-7, 1e-6, 3e-6, 1e-5, 2e-5, 4e-5, 6e-5, 1e-4, 1e-3])
    gi = torch.randint(0, len(gaps), (b,), generator=g)
    sel = rows % 3 == 0
    x[rows[sel], other[sel]] = x[rows[sel], top[sel]] - gaps[gi[sel]]
    # tanh-saturated ties (+10 after clipping) and exact ties
    x[rows % 17 == 1, :4] = 9.5
    x[rows % 19 == 2, 5] = x[rows % 19 == 2, 6]
    x[7, 3] = float("nan")
    x[8, 9] = float("inf")
    x[11, :] = 0.25
    mask = torch.rand(b, n, generator=g) > 0.2
    mask[rows, top] = True
    mask[13, :] = False  # all masked
    mask[14, :] = False
    mask[14, 2] = True  # one feasible action
    return x.to(dev), mask.to(dev)


def _decode(x, mask, clip, temp, mode):
    b, n = x.shape
    act = torch.empty(b, dtype=torch.int64, device=x.device)
    lp = torch.empty(b, dtype=torch.float32, device=x.device)
    st = torch.zeros(1, dtype=torch.int32, device=x.device)
    nat.call("co_decode_step", b, n, nat.ptr(x), n, nat.ptr(mask), float(clip), float(temp),
             mode, None, nat.ptr(act), nat.ptr(lp), None, 0, 0, nat.ptr(st), nat.stream_of(x))
    return act, lp


@pytest.mark.parametrize("n", [20, 100, 150])
@pytest.mark.parametrize("clip,temp", [(10.0, 1.0), (0.0, 1.0), (10.0, 0.5), (0.0, 2.0)])
def test_certified_greedy_actions_equal_exact(dev, n, clip, temp):
    x, mask = _adversarial_logits(4096, n, 3 + n, dev)
    a_e, lp_e = _decode(x, mask, clip, temp, 0)
    a_c, lp_c = _decode(x, mask, clip, temp, nat.DECODE_CERTIFIED)
    assert torch.equal(a_c, a_e)
    fin = torch.isfinite(lp_e)
    assert torch.equal(fin, torch.isfinite(lp_c))
    assert ((lp_c - lp_e)[fin].abs() <= 1e-5 * lp_e[fin].abs().clamp(min=1)).all()


def test_certified_fused_tsp_step_and_pomo_episode(dev):
    from rl4co_slap_amd.rollout.pomo import POMOEpisode

    torch.manual_seed(0)
    b, n = 64, 50
    locs = torch.rand(b, n, 2, device=dev)
    g = torch.Generator(device=dev).manual_seed(5)
    logits = torch.randn((n - 1, b * n, n), generator=g, device=dev)
    # near-ties in a slice of the rows of every step
    logits[:, ::7, 1] = logits[:, ::7, 2] + 2e-6
    eps = {}
    for name, kw in (("exact", {}), ("cert", {"certified": True})):
        ep = POMOEpisode(locs, logits, tanh_clipping=10.0, **kw)
        ep.run_eager()
        torch.cuda.synchronize()
        assert int(ep.status.item()) == 0
        eps[name] = ep
    e, c = eps["exact"], eps["cert"]
    assert torch.equal(c.acts, e.acts)
    assert torch.equal(c.reward, e.reward)
    assert ((c.ll - e.ll).abs() <= 1e-5 * e.ll.abs().clamp(min=1)).all()
