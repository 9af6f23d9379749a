"""CO_DECODE_CERTIFIED -- the decoding strategies' default decode math: greedy picks on the
fast math, certified per row by an error bound, the exact math for any wave holding an
uncertified row.  The actions must be the exact path's (which is bit-exact with ATen,
tests/test_gpu_decode_exact.py) on every row -- including adversarial near-ties at and
around the certification margin, exact ties, tanh-saturated ties, NaN / inf rows and
all-masked rows -- and the selected log-probabilities within the float tolerance of the
north star, |lp - ref| <= 1e-5 * max(1, |ref|).

The second half repeats tests/test_gpu_decode_exact.py's assertions against the oracle
(the stock one with torch.tanh, and the one with the correctly rounded tanh) for the
certified math: identical action assertions, log-probabilities within that tolerance."""
import pytest
import torch

from oracle import decoding as odec
from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.utils.decoding import decode_step

LP_TOL = 1e-5  # relative, floored at 1: the north star's float tolerance


def _lp_close(lp, ref):
    return bool(((lp - ref).abs() <= LP_TOL * ref.abs().clamp(min=1)).all())

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


@pytest.mark.parametrize("n", [20, 100, 150, 600, 1500])
@pytest.mark.parametrize("clip,temp", [(10.0, 1.0), (0.0, 1.0), (10.0, 0.5), (0.0, 2.0)])
def test_certified_greedy_actions_equal_exact(dev, n, clip, temp):
    """Adversarial rows through both fallback tiers: near-ties before and after the pick
    (tier 1 resolves them from the exact z of the candidates; a candidate before the pick
    within the rounding bound, or two candidates in one lane, takes tier 2), exact ties,
    saturated ties, NaN / inf / all-masked rows (tier 2); N up to 1,500 (16 / 32 elements
    per lane)."""
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
    for name, kw in (("exact", {"decode_math": "exact"}), ("cert", {"decode_math": "certified"})):
        ep = POMOEpisode(locs, logits, tanh_clipping=10.0, **kw)
        ep.run_eager()
        torch.cuda.synchronize()
        assert int(ep.status.item()) == 0
        eps[name] = ep
    e, c = eps["exact"], eps["cert"]
    assert torch.equal(c.acts, e.acts)
    assert torch.equal(c.reward, e.reward)
    assert ((c.ll - e.ll).abs() <= 1e-5 * e.ll.abs().clamp(min=1)).all()


def test_pomo_and_strategies_default_to_certified(dev):
    from rl4co_slap_amd.rollout.pomo import POMOEpisode
    from rl4co_slap_amd.utils.decoding import Greedy

    locs = torch.rand(2, 5, 2, device=dev)
    ep = POMOEpisode(locs, torch.zeros(4, 10, 5, device=dev))
    assert ep.decode_math == "certified" and ep.mode == nat.DECODE_CERTIFIED
    assert POMOEpisode(locs, torch.zeros(4, 10, 5, device=dev), certified=False).mode == 0
    assert Greedy().decode_math == "certified"
    assert Greedy(decode_math="exact")._math_flags == 0


def _case(b, n, seed, scale=3.0, p_mask=0.3):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(b, n, generator=g) * scale
    mask = torch.rand(b, n, generator=g) > p_mask
    mask[torch.arange(b), torch.randint(0, n, (b,), generator=g)] = True
    return logits, mask


@pytest.mark.parametrize("n", [3, 10, 16, 17, 20, 33, 50, 64, 100, 128, 129, 200, 256, 500,
                               1000, 2048])
def test_certified_no_clip_vs_oracle(dev, n):
    """test_gpu_decode_exact.test_greedy_full_logp_bit_exact_no_clip for the certified
    math: the greedy action of every row is the oracle's, the selected logp within 1e-5."""
    b = max(64, min(4096, 200000 // n))
    logits, mask = _case(b, n, n)
    want = odec.process_logits(logits.clone(), mask)
    act, lp, _ = decode_step(logits.to(dev), mask.to(dev), "greedy", math="certified")
    ref_act = odec.greedy(want, mask)
    assert torch.equal(act.cpu(), ref_act)
    assert _lp_close(lp.cpu(), want.gather(1, ref_act[:, None]).squeeze(1))


@pytest.mark.parametrize("n", [20, 50, 100, 129])
@pytest.mark.parametrize("temp", [1.0, 0.7, 2.5])
def test_certified_with_tanh_cr_vs_oracle(dev, n, temp):
    """test_gpu_decode_exact.test_greedy_bit_exact_with_tanh_cr for the certified math:
    tanh clipping 10 + temperature, every action equal to the oracle's (run with the
    correctly rounded tanh), logp within 1e-5; the fused TSP step likewise."""
    b = 2048
    logits, mask = _case(b, n, 100 + n)
    want = odec.process_logits(logits.clone(), mask, temp, 10.0, tanh=odec.tanh_cr)
    ref_act = odec.greedy(want, mask)
    ref_lp = want.gather(1, ref_act[:, None]).squeeze(1)
    act, lp, _ = decode_step(logits.to(dev), mask.to(dev), "greedy", temperature=temp,
                             tanh_clipping=10.0, math="certified")
    assert torch.equal(act.cpu(), ref_act)
    assert _lp_close(lp.cpu(), ref_lp)
    # the same rows through the decode step fused with TSPEnv._step
    d = dev
    out = torch.empty(b, dtype=torch.int64, device=d)
    lpf = torch.empty(b, device=d)
    first = torch.empty(b, dtype=torch.int64, device=d)
    m_out = torch.empty((b, n), dtype=torch.bool, device=d)
    i_in = torch.full((b, 1), 3, dtype=torch.int64, device=d)
    i_out = torch.empty((b, 1), dtype=torch.int64, device=d)
    done = torch.empty(b, dtype=torch.bool, device=d)
    srew = torch.empty(b, dtype=torch.bool, device=d)
    st = torch.zeros(1, dtype=torch.int32, device=d)
    lg, mk = logits.to(d), mask.to(d)
    nat.call("co_tsp_decode_step", b, n, nat.ptr(lg), n, nat.ptr(mk), 10.0, float(temp),
             nat.DECODE_CERTIFIED, None, nat.ptr(out), nat.ptr(lpf), 0, 0, nat.ptr(m_out),
             nat.ptr(i_in), nat.ptr(i_out), None, nat.ptr(first), 1, nat.ptr(done),
             nat.ptr(srew), None, nat.ptr(st), nat.stream_of(lg))
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref_act)
    assert _lp_close(lpf.cpu(), ref_lp)
    want_mask = mask.clone()
    want_mask[torch.arange(b), ref_act] = False
    assert torch.equal(m_out.cpu(), want_mask)


@pytest.mark.parametrize("n", [20, 100])
def test_certified_against_stock_oracle_with_clip(dev, n):
    """test_gpu_decode_exact.test_greedy_against_stock_oracle_with_clip for the certified
    math (same action assertions; logp within 1e-5 instead of bit-exact)."""
    b, clip = 8192, 10.0
    logits, mask = _case(b, n, 7 * n, scale=1.0)
    want = odec.process_logits(logits.clone(), mask, 1.0, clip)
    act, lp, _ = decode_step(logits.to(dev), mask.to(dev), "greedy", tanh_clipping=clip,
                             math="certified")
    act, lp = act.cpu(), lp.cpu()
    ref_act = odec.greedy(want, mask)
    same_tanh = (torch.tanh(logits) == odec.tanh_cr(logits)).all(1)
    assert same_tanh.float().mean() > 0.2
    assert torch.equal(act[same_tanh], ref_act[same_tanh])
    top2 = want.topk(2, dim=-1).values
    clear = (top2[:, 0] - top2[:, 1]) > 4.0 * clip * 2.0 ** -23
    assert torch.equal(act[clear], ref_act[clear])
    assert int((~clear).sum()) <= 0.02 * b
    assert int((act != ref_act).sum()) <= 0.002 * b
    assert _lp_close(lp, want.gather(1, act[:, None]).squeeze(1))


def _offset_rows(t, dev):
    """`t` on the device as a view one element into a larger buffer: rows that start off a
    16-byte (logits) / 4-byte (mask) boundary, so the decode takes its any-alignment path."""
    flat = torch.empty(t.numel() + 1, dtype=t.dtype, device=dev)
    view = flat[1:].view(t.shape)
    view.copy_(t)
    return view


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 6, 7, 9, 13, 101, 103])
@pytest.mark.parametrize("misaligned", [False, True])
def test_certified_rows_of_any_alignment_vs_oracle(dev, n, misaligned):
    """GreedyRow's VW = 3 load (every chunk one 16-byte + one 4-byte access clamped to the
    row's last four columns, the partial chunk shifted down; r05) and VW = 2 (N < 4): every
    N % 4 residue, rows starting off a 16-byte boundary, tanh clipping 10 -- every action
    the oracle's (correctly rounded tanh), logp within 1e-5; the exact math's actions too."""
    b = 2048
    logits, mask = _case(b, n, 300 + n)
    want = odec.process_logits(logits.clone(), mask, 1.0, 10.0, tanh=odec.tanh_cr)
    ref_act = odec.greedy(want, mask)
    ref_lp = want.gather(1, ref_act[:, None]).squeeze(1)
    lg = _offset_rows(logits, dev) if misaligned else logits.to(dev)
    mk = _offset_rows(mask, dev) if misaligned else mask.to(dev)
    for math in ("certified", "exact"):
        act, lp, _ = decode_step(lg, mk, "greedy", tanh_clipping=10.0, math=math)
        assert torch.equal(act.cpu(), ref_act), math
        assert _lp_close(lp.cpu(), ref_lp), math
