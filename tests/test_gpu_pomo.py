"""GPU parity for the POMO multistart greedy episode (BASELINE config 5) against the
oracle's multistart ConstructivePolicy loop + POMO shared baseline
(rl4co/models/zoo/pomo/model.py:87-144, rl4co/models/rl/reinforce/baselines.py:57-61,
reinforce.py:97-115).  Every comparison is unconditional: the decode step is bit-exact
(tests/test_gpu_decode_exact.py), so the actions of every env must match."""
import pytest
import torch

from oracle import decoding as odec
from oracle.envs import TSPOracle
from oracle.ops import unbatchify
from oracle.rollout import constructive_forward, pomo_loss
from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.rollout.pomo import POMOEpisode

pytestmark = pytest.mark.gpu


def _oracle_episode(b, n, logits, **kw):
    env = TSPOracle(num_loc=n, seed=n)
    td = env.reset(batch_size=[b])
    locs = td["locs"].clone()
    step = {"t": 0}

    def logits_fn(td):
        lg = logits[step["t"]]
        step["t"] += 1
        return lg.clone()

    out = constructive_forward(td, env, logits_fn, decode_type="multistart_greedy", **kw)
    return locs, out


def _check_pomo(dev, st, out, ref, b, s):
    r, rr = st["reward"].cpu(), out["reward"]
    assert ((r - rr).abs() <= 1e-5 * rr.abs().clamp(min=1)).all()
    ll, lr = st["log_likelihood"].cpu(), out["log_likelihood"]
    assert ((ll - lr).abs() <= 1e-5 * lr.abs().clamp(min=1)).all()
    assert torch.allclose(st["bl_val"].cpu(), ref["bl_val"].squeeze(1), rtol=1e-5, atol=1e-5)
    assert torch.allclose(st["max_reward"].cpu(), ref["max_reward"], rtol=1e-5, atol=1e-6)
    rw = unbatchify(out["reward"], s)
    assert torch.equal(st["best_start"].cpu(), rw.argmax(1))
    loss = -st["loss_terms"].cpu().sum() / (b * s)
    # the loss is a cancelling sum: bound the error by the magnitude of its terms
    llr = unbatchify(out["log_likelihood"], s)
    scale = ((rw - rw.mean(1, keepdim=True)).abs() * llr.abs()).mean()
    assert (loss - ref["loss"]).abs() <= 1e-5 * scale + 1e-6
    assert st["done"].all() and not st["action_mask"].any()


@pytest.mark.parametrize("b,n", [(8, 20), (33, 50), (16, 100)])
def test_pomo_episode_matches_oracle(dev, b, n):
    """tanh clipping 10 inside the kernel, against the oracle evaluated with the same
    (correctly rounded) tanh: every action of every env equal."""
    s = n
    g = torch.Generator().manual_seed(7)
    logits = torch.randn(n - 1, s * b, n, generator=g) * 2
    locs, out = _oracle_episode(b, n, logits, tanh_clipping=10.0, tanh=odec.tanh_cr)
    ref = pomo_loss(out["reward"], out["log_likelihood"], s)
    ep = POMOEpisode(locs.to(dev), logits.to(dev), tanh_clipping=10.0)
    ep.run_eager()
    torch.cuda.synchronize()
    assert int(ep.status.item()) == 0
    st = ep.final_state()
    assert torch.equal(st["actions"].cpu(), out["actions"])
    _check_pomo(dev, st, out, ref, b, s)


@pytest.mark.parametrize("b,n", [(16, 100)])
def test_pomo_episode_stock_tanh(dev, b, n):
    """Against the stock oracle (torch.tanh = MKL on the CPU): the post-clip logits the
    oracle decodes, fed with clip 0, reproduce it exactly; with the kernel's own tanh
    only envs with a near-tie somewhere in their 99 steps may diverge (<= 1 %)."""
    s = n
    g = torch.Generator().manual_seed(11)
    logits = torch.randn(n - 1, s * b, n, generator=g) * 2
    locs, out = _oracle_episode(b, n, logits, tanh_clipping=10.0)
    ref = pomo_loss(out["reward"], out["log_likelihood"], s)
    ep = POMOEpisode(locs.to(dev), (torch.tanh(logits) * 10.0).to(dev), tanh_clipping=0.0)
    ep.run_eager()
    torch.cuda.synchronize()
    st = ep.final_state()
    assert torch.equal(st["actions"].cpu(), out["actions"])
    _check_pomo(dev, st, out, ref, b, s)
    ep2 = POMOEpisode(locs.to(dev), logits.to(dev), tanh_clipping=10.0)
    ep2.run_eager()
    torch.cuda.synchronize()
    diverged = int((ep2.final_state()["actions"].cpu() != out["actions"]).any(1).sum())
    assert diverged <= 0.01 * s * b, diverged


def test_pomo_shared_baseline_fixed_inputs(dev):
    """co_pomo_shared_baseline on fixed rewards / log-likelihoods of config 5's per-rank
    shard (1,024 instances x 100 starts), against the oracle's POMO loss terms."""
    b, s = 1024, 100
    g = torch.Generator().manual_seed(3)
    reward = -(torch.rand(s * b, generator=g) * 20 + 5)
    reward[::7] = reward[1::7][: reward[::7].numel()]  # duplicated maxima: first argmax wins
    ll = -torch.rand(s * b, generator=g) * 40
    ref = pomo_loss(reward, ll, s)
    rd, lld = reward.to(dev), ll.to(dev)
    bl = torch.empty(b, device=dev)
    mx = torch.empty(b, device=dev)
    best = torch.empty(b, dtype=torch.int64, device=dev)
    adv = torch.empty(s * b, device=dev)
    lt = torch.empty(b, device=dev)
    nat.call("co_pomo_shared_baseline", b, s, nat.ptr(rd), nat.ptr(lld), nat.ptr(bl), nat.ptr(mx),
             nat.ptr(best), nat.ptr(adv), nat.ptr(lt), nat.stream_of(rd))
    torch.cuda.synchronize()
    rw = unbatchify(reward, s)
    assert torch.allclose(bl.cpu(), ref["bl_val"].squeeze(1), rtol=2e-6, atol=0)
    assert torch.equal(mx.cpu(), ref["max_reward"])
    assert torch.equal(best.cpu(), rw.argmax(1))
    want_adv = (rw - ref["bl_val"]).t().reshape(-1)  # back to the [S, B] env layout
    assert torch.allclose(adv.cpu(), want_adv, rtol=0, atol=4e-6)
    loss = -lt.cpu().sum() / (b * s)
    scale = ((rw - rw.mean(1, keepdim=True)).abs() * unbatchify(ll, s).abs()).mean()
    assert (loss - ref["loss"]).abs() <= 1e-5 * scale


def test_pomo_config5_shard(dev):
    """Config 5's per-rank shard at its real size: 1,024 instances x 100 starts (102,400
    envs, 99 decode-fused steps), checked env by env against the oracle loop."""
    b, n = 1024, 100
    s = n
    g = torch.Generator().manual_seed(5)
    logits = torch.randn(n - 1, s * b, n, generator=g) * 2
    prev = torch.get_num_threads()
    torch.set_num_threads(min(16, torch.get_num_threads()))
    try:
        locs, out = _oracle_episode(b, n, logits, tanh_clipping=10.0, tanh=odec.tanh_cr)
    finally:
        torch.set_num_threads(prev)
    ref = pomo_loss(out["reward"], out["log_likelihood"], s)
    ep = POMOEpisode(locs.to(dev), logits.to(dev), tanh_clipping=10.0).capture()
    ep.replay()
    torch.cuda.synchronize()
    assert int(ep.status.item()) == 0
    st = ep.final_state()
    assert torch.equal(st["actions"].cpu(), out["actions"])
    _check_pomo(dev, st, out, ref, b, s)
