"""The fork's own user path: ``ConstructivePolicy`` driving ``SLAPEnv`` with a policy shaped
like ``examples/slap.py:11-93`` (``AttentionModelPolicy(env_name="slap",
init_embedding=SLAPInitEmbedding, context_embedding=SLAPContext, dynamic_embedding=
StaticEmbedding)``; ``constructive/base.py:229-251`` is the loop).

The reference loop (``oracle/rollout.constructive_forward`` on ``SLAPOracle``, the
per-batch Python mask loop of ``slap/env.py:61-62`` included) is driven by the same
network evaluated on the device from the oracle's own state:
* greedy: actions, the final assignment / action mask / i / done bit-exact; reward and
  log-likelihood within 1e-5 (relative to max(1, |ref|));
* sampling (seeded): the sampled actions are feasible and distinct, and the oracle
  re-scores them in evaluate mode: the same assignment / masks, reward, log-likelihood;
* evaluate: given feasible action sequences, bit-exact state and 1e-5 reward / ll;
* config 4 (``examples/slap.py:75-76``, B = 16,384, seeds 1234): the whole batch on the
  device, the oracle on a 512-instance slice.
Then the fused ``co_slap_decode_step`` (one launch per loop step) against the two-launch
path (``co_decode_step`` + ``co_slap_step``) bit for bit, RNG use included, for SLAP and
CVRP (``co_cvrp_decode_step``).
"""
import numpy as np
import pytest
import torch

from oracle.envs import CVRPOracle, SLAPOracle
from oracle.rollout import constructive_forward
from oracle.td import TD
from rl4co_slap_amd import TensorDict
from rl4co_slap_amd.envs import CVRPEnv, SLAPEnv
from rl4co_slap_amd.envs.base import RL4COEnvBase
from rl4co_slap_amd.envs.slap import SLAPGenerator
from rl4co_slap_amd.rollout import ConstructivePolicy, LogitsDecoder

from am_pointer import PointerDecoder, SLAPPointerDecoder, slap_oracle_logits_fn

pytestmark = pytest.mark.gpu

TOL = 1e-5


def _close(a, b):
    a, b = a.cpu(), b.cpu()
    return bool(((a - b).abs() <= TOL * b.abs().clamp(min=1)).all())


def _slap_instance(b, seed):
    torch.manual_seed(seed)
    np.random.seed(seed)
    return SLAPOracle(seed=seed).generate([b])


def _pair(gen, dev):
    ref_env = SLAPOracle(seed=0)
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, gen["locs"].shape[:1]))
    env = SLAPEnv(device=dev)
    td = env.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()},
                              gen["locs"].shape[:1]))
    return ref_env, td_ref, env, td


def _check_state(td, td_ref):
    for k in ("assignment", "action_mask", "i", "done"):
        assert torch.equal(td[k].cpu(), td_ref[k]), k
    assert td["to_choose"].shape == td_ref["to_choose"].shape
    assert torch.equal(td["to_choose"].cpu(), td_ref["to_choose"])


def _feasible_actions(b, g):
    """Per instance: 20 distinct locations out of 1..99 (the depot is masked at reset)."""
    return torch.stack([torch.randperm(99, generator=g)[:20] + 1 for _ in range(b)])


@pytest.mark.parametrize("b", [1, 37, 64])
def test_slap_policy_greedy_matches_reference_loop(dev, b):
    gen = _slap_instance(b, 100 + b)
    ref_env, td_ref, env, td = _pair(gen, dev)
    dec = SLAPPointerDecoder(gen["locs"], dev)
    ref = constructive_forward(td_ref, ref_env, slap_oracle_logits_fn(dec, dev),
                               decode_type="greedy", tanh_clipping=10.0)
    pol = ConstructivePolicy(None, dec, env_name="slap", tanh_clipping=10.0)
    out = pol(td, env, phase="test", decode_type="greedy", return_actions=True)
    assert out["actions"].shape == (b, 20)
    assert torch.equal(out["actions"].cpu(), ref["actions"])
    _check_state(td, ref["td"])
    assert _close(out["reward"], ref["reward"])
    assert _close(out["log_likelihood"], ref["log_likelihood"])


def test_slap_policy_sampling_rescored_by_reference(dev):
    b = 48
    gen = _slap_instance(b, 7)
    ref_env, td_ref, env, td = _pair(gen, dev)
    dec = SLAPPointerDecoder(gen["locs"], dev)
    pol = ConstructivePolicy(None, dec, env_name="slap", tanh_clipping=10.0)
    torch.manual_seed(2024)
    out = pol(td, env, phase="train", decode_type="sampling", return_actions=True)
    acts = out["actions"].cpu()
    assert acts.shape == (b, 20)
    assert bool((acts >= 1).all()) and bool((acts < 100).all())  # the depot stays masked
    assert all(len(set(r.tolist())) == 20 for r in acts)  # a location is taken once
    # seeded: the same seed samples the same actions
    _, _, env2, td2 = _pair(gen, dev)
    torch.manual_seed(2024)
    out2 = pol(td2, env2, phase="train", decode_type="sampling", return_actions=True)
    assert torch.equal(out2["actions"], out["actions"])
    ref = constructive_forward(td_ref, ref_env, slap_oracle_logits_fn(dec, dev), actions=acts,
                               tanh_clipping=10.0)
    _check_state(td, ref["td"])
    assert _close(out["reward"], ref["reward"])
    assert _close(out["log_likelihood"], ref["log_likelihood"])


def test_slap_policy_evaluate_matches_reference_loop(dev):
    b = 40
    gen = _slap_instance(b, 11)
    ref_env, td_ref, env, td = _pair(gen, dev)
    dec = SLAPPointerDecoder(gen["locs"], dev)
    acts = _feasible_actions(b, torch.Generator().manual_seed(3))
    ref = constructive_forward(td_ref, ref_env, slap_oracle_logits_fn(dec, dev), actions=acts,
                               tanh_clipping=10.0)
    pol = ConstructivePolicy(None, dec, env_name="slap", tanh_clipping=10.0)
    out = pol(td, env, actions=acts.to(dev), return_actions=True)
    assert torch.equal(out["actions"].cpu(), acts)
    _check_state(td, ref["td"])
    assert _close(out["reward"], ref["reward"])
    assert _close(out["log_likelihood"], ref["log_likelihood"])


def test_slap_policy_config4_slice(dev):
    """BASELINE config 4 (examples/slap.py:75-76, B = 16,384; torch / numpy seeds 1234): the
    whole batch through ConstructivePolicy on the device, the reference loop on the first
    512 instances (the oracle's logits computed as rows of a 16,384-row batch)."""
    b, k = 16384, 512
    torch.manual_seed(1234)
    np.random.seed(1234)
    gen = SLAPGenerator(n_aisles=10, n_locs=10, materialize_dist_mat=False)(b)
    env = SLAPEnv(device=dev)
    td = env.reset(TensorDict({kk: v.to(dev) for kk, v in gen.items()}, [b]))
    dec = SLAPPointerDecoder(gen["locs"], dev)
    pol = ConstructivePolicy(None, dec, env_name="slap", tanh_clipping=10.0)
    out = pol(td, env, phase="test", decode_type="greedy", return_actions=True)
    ref_env = SLAPOracle(seed=0)
    td_ref = ref_env.reset(TD({kk: v[:k].clone() for kk, v in gen.items()}, [k]))
    ref = constructive_forward(td_ref, ref_env, slap_oracle_logits_fn(dec, dev, rows_total=b),
                               decode_type="greedy", tanh_clipping=10.0)
    assert torch.equal(out["actions"][:k].cpu(), ref["actions"])
    for kk in ("assignment", "action_mask", "i", "done"):
        assert torch.equal(td[kk][:k].cpu(), ref["td"][kk]), kk
    assert _close(out["reward"][:k], ref["reward"])
    assert _close(out["log_likelihood"][:k], ref["log_likelihood"])
    # the whole batch: every instance assigned 20 distinct free locations, all done
    a = out["actions"]
    assert bool((td["done"]).all()) and bool((td["i"] == 20).all())
    srt = a.sort(1).values
    assert bool((srt[:, 1:] != srt[:, :-1]).all()) and bool((a >= 1).all())
    assert torch.equal(td["assignment"].long(), a)  # product p took the p-th step's location


def test_slap_hand_episode_known_answer(dev):
    """A hand-built 3-product, 4-location SLAP instance with a known greedy sequence and
    reward (values from the reference semantics, not from the oracle): locations on a
    line x = 0, 1, 2, 3 (y = 0), location 0 the depot (masked at reset); logits favour
    location 3, then 1, then 2; products to_choose = 0, 1, 2 in order; orders
    [[0, 1], [2, 2]] -> reward = -(2*|x3 - x1|) - 0 = -4."""
    locs = torch.tensor([[[0.0, 0.0], [1.0, 0.0], [2.0, 0.0], [3.0, 0.0]]])
    td0 = {"locs": locs, "freq": torch.ones(1, 3, 1),
           "assignment": torch.full((1, 3), -1, dtype=torch.int32),
           "picklist": torch.tensor([[[0, 1], [2, 2]]]),
           "depot_loc_dist": torch.tensor([[0.0, 1.0, 2.0, 3.0]])}
    env = SLAPEnv(device=dev)
    td = env.reset(TensorDict({k: v.to(dev) for k, v in td0.items()}, [1]))
    table = torch.tensor([[0.0, 2.0, 1.0, 3.0]], device=dev)  # 3, then 1, then 2
    pol = ConstructivePolicy(None, LogitsDecoder(lambda t: table), env_name="slap")
    out = pol(td, env, phase="test", decode_type="greedy", return_actions=True)
    assert out["actions"].cpu().tolist() == [[3, 1, 2]]
    assert td["assignment"].cpu().tolist() == [[3, 1, 2]]
    assert td["action_mask"].cpu().tolist() == [[False, False, False, False]]
    assert float(out["reward"][0]) == -4.0


# ------------------------------------------------------------ fused vs two launches
def _cvrp_pair(b, n, dev, seed=5):
    ref_env = CVRPOracle(num_loc=n, seed=seed)
    gen = ref_env.generate([b])
    env = CVRPEnv(generator_params=dict(num_loc=n), device=dev)
    return gen, env


def _count_fused_calls(monkeypatch, env, calls):
    """Count the fused decode + env steps, whichever form runs: the native step glue
    (``native_decode_and_step``) or the Python ``decode_and_step``."""
    real = env.decode_and_step
    monkeypatch.setattr(env, "decode_and_step", lambda *a, **k: calls.append(1) or real(*a, **k))
    native = env.native_decode_and_step()
    if native is not None:
        counted = lambda *a, **k: calls.append(1) or native(*a, **k)  # noqa: E731
        monkeypatch.setattr(env, "native_decode_and_step", lambda: counted)


@pytest.mark.parametrize("name", ["slap", "cvrp"])
@pytest.mark.parametrize("decode_type", ["greedy", "sampling", "multistart_greedy", "evaluate"])
@pytest.mark.parametrize("math", ["certified", "exact"])
def test_fused_decode_env_step_equals_two_launches(dev, monkeypatch, name, decode_type, math):
    """ConstructivePolicy on SLAPEnv / CVRPEnv runs DecodingStrategy.step + env.step as one
    co_slap_decode_step / co_cvrp_decode_step launch (decode_and_step); the result must be
    the two-launch path's bit for bit: actions, log-likelihood, reward and the final state,
    including sampling's RNG use."""
    import rl4co_slap_amd.utils.decoding as dec_mod

    b = 40
    if name == "slap":
        gen = _slap_instance(b, 5)
        dec = SLAPPointerDecoder(gen["locs"], dev)
        acts = _feasible_actions(b, torch.Generator().manual_seed(1)).to(dev)
        keys = ("assignment", "action_mask", "i", "done", "to_choose")
    else:
        n = 23
        gen, _ = _cvrp_pair(b, n, dev)
        locs_all = torch.cat((gen["depot"][:, None], gen["locs"]), 1)
        dec = PointerDecoder(locs_all, dev, depot_env=True)
        acts = None
        keys = ("action_mask", "visited", "used_capacity", "current_node", "done")
        if decode_type == "evaluate":  # the greedy path's actions, re-scored
            decode_type = "evaluate_from_greedy"
    outs, launches = [], []
    for no_fused in (False, True):
        monkeypatch.setattr(dec_mod, "_NO_FUSED", no_fused)
        env = (SLAPEnv(device=dev) if name == "slap"
               else CVRPEnv(generator_params=dict(num_loc=23), device=dev))
        td = env.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()}, [b]))
        pol = ConstructivePolicy(None, dec, env_name=name, tanh_clipping=10.0)
        calls = []
        _count_fused_calls(monkeypatch, env, calls)
        torch.manual_seed(123)
        if decode_type == "evaluate":
            kw = {"actions": acts}
        elif decode_type == "evaluate_from_greedy":
            if acts is None:
                g_env = CVRPEnv(generator_params=dict(num_loc=23), device=dev)
                g_td = g_env.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()},
                                              [b]))
                acts = ConstructivePolicy(None, dec, env_name=name, tanh_clipping=10.0)(
                    g_td, g_env, decode_type="greedy", return_actions=True)["actions"]
            kw = {"actions": acts}
        else:
            kw = {"decode_type": decode_type}
            if name == "slap" and decode_type.startswith("multistart"):
                # the reference's SLAP start nodes are s % 0xFFFFFFFF + 1 (ops.py:158-163):
                # with all L = 100 starts the last one is location 100, out of range -- the
                # reference's mask write raises (slap/env.py:61-62), here the status bit does
                if no_fused:
                    with pytest.raises(IndexError):
                        pol(env.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()},
                                                 [b])), env, phase="test", decode_math=math, **kw)
                kw["num_starts"] = 50
        out = pol(td, env, phase="test", return_actions=True, decode_math=math, **kw)
        outs.append((out, {k: td[k].clone() for k in keys}))
        launches.append(len(calls))
    (a, sa), (b_, sb) = outs
    assert launches[0] > 0 and launches[1] == 0  # the fused path ran, the A/B switch held
    assert torch.equal(a["actions"], b_["actions"])
    assert torch.equal(a["log_likelihood"], b_["log_likelihood"])
    assert torch.equal(a["reward"], b_["reward"])
    for k in keys:
        assert torch.equal(sa[k], sb[k]), k


def test_fused_cvrp_decode_step_kernel_matches_two_launches_direct(dev):
    """co_cvrp_decode_step against co_decode_step + co_cvrp_step on arbitrary (not
    policy-reachable) states: random visited bytes incl. values > 1, used capacity near
    the vehicle capacity, out-of-range evaluate actions, N from 3 to 300, odd strides."""
    from rl4co_slap_amd import _native as nat
    from rl4co_slap_amd.utils.decoding import decode_step

    g = torch.Generator().manual_seed(17)
    for b, n, mode in [(1, 3, "greedy"), (37, 20, "greedy"), (64, 100, "sampling"),
                       (33, 101, "evaluate"), (50, 300, "greedy"), (65, 7, "evaluate")]:
        nc = n + 1
        logits = torch.randn(b, nc, generator=g)
        demand = (torch.randint(1, 10, (b, n), generator=g).float() / 30.0)
        used = (torch.rand(b, 1, generator=g) * 0.9)
        vcap = torch.ones(b, 1)
        visited = (torch.rand(b, nc, generator=g) < 0.3).to(torch.uint8)
        visited[: b // 3, 5 % nc] = 2
        mask = ~((visited[:, 1:] > 0) | (demand + used > vcap))
        mask = torch.cat(((~mask.any(-1, keepdim=True)) | (torch.rand(b, 1, generator=g) < .5),
                          mask), 1)
        mask[:, 0] |= ~mask[:, 1:].any(-1)
        ain = torch.randint(-1, nc + 1, (b,), generator=g) if mode == "evaluate" else None
        L, M, D, U, V, C = (x.to(dev) for x in (logits, mask, demand, used, visited, vcap))
        A = ain.to(dev) if ain is not None else None
        for math_flag in (0, nat.DECODE_CERTIFIED):
            st1 = torch.zeros(1, dtype=torch.int32, device=dev)
            st2 = torch.zeros(1, dtype=torch.int32, device=dev)
            mword = {"greedy": 0, "sampling": 1, "evaluate": 2}[mode] | math_flag
            # two launches
            act2 = torch.empty(b, dtype=torch.int64, device=dev)
            lp2 = torch.empty(b, dtype=torch.float32, device=dev)
            nat.call("co_decode_step", b, nc, nat.ptr(L), nc, nat.ptr(M), 10.0, 1.0, mword,
                     nat.ptr(A), nat.ptr(act2), nat.ptr(lp2), None, 99, 3, nat.ptr(st2),
                     nat.stream_of(L))
            a_env = A if mode == "evaluate" else act2
            o2 = [torch.empty_like(U), torch.empty_like(V), torch.empty(b, 1, dtype=torch.int64,
                  device=dev), torch.empty(b, dtype=torch.bool, device=dev),
                  torch.empty(b, dtype=torch.bool, device=dev), torch.empty_like(M)]
            nat.call("co_cvrp_step", b, n, nat.ptr(a_env), nat.ptr(D), nat.ptr(U), nat.ptr(o2[0]),
                     nat.ptr(C), nat.ptr(V), nat.ptr(o2[1]), nat.ptr(o2[2]), nat.ptr(o2[3]),
                     nat.ptr(o2[4]), nat.ptr(o2[5]), nat.ptr(st2), None, nat.stream_of(L))
            # fused
            act1 = torch.empty(b, dtype=torch.int64, device=dev)
            lp1 = torch.empty(b, dtype=torch.float32, device=dev)
            o1 = [torch.empty_like(x) for x in o2]
            nat.call("co_cvrp_decode_step", b, n, nat.ptr(L), nc, nat.ptr(M), 10.0, 1.0, mword,
                     nat.ptr(A), nat.ptr(act1), nat.ptr(lp1), 99, 3, nat.ptr(D), nat.ptr(U),
                     nat.ptr(o1[0]), nat.ptr(C), nat.ptr(V), nat.ptr(o1[1]), nat.ptr(o1[2]),
                     nat.ptr(o1[3]), nat.ptr(o1[4]), nat.ptr(o1[5]), None, nat.ptr(st1),
                     nat.stream_of(L))
            assert torch.equal(act1, a_env if mode == "evaluate" else act2), (b, n, mode)
            assert torch.equal(lp1, lp2), (b, n, mode)
            for x, y in zip(o1, o2):
                assert torch.equal(x, y), (b, n, mode)
            assert int(st1.item()) == int(st2.item()), (b, n, mode)


@pytest.mark.parametrize("name", ["slap", "cvrp"])
@pytest.mark.parametrize("decode_type", ["greedy", "sampling"])
def test_native_step_glue_equals_python_fused_path(dev, monkeypatch, name, decode_type):
    """The step glue (csrc/pycall/co_torchstep.cpp slap_step_td / cvrp_step_td) and the
    Python decode_and_step launch the same kernel on the same state: same actions, logp,
    reward and final state; the done-poll lower bound recorded on the new state."""
    b = 33
    if name == "slap":
        gen = _slap_instance(b, 21)
        dec = SLAPPointerDecoder(gen["locs"], dev)
        keys = ("assignment", "action_mask", "i", "done", "to_choose")
    else:
        gen, _ = _cvrp_pair(b, 23, dev, seed=8)
        dec = PointerDecoder(torch.cat((gen["depot"][:, None], gen["locs"]), 1), dev,
                             depot_env=True)
        keys = ("action_mask", "visited", "used_capacity", "current_node", "done")
    outs = []
    reads = []
    base_poll = RL4COEnvBase.poll_done
    monkeypatch.setattr(RL4COEnvBase, "poll_done",
                        lambda self, td: reads.append(1) or base_poll(self, td))
    for native in (True, False):
        env = (SLAPEnv(device=dev) if name == "slap"
               else CVRPEnv(generator_params=dict(num_loc=23), device=dev))
        if not native:
            monkeypatch.setattr(env, "native_decode_and_step", lambda: None)
        elif env.native_decode_and_step() is None:
            pytest.skip("step glue not built for this torch / interpreter")
        td = env.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()}, [b]))
        pol = ConstructivePolicy(None, dec, env_name=name, tanh_clipping=10.0)
        torch.manual_seed(5)
        outs.append((pol(td, env, phase="test", decode_type=decode_type, return_actions=True),
                     {k: td[k].clone() for k in keys}))
        if name == "slap":  # done known on the host (uniform i): the loop's poll reads nothing
            assert env._known_i(td["done"]) == 1 and not reads
    (a, sa), (b_, sb) = outs
    for k in ("actions", "log_likelihood", "reward"):
        assert torch.equal(a[k], b_[k]), k
    for k in keys:
        assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize("env_name", ["cvrp", "slap"])
def test_fused_env_decode_certified_actions_equal_exact_on_near_ties(dev, env_name):
    """The fused decode + env steps in the certified math (the drop-in default) pick the
    exact path's greedy action on adversarial rows -- near-ties straddling the
    certification margin before and after the pick (the fallback's tier 1), ties in one
    lane, exact / saturated ties, NaN / inf / all-masked rows (tier 2) -- with logp within
    1e-5 of the exact one; the env state follows the action."""
    from test_gpu_decode_certified import _adversarial_logits

    from rl4co_slap_amd import _native as nat

    g = torch.Generator().manual_seed(23)
    b = 2048
    n = 100 if env_name == "slap" else 100  # SLAP: L locations; CVRP: N customers (N+1 columns)
    nc = n if env_name == "slap" else n + 1
    x, m = _adversarial_logits(b, nc, 41, dev)
    if env_name == "cvrp":
        m[:, 0] = True  # a feasible depot keeps every row's mask a reachable CVRP mask
    for clip in (10.0, 0.0):
        # the exact reference action / logp (co_decode_step, no math flag)
        act_e = torch.empty(b, dtype=torch.int64, device=dev)
        lp_e = torch.empty(b, dtype=torch.float32, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        nat.call("co_decode_step", b, nc, nat.ptr(x), nc, nat.ptr(m), clip, 1.0, 0, None,
                 nat.ptr(act_e), nat.ptr(lp_e), None, 0, 0, nat.ptr(st), nat.stream_of(x))
        act = torch.empty(b, dtype=torch.int64, device=dev)
        lp = torch.empty(b, dtype=torch.float32, device=dev)
        st = torch.zeros(1, dtype=torch.int32, device=dev)
        if env_name == "cvrp":
            demand = (torch.randint(1, 10, (b, n), generator=g).float() / 30.0).to(dev)
            used = torch.zeros(b, 1, device=dev)
            vcap = torch.ones(b, 1, device=dev)
            vis = (~m).to(torch.uint8)
            vis[:, 0] = 1
            outs = [torch.empty_like(used), torch.empty_like(vis),
                    torch.empty(b, 1, dtype=torch.int64, device=dev),
                    torch.empty(b, dtype=torch.bool, device=dev),
                    torch.empty(b, dtype=torch.bool, device=dev), torch.empty_like(m)]
            nat.call("co_cvrp_decode_step", b, n, nat.ptr(x), nc, nat.ptr(m), clip, 1.0,
                     nat.DECODE_CERTIFIED, None, nat.ptr(act), nat.ptr(lp), 0, 0, nat.ptr(demand),
                     nat.ptr(used), nat.ptr(outs[0]), nat.ptr(vcap), nat.ptr(vis),
                     nat.ptr(outs[1]), nat.ptr(outs[2]), nat.ptr(outs[3]), nat.ptr(outs[4]),
                     nat.ptr(outs[5]), None, nat.ptr(st), nat.stream_of(x))
            rows = torch.arange(b, device=dev)
            ok = act < nc
            assert bool((outs[1][rows[ok], act[ok]] == 1).all())  # the action's node visited
        else:
            p = 20
            tc = torch.rand(b, p, generator=g).to(dev)
            asg_in = torch.full((b, p), -1, dtype=torch.int32, device=dev)
            asg_out = torch.empty_like(asg_in)
            i_in = torch.randint(0, p, (b, 1), generator=g).to(dev)
            outs = [asg_out, torch.empty_like(m), torch.empty_like(i_in),
                    torch.empty(b, 1, dtype=torch.bool, device=dev),
                    torch.empty(b, 1, dtype=torch.bool, device=dev)]
            nat.call("co_slap_decode_step", b, nc, p, nat.ptr(x), nc, nat.ptr(m), clip, 1.0,
                     nat.DECODE_CERTIFIED, None, nat.ptr(act), nat.ptr(lp), 0, 0, nat.ptr(tc), p,
                     nat.ptr(asg_in), nat.ptr(asg_out), nat.ptr(outs[1]), nat.ptr(i_in),
                     nat.ptr(outs[2]), nat.ptr(outs[3]), nat.ptr(outs[4]), None, nat.ptr(st),
                     nat.stream_of(x))
            assert torch.equal(outs[2], i_in + 1)
        torch.cuda.synchronize()
        assert torch.equal(act, act_e), clip
        fin = torch.isfinite(lp_e)
        assert torch.equal(fin, torch.isfinite(lp))
        assert bool(((lp - lp_e)[fin].abs() <= 1e-5 * lp_e[fin].abs().clamp(min=1)).all()), clip
