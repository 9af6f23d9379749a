"""GPU parity for the ConstructivePolicy decode loop (constructive/base.py:158-276) on the
device decoding strategy + env kernels, against the oracle's restatement of the same loop
(oracle/rollout.py constructive_forward).  The policy network is replaced by a
deterministic heuristic head (negative distance to the current node) evaluated with the
same torch elementwise ops on both sides, so greedy choices are compared bit-exact."""
import pytest
import torch

from oracle.envs import CVRPOracle, TSPOracle
from oracle.rollout import constructive_forward
from oracle.td import TD
from rl4co_slap_amd import TensorDict
from rl4co_slap_amd.envs import CVRPEnv, TSPEnv
from rl4co_slap_amd.rollout import ConstructivePolicy, LogitsDecoder

pytestmark = pytest.mark.gpu


def neg_dist_logits(td):
    locs = td["locs"]
    cur = td["current_node"].reshape(-1)
    p = locs.gather(1, cur[:, None, None].expand(-1, 1, 2))
    d = locs - p
    return -torch.sqrt(d[..., 0] * d[..., 0] + d[..., 1] * d[..., 1])


def _pair(name, b, n, seed, dev):
    if name == "tsp":
        ref_env, env = TSPOracle(num_loc=n, seed=seed), TSPEnv(
            generator_params=dict(num_loc=n), seed=seed, device=dev)
    else:
        ref_env, env = CVRPOracle(num_loc=n, seed=seed), CVRPEnv(
            generator_params=dict(num_loc=n), seed=seed, device=dev)
    gen = ref_env.generate([b])
    td_ref = ref_env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
    td = env.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()}, [b]))
    return ref_env, td_ref, env, td


@pytest.mark.parametrize("name,b,n", [("tsp", 64, 20), ("tsp", 33, 50), ("cvrp", 40, 20)])
@pytest.mark.parametrize("decode_type", ["greedy", "multistart_greedy"])
def test_policy_greedy_matches_oracle(dev, name, b, n, decode_type):
    ref_env, td_ref, env, td = _pair(name, b, n, 100 + n, dev)
    ref = constructive_forward(td_ref, ref_env, neg_dist_logits, decode_type=decode_type)
    pol = ConstructivePolicy(None, LogitsDecoder(neg_dist_logits), env_name=name)
    out = pol(td, env, phase="test", decode_type=decode_type, return_actions=True)
    assert torch.equal(out["actions"].cpu(), ref["actions"])
    r, rr = out["reward"].cpu(), ref["reward"]
    assert ((r - rr).abs() <= 1e-5 * rr.abs().clamp(min=1)).all()
    ll, lr = out["log_likelihood"].cpu(), ref["log_likelihood"]
    assert ((ll - lr).abs() <= 1e-4 * lr.abs().clamp(min=1)).all()


def test_policy_evaluate_and_sampling_consistency(dev):
    b, n = 48, 20
    ref_env, td_ref, env, td = _pair("tsp", b, n, 9, dev)
    acts = torch.rand(b, n, generator=torch.Generator().manual_seed(3)).argsort(1)
    ref = constructive_forward(td_ref, ref_env, neg_dist_logits, actions=acts)
    pol = ConstructivePolicy(None, LogitsDecoder(neg_dist_logits), env_name="tsp")
    out = pol(td, env, actions=acts.to(dev), return_actions=True, return_entropy=True)
    assert torch.equal(out["actions"].cpu(), acts)
    assert torch.allclose(out["log_likelihood"].cpu(), ref["log_likelihood"], rtol=1e-4,
                          atol=1e-4)
    assert torch.isfinite(out["entropy"]).all()
    # sampling: valid tours, and evaluate mode re-scores them to the same log-likelihood
    _, _, env2, td2 = _pair("tsp", b, n, 9, dev)
    smp = pol(td2, env2, phase="train", return_actions=True)  # train -> sampling
    a = smp["actions"]
    assert torch.equal(a.sort(1).values.cpu(), torch.arange(n).expand(b, n))
    _, _, env3, td3 = _pair("tsp", b, n, 9, dev)
    ev = pol(td3, env3, actions=a)
    assert torch.allclose(ev["log_likelihood"], smp["log_likelihood"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name,b,n,bw", [("tsp", 8, 10, 4), ("tsp", 5, 20, 20), ("cvrp", 6, 12, 3)])
@pytest.mark.parametrize("select_best", [True, False])
def test_policy_beam_search_matches_oracle(dev, name, b, n, bw, select_best):
    ref_env, td_ref, env, td = _pair(name, b, n, 300 + n, dev)
    ref = constructive_forward(td_ref, ref_env, neg_dist_logits, decode_type="beam_search",
                               beam_width=bw, select_best=select_best)
    pol = ConstructivePolicy(None, LogitsDecoder(neg_dist_logits), env_name=name)
    out = pol(td, env, phase="test", decode_type="beam_search", beam_width=bw,
              select_best=select_best, return_actions=True)
    assert torch.equal(out["actions"].cpu(), ref["actions"])
    r, rr = out["reward"].cpu(), ref["reward"]
    assert ((r - rr).abs() <= 1e-5 * rr.abs().clamp(min=1)).all()
    ll, lr = out["log_likelihood"].cpu(), ref["log_likelihood"]
    assert ((ll - lr).abs() <= 1e-4 * lr.abs().clamp(min=1)).all()


def test_policy_multisampling(dev):
    """decode_type="multisampling" with multisample=True: the td is batchified num_starts
    times without start-node selection (decoding.py:271-313) and every sample is a
    valid tour; select_best keeps the best sample per instance."""
    b, n, s = 16, 20, 4
    _, _, env, td = _pair("tsp", b, n, 7, dev)
    pol = ConstructivePolicy(None, LogitsDecoder(neg_dist_logits), env_name="tsp")
    out = pol(td, env, decode_type="multisampling", multisample=True, num_starts=s,
              return_actions=True)
    a = out["actions"]
    assert a.shape == (s * b, n)
    assert torch.equal(a.sort(1).values.cpu(), torch.arange(n).expand(s * b, n))
    _, _, env2, td2 = _pair("tsp", b, n, 7, dev)
    best = pol(td2, env2, decode_type="multisampling", multisample=True, num_starts=s,
               select_best=True, return_actions=True)
    assert best["actions"].shape == (b, n) and best["reward"].shape == (b,)
