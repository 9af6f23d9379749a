"""The fused decode + env step applies only to the env's own transition: an env
subclass that overrides ``_step`` (as the reference's CVRPTWEnv / SDVRPEnv do on top of
CVRPEnv) inherits ``decode_and_step`` but not the transition it fuses, so the decode loop
must take the two-call path and run the subclass's ``_step`` every step."""
import pytest
import torch

from rl4co_slap_amd import TensorDict
from rl4co_slap_amd.envs import CVRPEnv, SLAPEnv, TSPEnv
from rl4co_slap_amd.rollout import ConstructivePolicy
from rl4co_slap_amd.rollout.constructive import LogitsDecoder
from rl4co_slap_amd.utils.decoding import Greedy, _own_step


class CountingCVRP(CVRPEnv):
    """A CVRP variant with its own transition (here: the parent's, counted)."""

    def __init__(self, **kw):
        super().__init__(**kw)
        self.calls = 0

    def _step(self, td):
        self.calls += 1
        return super()._step(td)


class CountingTSP(TSPEnv):
    def _step(self, td):
        return super()._step(td)


def test_own_step_gate_cpu():
    for cls in (TSPEnv, CVRPEnv, SLAPEnv):
        assert _own_step(cls(device="cpu")), cls
    assert not _own_step(CountingCVRP(device="cpu"))
    assert not _own_step(CountingTSP(device="cpu"))
    env = TSPEnv(device="cpu")
    env._step = lambda td: td  # replaced on the instance
    assert not _own_step(env)


def test_step_env_fused_declines_overridden_step_cpu():
    env = CountingCVRP(device="cpu")
    s = Greedy()
    td = TensorDict({"action_mask": torch.ones(2, 3, dtype=torch.bool)}, [2])
    assert s.step_env_fused(torch.zeros(2, 3), td["action_mask"], td, env) is None
    assert s._fused[1] is None and s._fused[2] is None


@pytest.mark.gpu
def test_overridden_step_runs_every_step(dev):
    torch.manual_seed(5)
    b, n = 96, 20
    la = torch.rand(b, n + 1, 2)
    data = {"depot": la[:, 0].contiguous().to(dev), "locs": la[:, 1:].contiguous().to(dev),
            "demand": (((torch.rand(b, n) * 9).int() + 1).float() / 50.0).to(dev)}
    logits = torch.randn(b, n + 1).to(dev)
    outs = []
    for cls in (CVRPEnv, CountingCVRP):
        env = cls(generator_params=dict(num_loc=n), device=dev)
        pol = ConstructivePolicy(None, LogitsDecoder(lambda td: logits), env_name="cvrp")
        td = env.reset(TensorDict(dict(data), [b]))
        outs.append((env, pol(td, env, phase="test", decode_type="greedy", return_actions=True)))
    (_, base), (sub, over) = outs
    assert sub.calls == over["actions"].shape[1]  # the subclass's _step ran every step
    assert torch.equal(base["actions"], over["actions"])
    assert torch.equal(base["reward"], over["reward"])
