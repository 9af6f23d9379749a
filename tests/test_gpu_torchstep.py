"""The drop-in loop's step glue (csrc/pycall/co_torchstep.cpp): the same launches as the
Python step path with the outputs allocated natively.  Every output must equal the Python
path's bit for bit (same kernels, same arguments), the glue must be the path that runs on
the GPU box, and it must step aside (return None) whenever its operands do not fit."""
import pytest
import torch

from rl4co_slap_amd import TensorDict
from rl4co_slap_amd import _native as nat
from rl4co_slap_amd.envs import CVRPEnv, TSPEnv
from rl4co_slap_amd.rollout import ConstructivePolicy, LogitsDecoder

from am_pointer import PointerDecoder

pytestmark = pytest.mark.gpu


@pytest.fixture
def python_path():
    """Run the body with the glue disabled (the Python step path), then restore it."""
    saved = nat._tstep

    class _Off:
        def __enter__(self):
            nat._tstep = False

        def __exit__(self, *exc):
            nat._tstep = saved

    return _Off


def test_glue_is_loaded(dev):
    ts = nat.torchstep()
    assert ts is not None, "the step glue module must load on the GPU box"


def _run(env_cls, gen, dev, decode_type, dec_fn, name, **kw):
    env = env_cls(generator_params=dict(num_loc=kw.pop("n")), device=dev)
    td = env.reset(TensorDict({k: v.clone().to(dev) for k, v in gen.items()},
                              [gen[next(iter(gen))].shape[0]]))
    torch.manual_seed(77)
    pol = ConstructivePolicy(None, dec_fn, env_name=name, tanh_clipping=10.0)
    return pol(td, env, phase="test", decode_type=decode_type, return_actions=True, **kw)


def _same(a, b):
    for k in ("actions", "reward", "log_likelihood"):
        x, y = a[k], b[k]
        assert x.dtype == y.dtype and x.shape == y.shape, k
        assert torch.equal(x.view(torch.int32) if x.is_floating_point() else x,
                           y.view(torch.int32) if y.is_floating_point() else y), k


@pytest.mark.parametrize("decode_type", ["greedy", "sampling", "multistart_greedy"])
def test_tsp_glue_equals_python_path(dev, python_path, decode_type):
    b, n = 96, 30
    gen = {"locs": torch.rand(b, n, 2, generator=torch.Generator().manual_seed(4))}
    dec = PointerDecoder(gen["locs"], dev)
    glue = _run(TSPEnv, gen, dev, decode_type, dec, "tsp", n=n)
    with python_path():
        ref = _run(TSPEnv, gen, dev, decode_type, dec, "tsp", n=n)
    _same(glue, ref)


@pytest.mark.parametrize("decode_type", ["greedy", "sampling"])
def test_cvrp_glue_equals_python_path(dev, python_path, decode_type):
    b, n = 64, 20
    g = torch.Generator().manual_seed(8)
    gen = {"depot": torch.rand(b, 2, generator=g), "locs": torch.rand(b, n, 2, generator=g),
           "demand": ((torch.rand(b, n, generator=g) * 9).int() + 1).float() / 30.0}
    dec = PointerDecoder(torch.cat([gen["depot"][:, None], gen["locs"]], 1), dev,
                         depot_env=True)
    glue = _run(CVRPEnv, gen, dev, decode_type, dec, "cvrp", n=n)
    with python_path():
        ref = _run(CVRPEnv, gen, dev, decode_type, dec, "cvrp", n=n)
    _same(glue, ref)


def test_glue_evaluate_mode_and_logits_views(dev, python_path):
    """Evaluate mode (action_in) and a strided logits view (row stride > N) take the glue
    with the same results; int32 actions make it step aside (the Python path casts)."""
    b, n = 40, 25
    locs = torch.rand(b, n, 2, generator=torch.Generator().manual_seed(9))
    wide = torch.randn(b, n + 7, generator=torch.Generator().manual_seed(10)).to(dev)
    acts = torch.rand(b, n, generator=torch.Generator().manual_seed(11)).argsort(1).to(dev)
    outs = []
    for off in (False, True):
        for a in (acts, acts.int()):
            env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
            td = env.reset(TensorDict({"locs": locs.to(dev)}, [b]))
            pol = ConstructivePolicy(None, LogitsDecoder(lambda t: wide[:, :n]), env_name="tsp")
            if off:
                with python_path():
                    outs.append(pol(td, env, actions=a, return_actions=True))
            else:
                outs.append(pol(td, env, actions=a, return_actions=True))
    _same(outs[0], outs[2])  # int64 actions: glue vs Python path
    _same(outs[1], outs[3])  # int32 actions: both on the Python path
    assert torch.equal(outs[0]["log_likelihood"], outs[1]["log_likelihood"])


def test_glue_steps_aside(dev):
    ts = nat.torchstep()
    b, n = 8, 10
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    logits = torch.randn(b, n, device=dev)
    mask = torch.ones(b, n, dtype=torch.bool, device=dev)
    i = torch.zeros(b, 1, dtype=torch.int64, device=dev)
    # CPU operands, half logits, a non-contiguous mask: None (the Python path handles them)
    assert ts.tsp_decode_step(logits.cpu(), mask.cpu(), i.cpu(), None, None, st.cpu(), 0.0, 1.0,
                              0, 0, 0, 1) is None
    assert ts.tsp_decode_step(logits.half(), mask, i, None, None, st, 0.0, 1.0, 0, 0, 0,
                              1) is None
    assert ts.decode_step(logits, mask.t().contiguous().t(), None, st, 0.0, 1.0, 0, 0, 0,
                          False) is None
    assert ts.decode_step(logits.cpu(), None, None, None, 0.0, 1.0, 0, 0, 0, False) is None
    # a bad mode is the C ABI's error code, raised by the caller
    rc = ts.decode_step(logits, mask, None, st, 0.0, 1.0, 7, 0, 0, False)
    assert type(rc) is int and rc != 0
    # outputs are distinct, 256-byte aligned regions
    r = ts.tsp_decode_step(logits, mask, i, None, None, st, 0.0, 1.0, 0, 0, 0, 1)
    ptrs = sorted(t.data_ptr() for t in r)
    assert len(set(ptrs)) == len(ptrs) and all(p % 256 == 0 for p in ptrs)
    torch.cuda.synchronize()
    assert int(st.item()) == 0


def test_stale_records_fall_back(dev, python_path):
    """A decoder that touches td["i"] / td["action_mask"] in place (version bump) voids the
    host-side records on them: the native step steps aside, the loop takes the two-launch
    path with the device-side first-node test and polls `done` -- same results as the
    Python path."""
    b, n = 33, 12
    locs = torch.rand(b, n, 2, generator=torch.Generator().manual_seed(21))
    tab = torch.randn(n + 2, b, n, generator=torch.Generator().manual_seed(22)).to(dev)

    def run():
        env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
        td = env.reset(TensorDict({"locs": locs.to(dev)}, [b]))
        it = iter(range(10 ** 6))

        def fn(t):
            k = next(it)
            if k in (0, 4):
                t["i"].add_(0)
            if k == 6:
                t["action_mask"].mul_(True)
            return tab[k]

        pol = ConstructivePolicy(None, LogitsDecoder(fn), env_name="tsp")
        return pol(td, env, phase="test", decode_type="greedy", return_actions=True)

    glue = run()
    with python_path():
        ref = run()
    _same(glue, ref)
    assert glue["actions"].shape == (b, n)


def test_inplace_state_writes_off_gives_same_results(dev):
    """the SLAP step's in-place assignment / state-block writes rest on
    CPython reference counts; with them turned off (what a free-threaded or 3.12+ build
    compiles to, or CO_NO_INPLACE=1) every step takes fresh storages, with the same results."""
    import numpy as np

    from rl4co_slap_amd.envs import SLAPEnv
    from rl4co_slap_amd.envs.slap import SLAPGenerator

    ts = nat.torchstep()
    assert ts is not None
    b = 64
    torch.manual_seed(5)
    np.random.seed(5)
    data = SLAPGenerator(materialize_dist_mat=False)(b).to(dev)
    logits = torch.randn(b, 100, generator=torch.Generator().manual_seed(9)).to(dev)
    env = SLAPEnv(device=dev)
    pol = ConstructivePolicy(None, LogitsDecoder(lambda t: logits), env_name="slap")

    def episode():
        td = env.reset(TensorDict(dict(data.items()), [b]))
        out = pol(td, env, phase="test", decode_type="greedy", return_actions=True)
        return out, td

    from rl4co_slap_amd.utils.decoding import _MODES, math_flags

    mword = _MODES["greedy"] | math_flags("certified")
    native = env.native_decode_and_step()
    st = torch.zeros(2, dtype=torch.int32, device=dev)

    def ptrs_over_steps():
        """storage addresses of the td's assignment / action_mask after steps 1, 2, 3 (the
        test holds no reference to the tensors themselves)"""
        td = env.reset(TensorDict(dict(data.items()), [b]))
        seen = []
        for k in range(3):
            out = native(td, logits, mword, 1.0, 0.0, None, 0, k, st, "action")
            assert out is not None and type(out) is not int
            del out
            # data_ptr, not untyped_storage(): a Python storage object can keep a
            # reference that the glue's use-count test would see
            seen.append((td["assignment"].data_ptr(), td["action_mask"].data_ptr()))
        return seen

    on, td_on = episode()
    seen_on = ptrs_over_steps()
    assert seen_on[1][0] == seen_on[0][0] and seen_on[2][1] == seen_on[1][1]  # in place
    prev = ts.set_inplace(False)
    try:
        assert ts.inplace_policy()[1] is False
        seen_off = ptrs_over_steps()
        assert seen_off[1][0] != seen_off[0][0] and seen_off[2][1] != seen_off[1][1]  # fresh
        off, td_off = episode()
    finally:
        ts.set_inplace(prev)
    _same(on, off)
    for k in ("assignment", "action_mask", "i", "done"):
        assert torch.equal(td_on[k], td_off[k]), k


@pytest.mark.parametrize("env_name", ["tsp", "cvrp", "slap"])
def test_fast_step_equals_python_closure(dev, env_name, monkeypatch):
    """The greedy loop's per-step closure in C (co_torchstep.cpp: fast_step) against the
    Python closure it replaces (CO_NO_FAST_STEP): the same actions, rewards and
    log-likelihoods bit for bit, and the C closure is the one bound on the GPU box."""
    import numpy as np

    from rl4co_slap_amd.envs import SLAPEnv
    from rl4co_slap_amd.envs.slap import SLAPGenerator
    from rl4co_slap_amd.utils import decoding as D

    b = 48
    if env_name == "slap":
        torch.manual_seed(6)
        np.random.seed(6)
        data = dict(SLAPGenerator(materialize_dist_mat=False)(b).to(dev).items())
        env_f, na = (lambda: SLAPEnv(device=dev)), 100
    elif env_name == "tsp":
        data = {"locs": torch.rand(b, 40, 2, generator=torch.Generator().manual_seed(7)).to(dev)}
        env_f, na = (lambda: TSPEnv(generator_params=dict(num_loc=40), device=dev)), 40
    else:
        g = torch.Generator().manual_seed(8)
        data = {"depot": torch.rand(b, 2, generator=g).to(dev),
                "locs": torch.rand(b, 30, 2, generator=g).to(dev),
                "demand": (((torch.rand(b, 30, generator=g) * 9).int() + 1).float() / 30.0).to(dev)}
        env_f, na = (lambda: CVRPEnv(generator_params=dict(num_loc=30), device=dev)), 31
    tab = torch.randn(400, b, na, generator=torch.Generator().manual_seed(12)).to(dev)
    bound = []
    orig = D.DecodingStrategy.fast_stepper

    def spy(self, env):
        f = orig(self, env)
        bound.append(f)
        return f

    monkeypatch.setattr(D.DecodingStrategy, "fast_stepper", spy)

    def run():
        env = env_f()
        td = env.reset(TensorDict({k: v.clone() for k, v in data.items()}, [b]))
        it = iter(range(10 ** 6))
        pol = ConstructivePolicy(None, LogitsDecoder(lambda t: tab[next(it)]), env_name=env_name,
                                 tanh_clipping=10.0)
        return pol(td, env, phase="test", decode_type="greedy", return_actions=True)

    c = run()
    assert bound and getattr(bound[-1], "func", None) is nat.torchstep().fast_step
    monkeypatch.setattr(D, "_NO_FAST_STEP", True)
    py = run()
    assert bound[-1] is not None and getattr(bound[-1], "func", None) is None
    _same(c, py)

