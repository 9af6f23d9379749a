"""CPU-side checks: the C-ABI library loads and exports every symbol of
include/co_env.h; generators reproduce the reference RNG streams; registry and the
TensorDict stand-in behave like the reference API.  No kernel runs here."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import rl4co_slap_amd as ra
from oracle.envs import CVRPOracle, SLAPOracle, TSPOracle
from rl4co_slap_amd import _native
from rl4co_slap_amd.envs import CVRPEnv, SLAPEnv, TSPEnv, get_env
from rl4co_slap_amd.td import TensorDict
from rl4co_slap_amd.utils.ops import batchify, unbatchify

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "co_env.h")).read()
    return sorted(set(re.findall(r"^(?:int|const char\*)\s+(co_\w+)\(", src, re.M)))


def test_library_exports_every_header_symbol():
    lib = _native.load()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _native.exported_symbols(), f"{s} not bound in _native"
    assert b"gfx950" in lib.co_build_info()


def test_library_is_gfx950_code_object():
    data = open(_native.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_invalid_args_return_codes_without_gpu():
    lib = _native.load()
    # argument validation happens before any launch: these never touch a device
    assert lib.co_tsp_step(-1, 10, *([None] * 10), 0, None, None, None) == -1
    assert lib.co_decode_step(4, 10, None, 10, None, 0.0, 1.0, 7, None, None, None, None, 0, 0,
                              None, None) == -3
    assert lib.co_tsp_reset(0, 10, None, None, None, None, None, None) == 0  # empty batch is a no-op


def test_generators_match_reference_streams():
    for ours, ref, kw in [(TSPEnv, TSPOracle, dict(num_loc=20)), (CVRPEnv, CVRPOracle, dict(num_loc=20))]:
        e1 = ours(generator_params=kw, seed=1234, device="cpu")
        a = e1.generator(8)
        e2 = ref(seed=1234, **kw)
        b = e2.generate([8])
        for k in b:
            assert torch.equal(a[k], b[k]), k


def test_slap_generator_matches_reference_loop_order():
    torch.manual_seed(7)
    np.random.seed(7)
    ours = SLAPEnv(seed=7, device="cpu").generator(6)
    torch.manual_seed(7)
    np.random.seed(7)
    ref = SLAPOracle(seed=7).generate([6])
    for k in ref:
        assert torch.equal(ours[k], ref[k]), k
        assert ours[k].dtype == ref[k].dtype, k


def test_registry():
    assert set(ra.ENV_REGISTRY) == {"tsp", "cvrp", "slap"}
    assert isinstance(get_env("tsp", device="cpu"), TSPEnv)
    with pytest.raises(ValueError):
        get_env("ffsp")


def test_cpu_tensors_need_the_host_build(monkeypatch):
    """CPU TensorDicts run on the host build of the C ABI (libco_env_host.so), never on a
    Python/oracle fallback: without that library they raise."""
    from rl4co_slap_amd import _native as nat

    monkeypatch.setattr(nat, "HOST_LIB_PATH", "/nonexistent/libco_env_host.so")
    monkeypatch.setattr(nat, "_host", None)
    env = TSPEnv(generator_params=dict(num_loc=5), device="cpu")
    with pytest.raises(nat.NativeUnavailable, match="host library"):
        env.reset(batch_size=[2])


def test_td_standin_batchify_roundtrip():
    td = TensorDict({"locs": torch.randn(3, 5, 2), "i": torch.zeros(3, 1, dtype=torch.int64)}, [3])
    tb = batchify(td, 4)
    assert tb.batch_size == (12,) and tb["locs"].shape == (12, 5, 2)
    assert torch.equal(tb["locs"][2 * 3 + 1], td["locs"][1])
    tu = unbatchify(tb, 4)
    assert tu.batch_size == (3, 4) and torch.equal(tu["locs"][:, 3], td["locs"])


def test_fastcall_path_matches_ctypes_on_the_host_build():
    """The METH_FASTCALL trampoline (csrc/pycall/co_fastcall.cpp) is built, carries a kinds
    string for every bound entry point, and gives the ctypes path's results (a host CVRP
    reset: int64, pointer and float arguments, None as the null stream)."""
    fast = _native._fastcall()
    assert fast is not None, "_co_fastcall module missing: run the build"
    assert _native.FASTCALL_PATH.endswith(__import__("sysconfig").get_config_var("EXT_SUFFIX"))
    host = fast.table("host")  # the host table alone: the device library is not needed
    invoke = fast.invoke
    dev = fast.table("dev")
    assert set(dev) == set(_native._SIGS)  # every int-returning entry point
    assert set(host) == set(_native.HOST_SYMBOLS)
    assert all(len(k) == len(_native._SIGS[n]) for n, (_, k) in dev.items())
    lib = _native.load_host()
    b, n = 5, 7
    gen = torch.Generator().manual_seed(0)
    depot = torch.rand(b, 2, generator=gen)
    locs = torch.rand(b, n, 2, generator=gen)
    dem = torch.rand(b, n, generator=gen) * 0.3
    outs = []
    for path in ("fast", "ctypes"):
        o = {"locs": torch.empty(b, n + 1, 2), "cur": torch.empty(b, dtype=torch.int64),
             "used": torch.empty(b), "vcap": torch.empty(b), "vis": torch.empty(b, n + 1,
                                                                                 dtype=torch.uint8),
             "mask": torch.empty(b, n + 1, dtype=torch.bool)}
        args = (b, n, depot.data_ptr(), locs.data_ptr(), dem.data_ptr(), 0.75,
                o["locs"].data_ptr(), o["cur"].data_ptr(), o["used"].data_ptr(),
                o["vcap"].data_ptr(), o["vis"].data_ptr(), o["mask"].data_ptr(), None)
        if path == "fast":
            addr, kinds = host["co_cvrp_reset"]
            assert invoke(addr, kinds, *args) == 0
        else:
            assert lib.co_cvrp_reset(*args) == 0
        outs.append(o)
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
    assert (outs[0]["vcap"] == 0.75).all()
    # an error status comes back through both paths alike
    addr, kinds = host["co_cvrp_reset"]
    bad = (-1, n) + (0,) * 3 + (1.0,) + (0,) * 7
    assert invoke(addr, kinds, *bad) == lib.co_cvrp_reset(*bad) != 0


def test_fastcall_falls_back_to_ctypes_when_a_library_cannot_load(monkeypatch):
    """A library that fails to load leaves its fast-call table empty: calls then take the
    ctypes path, which raises the library's own error (no exception from the table)."""
    fc = _native._FastCall(invoke=None)

    def boom():
        raise OSError("cannot load")

    monkeypatch.setattr(_native, "load", boom)
    assert fc.table("dev") == {}
    assert set(fc.table("host")) == set(_native.HOST_SYMBOLS)


def test_step_glue_inplace_guard():
    """the step glue's in-place state writes (a td-held tensor rewritten
    when CPython's reference count says nothing else holds it) are compiled in only for the
    interpreter kind they were tested on (GIL build, < 3.12), can be switched off at run time,
    and CO_NO_INPLACE=1 forces the fresh-storage fallback from import on."""
    import subprocess
    import sys
    import sysconfig

    ts = _native.torchstep()
    if ts is None:
        pytest.skip("step glue not built")
    build_ok, enabled = ts.inplace_policy()
    expect = sys.version_info < (3, 12) and not sysconfig.get_config_var("Py_GIL_DISABLED")
    assert build_ok is expect
    assert enabled is (expect and not os.environ.get("CO_NO_INPLACE"))
    prev = ts.set_inplace(False)
    try:
        assert ts.inplace_policy() == (build_ok, False)
        ts.set_inplace(True)
        assert ts.inplace_policy() == (build_ok, build_ok)  # never on where the build forbids it
    finally:
        ts.set_inplace(prev)
    code = ("from rl4co_slap_amd import _native as nat; p = nat.torchstep().inplace_policy(); "
            "print(int(p[0]), int(p[1]))")
    env = dict(os.environ, CO_NO_INPLACE="1")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True,
                         cwd=ROOT, timeout=300)
    assert out.returncode == 0, out.stderr
    assert out.stdout.split()[-2:] == [str(int(expect)), "0"]


def test_fast_step_steps_aside():
    """fast_step returns False, having done nothing, for a td of another type or a mask
    that is not the td's action_mask; and it checks its list arguments."""
    ts = _native.torchstep()
    if ts is None:
        pytest.skip("step glue module not built")
    fs = ts.fast_step
    calls = []

    def native(*a):
        calls.append(a)
        return None

    class Strat:
        _step_idx = 3

    s = Strat()
    mask = torch.ones(2, 3, dtype=torch.bool)
    td = TensorDict({"action_mask": mask}, [2])
    acts, lps = [], []
    args = (native, TensorDict, 0, 1.0, 0.0, None, "action", acts, lps, s, "_step_idx",
            _native.check_rc)
    assert fs(*args, dict(td), None, mask) is False  # not a TensorDict
    assert fs(*args, td, None, mask.clone()) is False  # not the td's mask
    assert not calls
    assert fs(*args, td, None, mask) is False  # the glue stepped aside (None)
    assert len(calls) == 1 and calls[0][7] == 3 and s._step_idx == 3 and not acts
    with pytest.raises(RuntimeError):  # an error code goes to check_rc
        fs(lambda *a: 5, *args[1:], td, None, mask)
    fs(lambda *a: ("a", "l"), *args[1:], td, None, mask)
    assert s._step_idx == 4 and acts == ["a"] and lps == ["l"]
    with pytest.raises(TypeError):
        fs(*args[:7], (), lps, *args[9:], td, None, mask)
