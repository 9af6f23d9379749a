"""ctypes binding of the gfx950 C-ABI library (``include/co_env.h``).

The library is the product: every env/decode/gather call on a device tensor goes
through it.  There is no CPU or PyTorch fallback -- if the library is missing or
the tensors are not on a HIP device, calls raise.

``torch`` is imported before the library is loaded so that ``libamdhip64.so.7``
resolves (by SONAME) to the HIP runtime torch already mapped: one runtime per
process, so torch streams and allocations are valid handles for the kernels.
"""
from __future__ import annotations

import ctypes
import os
import warnings
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "_lib", "libco_env.so")
_PRODUCT_LIB_PATH = LIB_PATH

_i64, _i32, _f32, _u64, _p = ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_uint64, ctypes.c_void_p
_f64 = ctypes.c_double

# name -> argtypes (all return int status)
_SIGS = {
    "co_tsp_reset": [_i64, _i64, _p, _p, _p, _p, _p, _p],
    "co_tsp_step": [_i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _p, _p, _p],
    "co_tsp_steps": [_i64, _i64, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _p, _p],
    "co_slap_closest_steps": [_i64, _i64, _i64, _i64, _p, _p, _i64, _p, _p, _p, _p, _p, _p, _p,
                              _i64, _p, _p, _p, _p],
    "co_tsp_reward": [_i64, _i64, _i64, _p, _i64, _p, _i64, _i64, _i32, _p, _p, _p],
    "co_cvrp_reset": [_i64, _i64, _p, _p, _p, _f32, _p, _p, _p, _p, _p, _p, _p],
    "co_cvrp_step": [_i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    "co_cvrp_action_mask": [_i64, _i64, _p, _p, _p, _p, _p, _p, _p],
    "co_cvrp_reward": [_i64, _i64, _i64, _p, _p, _i64, _i64, _p, _p, _i32, _p, _p, _p],
    "co_slap_reset": [_i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p],
    "co_slap_step": [_i64, _i64, _i64, _p, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    "co_slap_reward": [_i64, _i64, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p],
    "co_gather_by_index": [_p, _i64, _i64, _i64, _i64, _i64, _p, _i64, _i64, _i64, _p, _p, _p],
    "co_any_eq_i64": [_p, _i64, _i64, _p, _p],
    "co_decode_step": [_i64, _i64, _p, _i64, _p, _f32, _f32, _i32, _p, _p, _p, _p, _u64, _u64,
                       _p, _p],
    "co_decode_step_ex": [_i64, _i64, _p, _i64, _p, _f32, _f32, _i32, _f64, _i32, _p, _p, _p, _p,
                          _u64, _u64, _p, _p],
    "co_beam_select": [_i64, _i64, _i64, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p],
    "co_distance_matrix": [_i64, _i64, _p, _p, _p],
    "co_tsp_nearest_action": [_i64, _i64, _p, _p, _p, _i32, _p, _p],
    "co_cvrp_nearest_action": [_i64, _i64, _p, _p, _p, _p, _p],
    "co_cvrp_nearest_step": [_i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                             _p, _p, _p],
    "co_slap_closest_free_action": [_i64, _i64, _p, _p, _p, _p],
    "co_slap_closest_step": [_i64, _i64, _i64, _p, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                             _p, _p],
    "co_count_not_done": [_p, _i64, _p, _p],
    "co_row_deficit_max": [_p, _i64, _i64, _i64, _p, _p],
    "co_probe_copy": [_p, _p, _i64, _p],
    "co_episode_stack": [_i64, _i64, _p, _i64, _p, _i64, _p, _p, _p, _p, _p],
    "co_uniform_fill": [_p, _i64, _f32, _f32, _f32, _i32, _u64, _u64, _p],
    "co_randint_fill": [_p, _i64, _i64, _i64, _u64, _u64, _p],
    "co_pomo_shared_baseline": [_i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p],
    "co_tsp_decode_step": [_i64, _i64, _p, _i64, _p, _f32, _f32, _i32, _p, _p, _p, _u64, _u64, _p,
                           _p, _p, _p, _p, _i32, _p, _p, _p, _p, _p],
    "co_slap_decode_step": [_i64, _i64, _i64, _p, _i64, _p, _f32, _f32, _i32, _p, _p, _p, _u64,
                            _u64, _p, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    "co_cvrp_decode_step": [_i64, _i64, _p, _i64, _p, _f32, _f32, _i32, _p, _p, _p, _u64, _u64,
                            _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p],
    "co_tsp_rollout": [_i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i32, _p, _p],
    "co_tsp_rollout_ex": [_i64, _i64, _p, _p, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _i32,
                          _p, _p],
    "co_slap_rollout": [_i64, _i64, _i64, _i64, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                        _p, _p, _p, _p],
    "co_dihedral8_augment": [_i64, _i64, _p, _p, _p],
    "co_slap_generate": [_i64, _i64, _i64, _f64, _f64, _i64, _p, _p, _p, _p, _p],
    "co_symmetric_augment": [_i64, _i64, _p, _p, _f32, _p, _p],
    "co_cvrp_rollout": [_i64, _i64, _p, _p, _p, _f32, _i64, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                        _p, _p, _p, _p, _p],
}

ST_INVALID_TOUR = 1
ST_OVER_CAPACITY = 2
ST_INFEASIBLE = 4
ST_INDEX_RANGE = 8
ST_TRUNCATED = 16
ST_LOGP_NEG_INF = 32
DECODE_FAST = 0x100  # CO_DECODE_FAST mode flag (opt-in fast math; not bit-exact)
DECODE_CERTIFIED = 0x200  # CO_DECODE_CERTIFIED: fast math, greedy actions certified exact

_lock = threading.Lock()
_lib = None


class NativeUnavailable(RuntimeError):
    pass


def load():
    """Load (once) and return the ctypes handle; raise if the library is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeUnavailable(
                f"rl4co_slap_amd: HIP library {LIB_PATH} is missing; build it with "
                "`python -m rl4co_slap_amd.csrc.build` (hipcc, gfx950). There is no CPU fallback.")
        lib = ctypes.CDLL(LIB_PATH)
        for name, argtypes in _SIGS.items():
            if LIB_PATH != _PRODUCT_LIB_PATH and not hasattr(lib, name):
                continue  # an older variant library a measurement tool points at
            fn = getattr(lib, name)
            fn.argtypes = argtypes
            fn.restype = ctypes.c_int
        lib.co_build_info.restype = ctypes.c_char_p
        lib.co_build_info.argtypes = []
        if hasattr(lib, "co_variant_timing_cut") or hasattr(lib, "co_variant_timing_cut_decode"):
            # a diagnostic build (csrc/co_diag.hpp: CO_DIAG_* / CO_CVRP_CUT / CO_CVRP_RCUT):
            # its results and status bits are wrong by design.  In the product's slot it is
            # refused; a measurement tool that points LIB_PATH at a variant (or sets
            # CO_ALLOW_DIAG_LIB=1) gets a warning.
            msg = (f"rl4co_slap_amd: {LIB_PATH} is a diagnostic build (timing cut / counting "
                   "variant): its results and status bits are not valid")
            if LIB_PATH == _PRODUCT_LIB_PATH and not os.environ.get("CO_ALLOW_DIAG_LIB"):
                raise NativeUnavailable(msg + "; rebuild with `python -m rl4co_slap_amd.csrc.build`")
            warnings.warn(msg, RuntimeWarning, stacklevel=2)
        _lib = lib
        return lib


HOST_LIB_PATH = os.path.join(_HERE, "_lib", "libco_env_host.so")
_host = None
# the host (CPU) library exports the env / decode subset of the C ABI (csrc/host)
HOST_SYMBOLS = ["co_tsp_reset", "co_tsp_step", "co_tsp_reward", "co_any_eq_i64",
                "co_cvrp_reset", "co_cvrp_step", "co_cvrp_action_mask", "co_cvrp_reward",
                "co_slap_reset", "co_slap_step", "co_slap_reward", "co_gather_by_index",
                "co_decode_step"]


class _HostStream:
    """`stream_of` for a CPU tensor: routes the call to the host library."""

    def __repr__(self):
        return "HOST"


HOST = _HostStream()


def load_host():
    """The host build (TensorDicts on the CPU, BASELINE config 1); raises if missing."""
    global _host
    if _host is not None:
        return _host
    with _lock:
        if _host is not None:
            return _host
        if not os.path.exists(HOST_LIB_PATH):
            raise NativeUnavailable(
                f"rl4co_slap_amd: host library {HOST_LIB_PATH} is missing (CPU TensorDicts); "
                "build it with `python -m rl4co_slap_amd.csrc.build`.")
        lib = ctypes.CDLL(HOST_LIB_PATH)
        for name in HOST_SYMBOLS:
            fn = getattr(lib, name)
            fn.argtypes = _SIGS[name]
            fn.restype = ctypes.c_int
        _host = lib
        return lib


def provenance() -> dict:
    """What the loaded device library was built from (co_build_provenance) and whether
    that matches the sources in this tree."""
    import json

    lib = load()
    try:
        fn = lib.co_build_provenance
    except AttributeError:
        return {"source_sha256": None, "matches_tree": False}
    fn.restype = ctypes.c_char_p
    fn.argtypes = []
    info = json.loads(fn().decode())
    try:
        from .csrc.build import source_hash

        info["tree_sha256"] = source_hash()
        info["matches_tree"] = info["tree_sha256"] == info["source_sha256"]
    except OSError:  # sources not shipped
        info["matches_tree"] = None
    return info


def exported_symbols():
    return list(_SIGS) + ["co_build_info"]


def ptr(t):
    return None if t is None else t.data_ptr()


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_of(t: torch.Tensor):
    """The current HIP stream of the tensor's device, as a handle (the raw-stream query:
    ~0.3 us against ~4 us for torch.cuda.current_stream(dev).cuda_stream per call); for a
    CPU tensor the HOST marker (the call goes to the host library)."""
    if t.device.type == "cpu":
        return HOST
    idx = t.device.index
    if _raw_stream is not None and idx is not None:
        return _raw_stream(idx)
    return torch.cuda.current_stream(t.device).cuda_stream


def require_device(*tensors):
    """All tensors on the HIP device, or all on the CPU (the host build; the caller's
    C-ABI call then goes to libco_env_host.so).  Mixed devices raise."""
    devs = {t.device.type for t in tensors if t is not None}
    if devs <= {"cuda"}:
        return
    if devs == {"cpu"}:
        load_host()  # raises when the host library was not built
        return
    raise RuntimeError(f"rl4co_slap_amd: tensors on mixed devices {sorted(devs)}; the env "
                       "runs on the HIP device or, for CPU TensorDicts, the host build")


_KIND = {_i64: "i", _i32: "i", _u64: "i", _p: "i", _f32: "f", _f64: "d"}


def _fastcall_path() -> str:
    """The fast-call module built for THIS interpreter (csrc/build.py names it with the
    interpreter's EXT_SUFFIX, so a module built against other Python headers is never
    picked up)."""
    import sysconfig

    return os.path.join(_HERE, "_lib", "_co_fastcall" + (sysconfig.get_config_var("EXT_SUFFIX")
                                                         or ".so"))


FASTCALL_PATH = _fastcall_path()


class _FastCall:
    """The CPython fast-call module (csrc/pycall/co_fastcall.cpp) and, per library, the
    entry points' addresses and argument classes.  Each table is built on its first use,
    so host-only callers never load the device library; any failure to load the module or
    a library leaves that table empty and the call goes through ctypes."""

    def __init__(self, invoke):
        self.invoke = invoke
        self._tables = {}

    @staticmethod
    def _table(lib, names):
        return {n: (ctypes.cast(getattr(lib, n), ctypes.c_void_p).value,
                    "".join(_KIND[t] for t in _SIGS[n]).encode()) for n in names}

    def table(self, which):
        t = self._tables.get(which)
        if t is None:
            try:
                t = (self._table(load(), list(_SIGS)) if which == "dev"
                     else self._table(load_host(), HOST_SYMBOLS))
            except Exception:  # missing / unloadable library: ctypes raises the real error
                t = {}
            self._tables[which] = t
        return t


_fast = None  # a _FastCall once loaded, False when unavailable


def _fastcall():
    """The fast-call path, or None (then ctypes is used)."""
    global _fast
    if _fast is not None:
        return _fast or None
    _fast = False
    if os.environ.get("CO_NO_FASTCALL") or not os.path.exists(FASTCALL_PATH):
        return None
    try:
        import importlib.machinery
        import importlib.util

        loader = importlib.machinery.ExtensionFileLoader("_co_fastcall", FASTCALL_PATH)
        spec = importlib.util.spec_from_file_location("_co_fastcall", FASTCALL_PATH,
                                                      loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
    except Exception as e:  # built for another interpreter / unloadable: ctypes instead
        warnings.warn(f"rl4co_slap_amd: fast-call module unusable ({e}); using ctypes",
                      RuntimeWarning, stacklevel=2)
        return None
    _fast = _FastCall(mod.invoke)
    return _fast


TORCHSTEP_PATH = os.path.join(_HERE, "_lib", "_co_torchstep" + (
    __import__("sysconfig").get_config_var("EXT_SUFFIX") or ".so"))
_tstep = None  # the loaded glue module once tried, False when unavailable


class _TorchStep:
    """The drop-in loop's step glue (csrc/pycall/co_torchstep.cpp): per fused step, output
    allocation + the C-ABI launch in one call.  Each function is bound to its entry point's
    address in the loaded device library (the glue calls through it; it links no kernels)."""

    def __init__(self, mod):
        import functools

        lib = load()

        def bound(fn, entry):
            return functools.partial(fn, ctypes.cast(getattr(lib, entry), ctypes.c_void_p).value)

        self.tsp_decode_step = bound(mod.tsp_decode_step, "co_tsp_decode_step")
        self.tsp_step_td = bound(mod.tsp_step_td, "co_tsp_decode_step")
        self.decode_step = bound(mod.decode_step, "co_decode_step")
        self.cvrp_step = bound(mod.cvrp_step, "co_cvrp_step")
        self.slap_step_td = bound(mod.slap_step_td, "co_slap_decode_step")
        self.cvrp_step_td = bound(mod.cvrp_step_td, "co_cvrp_decode_step")
        self.slap_reset_td = bound(mod.slap_reset_td, "co_slap_reset")
        self.episode_stack = bound(mod.episode_stack, "co_episode_stack")
        self.slab_fresh = mod.slab_fresh
        self.fast_step = getattr(mod, "fast_step", None)
        self.clear_pool = mod.clear_pool
        self.set_inplace = mod.set_inplace
        self.inplace_policy = mod.inplace_policy


def torchstep():
    """The step glue, or None (built against another torch / interpreter, not built, or
    ``CO_NO_TORCHSTEP`` set): callers then take their Python path, same results."""
    global _tstep
    if _tstep is not None:
        return _tstep or None
    _tstep = False
    if os.environ.get("CO_NO_TORCHSTEP") or not os.path.exists(TORCHSTEP_PATH):
        return None
    try:
        import importlib.machinery
        import importlib.util

        loader = importlib.machinery.ExtensionFileLoader("_co_torchstep", TORCHSTEP_PATH)
        spec = importlib.util.spec_from_file_location("_co_torchstep", TORCHSTEP_PATH,
                                                      loader=loader)
        mod = importlib.util.module_from_spec(spec)
        loader.exec_module(mod)
        _tstep = _TorchStep(mod)
    except Exception as e:  # e.g. undefined torch symbols: a build for another torch
        warnings.warn(f"rl4co_slap_amd: step glue module unusable ({e}); using the Python "
                      "step path", RuntimeWarning, stacklevel=2)
        return None
    return _tstep


def check_rc(name, rc):
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")


def call(name, *args):
    fast = _fast if _fast else _fastcall()
    if args and args[-1] is HOST:
        lib = load_host()
        if name not in HOST_SYMBOLS:
            raise NotImplementedError(f"{name} has no host (CPU) build; move the TensorDict "
                                      "to the HIP device")
        args = args[:-1] + (None,)
        ent = fast.table("host").get(name) if fast else None
        rc = fast.invoke(ent[0], ent[1], *args) if ent else getattr(lib, name)(*args)
    else:
        ent = fast.table("dev").get(name) if fast else None
        rc = fast.invoke(ent[0], ent[1], *args) if ent else getattr(load(), name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with status {rc}")


def bind(name, *args):
    """Pre-convert every argument but the trailing stream once; returns
    ``launch(stream)``.  For launch-bound loops that call one entry point on fixed
    buffers (the fused episodes): a plain ``call`` re-reads ``data_ptr()`` and re-converts
    each argument per launch, which costs about as much host time as a 20 us kernel."""
    fn = getattr(load(), name)
    conv = tuple(None if a is None else t(a) for t, a in zip(_SIGS[name][:-1], args))
    assert len(conv) == len(_SIGS[name]) - 1, name

    def launch(stream):
        rc = fn(*conv, stream)
        if rc != 0:
            raise RuntimeError(f"{name} failed with status {rc}")

    return launch


_zero_words = {}  # (device type, index, words) -> status tensors a host read found all zero


def scratch_status(device, words: int = 1) -> torch.Tensor:
    """``words`` zeroed int32 words for data-dependent error bits.  A status tensor whose
    host read found every word zero (``release_status``: the read synchronised, nothing
    writes it since) is handed out again instead of zero-filling a new one -- a fill is a
    kernel launch, ~4 us of host time on an episode's fixed path."""
    device = torch.device(device)
    free = _zero_words.get((device.type, device.index, words))
    if free:
        return free.pop()
    return torch.zeros(words, dtype=torch.int32, device=device)


def release_status(t: torch.Tensor, values) -> None:
    """Return a status tensor to the zero pool after a host read of it (``values``) found
    no bit set; the caller must not use it afterwards."""
    if any(values) or t.dim() != 1 or t._base is not None:
        return
    d = t.device
    free = _zero_words.setdefault((d.type, d.index, t.shape[0]), [])
    if len(free) < 8:
        free.append(t)


# Per-device word that kernels without a caller-held status (gather_by_index) OR their
# error bits into.  It is read together with the next status read the host makes anyway
# (an env's reward / status check, post_decoder_hook) -- the analogue of the device-side
# assert torch.gather raises on a HIP tensor, which also surfaces at the next sync.
# CO_SYNC_CHECKS=1 reads it right after every such kernel instead (debugging).
_deferred = {}
SYNC_CHECKS = bool(os.environ.get("CO_SYNC_CHECKS"))
_DEFERRED_MSGS = ((ST_INDEX_RANGE, "gather_by_index: index out of range (torch.gather: index "
                                   "out of bounds for the gathered dimension)"),)


def deferred_status(device) -> torch.Tensor:
    device = torch.device(device)
    key = (device.type, device.index)
    w = _deferred.get(key)
    if w is None:
        w = _deferred[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return w


def pending_deferred(device):
    """The device's deferred word if one exists (else None): read it with the caller's own
    status read, then pass the bits to ``raise_deferred``."""
    device = torch.device(device)
    return _deferred.get((device.type, device.index))


def raise_deferred(bits: int, device) -> None:
    """Raise the error the deferred bits stand for (clearing the word first, so the error
    is reported once)."""
    if not bits:
        return
    w = pending_deferred(device) if device is not None else None
    if w is not None:
        w.zero_()
    for bit, msg in _DEFERRED_MSGS:
        if bits & bit:
            raise RuntimeError(msg)


def check_deferred(device) -> None:
    """Read (one host sync) and raise the device's deferred error bits."""
    w = pending_deferred(device)
    if w is not None:
        raise_deferred(int(w.item()), device)
