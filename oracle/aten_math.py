"""ctypes access to the oracle's C restatement of ATen's CPU log_softmax math
(``oracle/c/aten_math.c``) and to torch's bundled SLEEF (``oracle/c/sleef_probe.c``).
TEST INFRASTRUCTURE ONLY."""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .build import MATH_LIB, PROBE_LIB, build

_lib = None
_probe = None


def _math():
    global _lib
    if _lib is None:
        if not os.path.exists(MATH_LIB):
            build()
        _lib = ctypes.CDLL(MATH_LIB)
    return _lib


def probe():
    """torch's own SLEEF (None when the host lacks AVX512F or the probe is not built)."""
    global _probe
    if _probe is None and os.path.exists(PROBE_LIB):
        _probe = ctypes.CDLL(PROBE_LIB)
    return _probe


def _vp(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _unary(lib, name, x):
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    y = np.empty_like(x)
    getattr(lib, name)(_vp(x), _vp(y), ctypes.c_long(x.size))
    return y


def expf(x):
    return _unary(_math(), "aten_expf_batch", x)


def logf(x):
    return _unary(_math(), "aten_logf_batch", x)


def tanh_cr(x):
    return _unary(_math(), "tanh_cr_batch", x)


def sleef_expf(x):
    """torch's SLEEF expf_u10 (x.size a multiple of 16)."""
    return _unary(probe(), "probe_sleef_expf", x)


def sleef_logf(x):
    return _unary(probe(), "probe_sleef_logf", x)


def log_softmax(x, width: int = 16):
    """F.log_softmax(x, -1) of a 2-D f32 array as ATen's CPU kernel evaluates it."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    b, n = x.shape
    out = np.empty_like(x)
    _math().aten_log_softmax(_vp(x), _vp(out), ctypes.c_long(b), ctypes.c_long(n),
                             ctypes.c_int(width))
    return out
