"""Build the oracle's C restatements (TEST INFRASTRUCTURE ONLY) with gcc:

* ``oracle/_build/libaten_math.so`` from ``oracle/c/aten_math.c`` (ATen's CPU
  log_softmax math: SLEEF expf/logf + vec::map_reduce_all order; tanh rounded from f64);
* ``oracle/_build/libsleef_probe.so`` from ``oracle/c/sleef_probe.c`` (calls the SLEEF
  symbols torch's own libtorch_cpu exports; built only on an AVX512F host).

``-ffp-contract=off`` keeps every fmaf explicit and nothing else fused.  The outputs are
git-ignored and travel to the GPU box with the tree like the product library.
Usage: ``python -m oracle.build``.
"""
from __future__ import annotations

import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_build")
MATH_LIB = os.path.join(OUT, "libaten_math.so")
PROBE_LIB = os.path.join(OUT, "libsleef_probe.so")


def _avx512() -> bool:
    try:
        with open("/proc/cpuinfo") as f:
            return " avx512f" in f.read()
    except OSError:
        return False


def build(force: bool = False) -> str:
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(HERE, "c", "aten_math.c")
    if force or not os.path.exists(MATH_LIB) or os.path.getmtime(src) > os.path.getmtime(MATH_LIB):
        subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-shared", "-fPIC",
                        "-o", MATH_LIB, src, "-lm"], check=True)
    probe = os.path.join(HERE, "c", "sleef_probe.c")
    if _avx512() and (force or not os.path.exists(PROBE_LIB)
                      or os.path.getmtime(probe) > os.path.getmtime(PROBE_LIB)):
        import torch

        tlib = os.path.join(os.path.dirname(torch.__file__), "lib")
        subprocess.run(["gcc", "-O2", "-mavx512f", "-shared", "-fPIC", "-o", PROBE_LIB, probe,
                        f"-L{tlib}", "-ltorch_cpu", f"-Wl,-rpath,{tlib}"], check=True)
    return MATH_LIB


if __name__ == "__main__":
    print(build(force=True))
