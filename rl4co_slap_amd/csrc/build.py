"""Build the gfx950 C-ABI library ``rl4co_slap_amd/_lib/libco_env.so`` with hipcc.

No torch types cross the ABI, so the library is a plain ``hipcc -shared`` build;
it links ``libamdhip64.so.7`` by SONAME and therefore binds to the HIP runtime
torch has already loaded when imported after ``import torch`` (one runtime per
process).  Usage: ``python -m rl4co_slap_amd.csrc.build [--force]``.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
OUT_DIR = os.path.join(PKG, "_lib")
LIB = os.path.join(OUT_DIR, "libco_env.so")
SOURCES = ["tsp.hip", "cvrp.hip", "slap.hip", "ops.hip", "decode_step.hip", "decode_tsp.hip",
           "decode_env.hip",
           "rollout.hip",
           "nearest.hip"]
HEADERS = ["co_common.hpp", "co_tile.hpp", "co_math.hpp", "decode_common.hpp"]
ARCH = "gfx950"


def hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found: the gfx950 library cannot be built")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(HERE, f) for f in SOURCES + HEADERS]
    deps.append(os.path.join(ROOT, "include", "co_env.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def source_hash() -> str:
    """sha256 over the device library's sources, headers and the ABI header (in order)."""
    import hashlib

    h = hashlib.sha256()
    for f in SOURCES + HEADERS:
        with open(os.path.join(HERE, f), "rb") as fh:
            h.update(f.encode() + b"\0" + fh.read())
    with open(os.path.join(ROOT, "include", "co_env.h"), "rb") as fh:
        h.update(b"co_env.h\0" + fh.read())
    return h.hexdigest()


def _provenance_object(obj_dir: str, verbose: bool) -> str:
    """A host-only object exporting co_build_provenance(): the source hash the library was
    built from, the build time and the compiler, so a run can show which sources the
    loaded library came from (tests/test_gpu_provenance.py, bench.py "build")."""
    import json
    import time

    ver = subprocess.run([hipcc(), "--version"], capture_output=True, text=True).stdout
    ver = next((ln for ln in ver.splitlines() if "clang version" in ln or "HIP version" in ln), "")
    info = json.dumps({"source_sha256": source_hash(), "built_at": time.strftime(
        "%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "compiler": ver.strip(), "arch": ARCH})
    src = os.path.join(obj_dir, "provenance.cpp")
    with open(src, "w") as f:
        f.write('extern "C" __attribute__((visibility("default"))) const char* '
                "co_build_provenance(void) { return " + json.dumps(info) + "; }\n")
    obj = os.path.join(obj_dir, "provenance.o")
    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    cmd = [cxx, "-O2", "-fPIC", "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return obj


def build(force=False, verbose: bool = False) -> str:
    """Compile each source to an object in parallel, then link the shared library.
    ``force="incremental"`` (``--incremental``) recompiles only objects older than their
    source or a header (development); ``force=True`` recompiles everything."""
    from concurrent.futures import ThreadPoolExecutor

    if not force and not _stale():
        if not os.path.exists(HOST_LIB) or os.path.getmtime(HOST_LIB) < os.path.getmtime(HOST_SRC):
            build_host(verbose=verbose)
        if (not os.path.exists(FASTCALL_LIB)
                or os.path.getmtime(FASTCALL_LIB) < os.path.getmtime(FASTCALL_SRC)):
            build_fastcall(verbose=verbose)
        if _torchstep_stale():
            build_torchstep(verbose=verbose)
        return LIB
    os.makedirs(OUT_DIR, exist_ok=True)
    obj_dir = os.path.join(OUT_DIR, "obj")
    os.makedirs(obj_dir, exist_ok=True)
    flags = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
             "-fno-fast-math", "-Wall", "-Wno-unused-result", "-I", os.path.join(ROOT, "include")]

    hdr_t = max(os.path.getmtime(d) for d in
                [os.path.join(HERE, h) for h in HEADERS] + [os.path.join(ROOT, "include", "co_env.h")])
    incremental = force == "incremental"

    def compile_one(src):
        obj = os.path.join(obj_dir, os.path.splitext(src)[0] + ".o")
        if incremental and os.path.exists(obj):
            t = os.path.getmtime(obj)
            if t > hdr_t and t > os.path.getmtime(os.path.join(HERE, src)):
                return obj  # object newer than its source and every header
        cmd = [hipcc()] + flags + ["-c", os.path.join(HERE, src), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return obj

    jobs = min(len(SOURCES), max(1, min(os.cpu_count() or 1, 8)))
    with ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, SOURCES))
    objs.append(_provenance_object(obj_dir, verbose))
    tmp = LIB + ".tmp"
    cmd = [hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, "-x", "none"] + objs
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(tmp, LIB)
    build_host(verbose=verbose)
    build_fastcall(verbose=verbose)
    build_torchstep(verbose=verbose)
    return LIB


HOST_SRC = os.path.join(HERE, "host", "co_env_host.cpp")
HOST_LIB = os.path.join(OUT_DIR, "libco_env_host.so")
HOST_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-fno-fast-math",
              "-Wall", "-Wextra"]


FASTCALL_SRC = os.path.join(HERE, "pycall", "co_fastcall.cpp")


def _ext_suffix() -> str:
    """The running interpreter's extension suffix (e.g. ``.cpython-310-x86_64-linux-gnu.so``):
    the fast-call module is built against this interpreter's headers, and the ABI tag in
    its file name keeps another interpreter from loading it."""
    import sysconfig

    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


FASTCALL_LIB = os.path.join(OUT_DIR, "_co_fastcall" + _ext_suffix())


def build_fastcall(verbose: bool = False) -> str:
    """The CPython fast-call module (csrc/pycall): the env loop's C-ABI calls without
    ctypes' per-call marshalling.  Optional: _native falls back to ctypes without it."""
    import sysconfig

    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    inc = sysconfig.get_paths()["include"]
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I", inc, "-o",
           FASTCALL_LIB + ".tmp", FASTCALL_SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(FASTCALL_LIB + ".tmp", FASTCALL_LIB)
    return FASTCALL_LIB


TORCHSTEP_SRC = os.path.join(HERE, "pycall", "co_torchstep.cpp")
TORCHSTEP_LIB = os.path.join(OUT_DIR, "_co_torchstep" + _ext_suffix())


def _torchstep_stale() -> bool:
    if not os.path.exists(TORCHSTEP_LIB):
        return True
    t = os.path.getmtime(TORCHSTEP_LIB)
    return any(os.path.getmtime(d) > t for d in (TORCHSTEP_SRC, os.path.join(ROOT, "include",
                                                                           "co_env.h")))


def build_torchstep(verbose: bool = False) -> str:
    """The drop-in loop's step glue (csrc/pycall/co_torchstep.cpp): a CPython module
    against this torch's headers and libraries (g++, no device code).  Optional: without
    it the env steps take their Python path."""
    import sysconfig

    import torch
    from torch.utils import cpp_extension

    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    libdir = cpp_extension.library_paths()[0]
    cmd = [cxx, "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-D__HIP_PLATFORM_AMD__=1",
           "-DUSE_ROCM=1", f"-D_GLIBCXX_USE_CXX11_ABI={int(torch._C._GLIBCXX_USE_CXX11_ABI)}",
           "-I", sysconfig.get_paths()["include"], "-I", "/opt/rocm/include",
           "-I", os.path.join(ROOT, "include")]
    for inc in cpp_extension.include_paths():
        cmd += ["-isystem", inc]
    cmd += ["-o", TORCHSTEP_LIB + ".tmp", TORCHSTEP_SRC, "-L", libdir, "-Wl,-rpath," + libdir,
            "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu", "-ltorch_python"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(TORCHSTEP_LIB + ".tmp", TORCHSTEP_LIB)
    return TORCHSTEP_LIB


def build_host(verbose: bool = False, out: str = HOST_LIB, extra=()) -> str:
    """The host (CPU) build of the env / decode entry points (csrc/host): g++, the same
    C ABI, for TensorDicts on the CPU.  ``extra`` adds flags (the sanitizer build)."""
    cxx = os.environ.get("CXX") or shutil.which("g++") or "g++"
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [cxx] + HOST_FLAGS + list(extra) + ["-o", out + ".tmp", HOST_SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build(force="incremental" if "--incremental" in sys.argv else "--force" in sys.argv,
                verbose=True))
