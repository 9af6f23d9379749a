"""The host build's indexing under AddressSanitizer + UndefinedBehaviorSanitizer
(sanitizers on host code): tests/host_asan/driver.cpp is compiled
together with csrc/host/co_env_host.cpp by g++ with -fsanitize=address,undefined
(-fno-sanitize-recover: any report fails the run) and executed as its own process.  CPU
only; skipped where g++ or the sanitizer runtimes are absent."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_host_build_is_sanitizer_clean(tmp_path):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = tmp_path / "host_asan"
    cmd = [cxx, "-O1", "-g", "-std=c++17", "-fno-omit-frame-pointer", "-ffp-contract=off",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
           os.path.join(ROOT, "tests", "host_asan", "driver.cpp"),
           os.path.join(ROOT, "rl4co_slap_amd", "csrc", "host", "co_env_host.cpp"),
           "-o", str(exe)]
    b = subprocess.run(cmd, capture_output=True, text=True)
    if b.returncode != 0 and ("-lasan" in b.stderr or "-lubsan" in b.stderr):
        pytest.skip("sanitizer runtimes not available: " + b.stderr[-300:])
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "ran clean" in r.stdout
