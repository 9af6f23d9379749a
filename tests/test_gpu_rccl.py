"""RCCL on the device: ``global_metrics``' all-gather through an
``nccl`` process group of world size 1 -- the call path the multi-GPU bench takes -- in a
child process (the group is initialised before any other GPU work there; the child is
started with subprocess, never exec'd from this GPU-initialised process), compared bit for
bit with the local values."""
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


@pytest.mark.gpu
def test_global_metrics_through_rccl_world1(dev):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["MASTER_ADDR"] = "127.0.0.1"
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_world1_child.py"),
                        str(_free_port())], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "RCCL_OK nccl 64" in r.stdout, r.stdout[-2000:]
