"""Host-side profile of the SLAP drop-in loop (bench.bench_dropin_slap's path) at a small
batch, where the device work is negligible and every microsecond is Python / glue:
per-episode wall time split into env.reset, the policy forward and the rest, then a
cProfile of the same episodes (top functions by own time).

    python tools/prof_dropin_slap.py [--b 64] [--episodes 300]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=64)
    ap.add_argument("--episodes", type=int, default=300)
    ap.add_argument("--top", type=int, default=35)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from rl4co_slap_amd.envs import SLAPEnv
    from rl4co_slap_amd.envs.slap import SLAPGenerator
    from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder
    from rl4co_slap_amd.td import TensorDict

    torch.manual_seed(1234)
    np.random.seed(1234)
    data = SLAPGenerator(materialize_dist_mat=False)(a.b).to(dev)
    logits = torch.randn(a.b, data["locs"].shape[1], generator=torch.Generator().manual_seed(11))
    logits = logits.to(dev)
    env = SLAPEnv(device=dev)
    pol = ConstructivePolicy(None, LogitsDecoder(lambda td, lg=logits: lg), env_name="slap",
                             tanh_clipping=10.0)
    items = dict(data.items())

    def episode(split=None):
        t0 = time.perf_counter()
        td = env.reset(TensorDict(dict(items), [a.b]))
        t1 = time.perf_counter()
        out = pol(td, env, phase="test", decode_type="greedy")
        t2 = time.perf_counter()
        if split is not None:
            split[0] += t1 - t0
            split[1] += t2 - t1
        return out

    # host enqueue time: the episode's one status read (_Checks.read) marks the end of
    # the host's launches; the rest of the episode is the device draining behind it
    from rl4co_slap_amd.utils import decoding as D

    marks = []
    orig_read = D._Checks.read

    def read(self):
        marks.append(time.perf_counter())
        return orig_read(self)

    D._Checks.read = read
    for _ in range(20):
        episode()
    torch.cuda.synchronize()
    enq = tot_e = 0.0
    for _ in range(a.episodes):
        marks.clear()
        t0 = time.perf_counter()
        episode()
        t1 = time.perf_counter()
        enq += marks[0] - t0
        tot_e += t1 - t0
    print(f"B={a.b}: host enqueue {enq / a.episodes * 1e6:.1f} us of {tot_e / a.episodes * 1e6:.1f}"
          " us per episode (the rest: the device's tail after the last launch)")
    # device time per episode: a 5 ms sleep queued ahead of each episode hides the host
    # (it enqueues everything while the device sleeps), so wall - sleep = device time
    sl = int(os.environ.get("CO_SLEEP_CYCLES", "10000000"))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        torch.cuda._sleep(sl)
    torch.cuda.synchronize()
    t_sleep = (time.perf_counter() - t0) / 20
    dev_t = 0.0
    for _ in range(20):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda._sleep(sl)
        episode()
        dev_t += time.perf_counter() - t0 - t_sleep
    print(f"B={a.b}: device ~{dev_t / 20 * 1e6:.1f} us per episode (sleep {t_sleep * 1e6:.0f} us "
          "hides the host)")
    D._Checks.read = orig_read
    torch.cuda.synchronize()
    split = [0.0, 0.0]
    t0 = time.perf_counter()
    for _ in range(a.episodes):
        episode(split)
    torch.cuda.synchronize()
    tot = time.perf_counter() - t0
    e = a.episodes
    print(f"B={a.b}: {tot / e * 1e6:.1f} us per episode; reset {split[0] / e * 1e6:.1f}, "
          f"forward {split[1] / e * 1e6:.1f}")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(a.episodes):
        episode()
    torch.cuda.synchronize()
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(a.top)
    print(s.getvalue())


if __name__ == "__main__":
    main()
