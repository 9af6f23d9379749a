"""Env-steps/sec benchmark of the MI355X CO-env engine (BASELINE.json metric).

``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (one rank per GPU, RCCL).  A *step* of this benchmark is
one full episode of the hot path over one batch resident in HBM: reset, every env
step, and the episode-end reward (+ validity check).  Workload (BASELINE.json
config 2): TSP-100, B = 65,536 instances per GPU (weak scaling), seeded synthetic
instances ``manual_seed(1234); rand(B,100,2)`` and teacher-forced actions
``manual_seed(4321); rand(B,100).argsort(1)`` (Evaluate-mode rollout).

``value`` = env-steps/s over all ranks = world * B * N * K / max-over-ranks time.
Rank 0 prints ONE JSON line.  ``cpu_baseline`` times the CPU oracle (the plain
PyTorch restatement of the reference op sequence) on a bounded sample on this
host; ``roofline`` prices the dominant kernel against HBM (8.0 TB/s).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--num-loc", type=int, default=100)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--extra", action="store_true", help="also time SLAP / stepwise modes")
    return ap.parse_args()


def setup_dist():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def barrier(world):
    if world > 1:
        dist.barrier()


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def tsp_inputs(b, n, rank, dev):
    torch.manual_seed(1234 + rank)
    locs = torch.rand(b, n, 2)
    torch.manual_seed(4321 + rank)
    acts = torch.rand(b, n).argsort(1)
    return locs.to(dev), acts.to(dev)


def time_graph(ep, steps, warmup, world, dev, stream):
    for _ in range(warmup):
        ep.replay()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        ep.replay()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    return wall, ev0.elapsed_time(ev1) / 1e3


def cpu_baseline_tsp(n, b_cpu=16384, episodes=3):
    """The oracle (reference op sequence on CPU torch) timed on this host."""
    from oracle.envs import TSPOracle
    from oracle.rollout import rollout

    threads = os.cpu_count() or 1
    torch.set_num_threads(threads)
    env = TSPOracle(num_loc=n, seed=1234)
    torch.manual_seed(4321)
    acts = torch.rand(b_cpu, n).argsort(1)
    times = []
    for e in range(episodes + 1):
        td = env.reset(batch_size=[b_cpu])
        it = iter(range(n))
        t0 = time.perf_counter()
        rollout(env, td, lambda td: acts[:, next(it)])
        times.append(time.perf_counter() - t0)
    times = sorted(times[1:])
    med = times[len(times) // 2]
    return {"value": b_cpu * n / med, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle TSP-{n} teacher-forced rollout (reset+{n} steps+reward), "
                      f"B={b_cpu}, median of {episodes} episodes after 1 warm-up, "
                      f"torch.set_num_threads({threads})"}


def main():
    args = parse()
    world, rank, dev = setup_dist()
    from rl4co_slap_amd import _native
    from rl4co_slap_amd.rollout.engine import TSPStepwiseEpisode

    _native.load()
    b, n = args.batch, args.num_loc
    locs, acts = tsp_inputs(b, n, rank, dev)
    ep = TSPStepwiseEpisode(locs, acts, policy="teacher", check=True).capture()
    wall, gpu_s = time_graph(ep, args.steps, args.warmup, world, dev, ep.stream)
    assert int(ep.status.item()) == 0, "invalid tour / index error in the benchmark episode"
    t = max_over_ranks(wall, world, dev)
    value = world * b * n * args.steps / t

    # dominant kernel: co_tsp_step; time a graph of N back-to-back steps with events
    steps_only = _StepsOnly(ep)
    steps_only.capture()
    sw, sg = time_graph(steps_only, max(3, args.steps // 2), 2, world, dev, steps_only.stream)
    per_launch = sg / (max(3, args.steps // 2) * n)
    bytes_per_launch = (2 * n + 50) * b  # 2N+50 B per TSP env-step
    achieved = bytes_per_launch / per_launch / 1e9

    out = {
        "metric": "env-steps/sec (batch×decode) SLAP & TSP-100 at 1/2/4/8 MI355X",
        "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": t / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8+i64+f32",
        "data": "synthetic (seeded torch.rand instances, teacher-forced argsort actions)",
        "config": {"workload": f"TSP-{n} teacher-forced episode (reset + {n} x step + reward), "
                               f"stepwise HIP-graph", "batch_per_gpu": b, "num_loc": n,
                   "parallelism": f"dp{world} (instance shards, no data-path collective)"},
        "roofline": {"bound": "hbm", "kernel": "co_tsp_step (tsp_step_kernel)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None,
                     "per_launch_us": per_launch * 1e6,
                     "note": "event time / launches of a graph of back-to-back step kernels "
                             "(includes the launch boundary)"},
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_tsp(n)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


class _StepsOnly:
    """A graph of the episode's N step launches only (for per-launch timing)."""

    def __init__(self, ep):
        self.ep = ep
        self.stream = ep.stream
        self.graph = None

    def _launch(self, s):
        from rl4co_slap_amd import _native as nat

        ep = self.ep
        b, n = ep.b, ep.n
        for t in range(n):
            src, dst = t & 1, (t + 1) & 1
            nat.call("co_tsp_step", b, n, nat.ptr(ep.acts[t]), nat.ptr(ep.mask[src]),
                     nat.ptr(ep.mask[dst]), nat.ptr(ep.i[src]), nat.ptr(ep.i[dst]),
                     nat.ptr(ep.first[src]), nat.ptr(ep.first[dst]), nat.ptr(ep.cur),
                     nat.ptr(ep.done), nat.ptr(ep.step_reward), 0, None, nat.ptr(ep.status), s)

    def capture(self):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream):
            self._launch(torch.cuda.current_stream().cuda_stream)
        self.graph = g

    def replay(self):
        self.graph.replay()


if __name__ == "__main__":
    main()
