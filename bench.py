"""Env-steps/sec benchmark of the MI355X CO-env engine (BASELINE.json metric).

``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched by
``torch.distributed.run`` (one rank per GPU; RCCL only for the timing reduction --
the instance shards never exchange data).  A *step* of this benchmark is one full
episode of the hot path over one batch resident in HBM: reset, every env step and
the episode-end reward with the validity check.

Headline workload (BASELINE.json config 2): TSP-100, B = 65,536 instances per GPU
(weak scaling), ``manual_seed(1234 + rank); rand(B,100,2)``, teacher-forced actions
``manual_seed(4321 + rank); rand(B,100).argsort(1)`` (Evaluate-mode rollout), run as
the fused one-launch episode kernel ``co_tsp_rollout``.
``value`` = world * B * 100 * K / (max over ranks of the timed wall time).

Also reported (``modes``): the same episode stepwise (one launch per env step,
TensorDict state in HBM between steps, HIP graph), the in-kernel nearest-unvisited
policy, and SLAP (examples/slap.py instance, B = 16,384).  ``cpu_baseline`` is the
CPU oracle (plain-PyTorch restatement of the reference op sequence) on this host.
"""
from __future__ import annotations

import argparse
import itertools
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
FP32_VECTOR_PEAK_TFS = 157.3  # MI355X FP32 vector (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=65536)
    ap.add_argument("--num-loc", type=int, default=100)
    ap.add_argument("--slap-batch", type=int, default=16384)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-modes", action="store_true", help="headline only")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU plumbing check: gloo ranks, the CPU oracle episode as the step "
                         "(no GPU, no HIP library); rehearses --gpus N launches in a container")
    return ap.parse_args()


def launch_ranks(args):
    """--gpus N > 1 without a torch.distributed launcher around us: start one rank per GPU
    as children of this process (which has not touched the GPU) through
    torch.distributed.run on 127.0.0.1 and exit with its status."""
    import socket
    import subprocess

    sock = socket.socket()
    sock.bind(("127.0.0.1", 0))
    port = sock.getsockname()[1]
    sock.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def setup_dist(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch one rank "
                         f"per GPU (torch.distributed.run --nproc-per-node {args.gpus}) or drop "
                         f"the launcher and let bench.py start them")
    if args.dry_run:
        if world > 1:
            dist.init_process_group("gloo")
        return world, rank, torch.device("cpu")
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, torch.device("cuda", local)


def barrier(world):
    if world > 1:
        dist.barrier()


def sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def max_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world, dev):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def timed(run, steps, warmup, world, dev):
    """W untimed runs, then exactly K timed runs bracketed by barrier + synchronize.
    Returns (wall seconds, HIP-event seconds on the launching stream)."""
    for _ in range(warmup):
        run()
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    cur = torch.cuda.current_stream(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(cur)
    for _ in range(steps):
        run()
    ev1.record(cur)
    torch.cuda.synchronize(dev)
    barrier(world)
    torch.cuda.synchronize(dev)
    return time.perf_counter() - t0, ev0.elapsed_time(ev1) / 1e3


def tsp_inputs(b, n, rank, salt=0):
    torch.manual_seed(1234 + rank + 104729 * salt)
    locs = torch.rand(b, n, 2)
    torch.manual_seed(4321 + rank + 104729 * salt)
    acts = torch.rand(b, n).argsort(1)
    return locs, acts


MALL_BYTES = 256 << 20  # Infinity Cache (MI355X_MICROARCH.md, chip-level parameters)


def rotation(input_bytes):
    """Distinct input batches a timed loop cycles through so that no launch finds its
    inputs Infinity-Cache resident from their previous use: together they exceed the
    256 MiB cache by 25 % (a cyclic sweep larger than an LRU cache misses every line), so
    the rates below are HBM rates.  (One batch repeated would stay resident: 105 MB of
    TSP-100 inputs at B = 65,536.)"""
    return max(2, min(16, -(-int(1.25 * MALL_BYTES) // max(1, int(input_bytes)))))


def copy_probe(traffic_bytes, dev, k):
    """The streaming ceiling beside the roofline: co_probe_copy (16-B loads and stores)
    moving the same HBM bytes as one headline launch (source buffers cycled past the
    Infinity Cache), and 2 GiB (asymptotic)."""
    from rl4co_slap_amd import _native as nat

    res = {}
    s = torch.cuda.current_stream(dev).cuda_stream
    for label, traffic in (("same_bytes", traffic_bytes), ("2GiB", 2 << 30)):
        n = (traffic // 2) // 16 * 16
        r = rotation(n) if n < MALL_BYTES else 1
        bufs = [(torch.ones(n, dtype=torch.uint8, device=dev),
                 torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(r)]
        fs = [nat.bind("co_probe_copy", nat.ptr(a), nat.ptr(c), n) for a, c in bufs]
        for f in fs:
            f(s)
        reps = max(k, 10, r)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            fs[i % r](s)
        e1.record()
        torch.cuda.synchronize(dev)
        t = e0.elapsed_time(e1) / 1e3 / reps
        res[label] = {"bytes": 2 * n, "us": t * 1e6, "GBps": 2 * n / t / 1e9, "buffers_cycled": r}
        del bufs, fs
    return res


def time_bound(f, dev, reps=50):
    """Average HIP-event time (s) of `reps` back-to-back launches of a bound C-ABI call."""
    s = torch.cuda.current_stream(dev).cuda_stream
    for _ in range(3):
        f(s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f(s)
    e1.record()
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / 1e3 / reps


def time_graph(f, dev, reps=50):
    """Average HIP-event time (s) per launch of `reps` launches of a bound C-ABI call replayed
    from one HIP graph: the GPU-side time per kernel, without the host's issue rate
    (eager launches from Python cost >= 3.6 us each even for an empty kernel:
    tools/launch_ceiling.py)."""
    gs = torch.cuda.Stream(dev)
    with torch.cuda.stream(gs):
        f(gs.cuda_stream)
        torch.cuda.synchronize(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=gs):
            for _ in range(reps):
                f(gs.cuda_stream)
    g.replay()
    torch.cuda.synchronize(dev)
    rs = torch.cuda.current_stream(dev)  # replay() runs on the current stream
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(rs)
    g.replay()
    e1.record(rs)
    torch.cuda.synchronize(dev)
    return e0.elapsed_time(e1) / 1e3 / reps


def step_kernels_vs_copy(dev):
    """Each stepwise env kernel alone (one launch = one env step over the batch, state
    re-read from where the previous launch left it, as in the stepwise graphs) beside
    co_probe_copy moving the same bytes through the same kind of buffer (one buffer pair
    reused, i.e. Infinity-Cache resident like the stepwise state): the small-launch
    ceiling a step kernel of that size can reach.  Bytes per env
    step: SURVEY.md 8d (TSP 2N+50, CVRP 7N+33, SLAP 2L+34).  Both timed as HIP-graph
    replays (time_graph: the GPU-side time per launch, as inside the stepwise graphs); the
    eager (Python-issued) times beside them sit at the host's issue floor for the copy."""
    from rl4co_slap_amd import _native as nat

    out = {}
    d = dev

    def copy_us(nbytes):
        n = (nbytes // 2) // 16 * 16
        a, c = torch.ones(n, dtype=torch.uint8, device=d), torch.empty(n, dtype=torch.uint8, device=d)
        f = nat.bind("co_probe_copy", nat.ptr(a), nat.ptr(c), n)
        return time_graph(f, d) * 1e6, time_bound(f, d) * 1e6

    def rec(name, f, nbytes):
        us, us_eager = time_graph(f, d) * 1e6, time_bound(f, d) * 1e6
        cu, cu_eager = copy_us(nbytes)
        out[name] = {"bytes": nbytes, "kernel_us": us, "kernel_GBps": nbytes / us / 1e3,
                     "copy_same_bytes_us": cu, "copy_GBps": nbytes / cu / 1e3,
                     "frac_of_copy": cu / us, "hbm_frac": nbytes / us / 1e3 / HBM_PEAK_GBS,
                     "kernel_us_eager": us_eager, "copy_same_bytes_us_eager": cu_eager}

    # TSP-100, B = 65,536 (co_tsp_step, first_mode 0)
    b, n = 65536, 100
    act = torch.randint(0, n, (b,), device=d)
    mask = torch.ones(b, n, dtype=torch.bool, device=d)
    i = torch.zeros(b, 1, dtype=torch.int64, device=d)
    first, cur = torch.zeros(b, dtype=torch.int64, device=d), torch.empty(b, dtype=torch.int64, device=d)
    done, rw = torch.empty(b, dtype=torch.bool, device=d), torch.empty(b, dtype=torch.bool, device=d)
    st = torch.zeros(1, dtype=torch.int32, device=d)
    f = nat.bind("co_tsp_step", b, n, nat.ptr(act), nat.ptr(mask), nat.ptr(mask), nat.ptr(i),
                 nat.ptr(i), nat.ptr(first), nat.ptr(first), nat.ptr(cur), nat.ptr(done),
                 nat.ptr(rw), 0, None, nat.ptr(st))
    rec("tsp_step_b65536", f, b * (2 * n + 50))
    del act, mask, i, first, cur, done, rw
    # CVRP-100, B = 32,768 (co_cvrp_step, fused mask)
    b = 32768
    act = torch.randint(0, n + 1, (b,), device=d)
    dem = torch.rand(b, n, device=d) * 0.1
    used, used2 = torch.zeros(b, 1, device=d), torch.zeros(b, 1, device=d)
    vcap = torch.ones(b, 1, device=d)
    vis = torch.zeros(b, n + 1, dtype=torch.uint8, device=d)
    cur = torch.empty(b, dtype=torch.int64, device=d)
    done, rw = torch.empty(b, dtype=torch.bool, device=d), torch.empty(b, dtype=torch.bool, device=d)
    m = torch.empty(b, n + 1, dtype=torch.bool, device=d)
    f = nat.bind("co_cvrp_step", b, n, nat.ptr(act), nat.ptr(dem), nat.ptr(used), nat.ptr(used2),
                 nat.ptr(vcap), nat.ptr(vis), nat.ptr(vis), nat.ptr(cur), nat.ptr(done), nat.ptr(rw),
                 nat.ptr(m), nat.ptr(st), None)
    rec("cvrp_step_b32768", f, b * (7 * n + 33))
    del act, dem, used, used2, vcap, vis, cur, done, rw, m
    # SLAP, B = 16,384, L = 100, P = 20 (co_slap_step, in-place assignment)
    b, l, pp = 16384, 100, 20
    act = torch.randint(1, l, (b,), device=d)
    tc = torch.arange(pp, dtype=torch.float32, device=d).repeat(b, 1)
    asg = torch.full((b, pp), -1, dtype=torch.int32, device=d)
    mask = torch.ones(b, l, dtype=torch.bool, device=d)
    i = torch.zeros(b, 1, dtype=torch.int64, device=d)
    done, rw = torch.empty(b, 1, dtype=torch.bool, device=d), torch.empty(b, 1, dtype=torch.bool, device=d)
    f = nat.bind("co_slap_step", b, l, pp, nat.ptr(act), nat.ptr(tc), pp, nat.ptr(asg), nat.ptr(asg),
                 nat.ptr(mask), nat.ptr(mask), nat.ptr(i), nat.ptr(i), nat.ptr(done), nat.ptr(rw),
                 nat.ptr(st))
    rec("slap_step_b16384", f, b * (2 * l + 34))
    # the bench policy fused with it (co_slap_closest_step): + depot distances 4L read
    dd = torch.rand(b, l, device=d)
    f = nat.bind("co_slap_closest_step", b, l, pp, nat.ptr(dd), nat.ptr(tc), pp, nat.ptr(asg),
                 nat.ptr(asg), nat.ptr(mask), nat.ptr(mask), nat.ptr(act), nat.ptr(i), nat.ptr(i), nat.ptr(done),
                 nat.ptr(rw), nat.ptr(st))
    rec("slap_closest_step_b16384", f, b * (6 * l + 34))
    return out


def cpu_threads():
    """Threads for the CPU baseline: the CPU share this process was given.  On the GPU pool
    a one-GPU job owns 16 of the host's CPUs (OMP_NUM_THREADS is set to that share);
    os.cpu_count() counts the whole host, whose other CPUs belong to the jobs on its other
    GPUs -- running 256 threads there would time oversubscription, not the reference."""
    return int(os.environ.get("OMP_NUM_THREADS", "0")) or min(os.cpu_count() or 1, 16)


def _loadavg():
    try:
        return [round(x, 2) for x in os.getloadavg()]
    except OSError:
        return None


def _spread(times, work, load_before=None):
    """min / median / max rate over the timed episodes (the first, a warm-up, dropped), and
    the host's load average (1 / 5 / 15 min) before and after them: a CPU baseline taken
    on a loaded host reads low, and the driver's records should show it."""
    ts = sorted(times[1:])
    return {"value": work / ts[len(ts) // 2], "value_min": work / ts[-1], "value_max": work / ts[0],
            "episodes": len(ts), "host_loadavg_before": load_before,
            "host_loadavg_after": _loadavg()}


def host_cpu():
    """The host the CPU baseline ran on (BASELINE.md 2 asks for the CPU model and cores)."""
    model, cores, sockets = None, set(), set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name" and model is None:
                model = v
            elif k == "physical id":
                phys = v
                sockets.add(v)
            elif k == "core id":
                core = v
                cores.add((phys, core))
    except OSError:
        pass
    return {"cpu_model": model, "logical_cpus": os.cpu_count(),
            "physical_cores": len(cores) or None, "sockets": len(sockets) or None,
            "threads_used": cpu_threads(),
            "aten_capability": torch.backends.cpu.get_cpu_capability()}


def cpu_baseline_tsp(locs, acts, episodes=5):
    """The oracle (reference op sequence on CPU torch) on the same TSP workload."""
    from oracle.envs import TSPOracle
    from oracle.rollout import rollout
    from oracle.td import TD

    threads = cpu_threads()
    torch.set_num_threads(threads)
    b, n = acts.shape
    env = TSPOracle(num_loc=n, seed=1234)
    times, load0 = [], _loadavg()
    for _ in range(episodes + 1):
        td = env.reset(TD({"locs": locs}, [b]))
        it = iter(range(n))
        t0 = time.perf_counter()
        rollout(env, td, lambda td: acts[:, next(it)])
        times.append(time.perf_counter() - t0)
    return {**_spread(times, b * n, load0), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle (CPU PyTorch restatement) TSP-{n} teacher-forced rollout: reset + "
                      f"{n} x _step + get_reward with the double validity sort, B={b} (the full "
                      f"GPU workload), median (min / max beside it) of {episodes} episodes after "
                      f"1 warm-up, torch.set_num_threads({threads}) = the job's CPU share"}


def cpu_baseline_slap(b=16384, episodes=5):
    """The oracle's SLAP rollout at config 4's batch (the GPU modes' B=16,384): the
    closest-free policy, the per-batch Python loop of slap/env.py:61-62 and the per-order
    reward loop kept.  The instances' grid columns (identical for every instance: the
    generator's analytic aisle grid) come from one generated block of 2,048 tiled to B --
    the generator's own B x L Python loop (slap/generator.py:67-81) is not the workload
    timed; freq and picklists are drawn for all B."""
    import numpy as np

    from oracle.envs import SLAPOracle, slap_closest_free_action
    from oracle.rollout import rollout
    from oracle.td import TD

    torch.set_num_threads(cpu_threads())
    env = SLAPOracle(seed=1234)
    np.random.seed(1234)
    blk = min(b, 2048)
    g0 = env.generate([blk])
    reps = (b + blk - 1) // blk
    gen = {k: torch.cat([g0[k]] * reps)[:b] for k in ("locs", "dist_mat", "depot_loc_dist",
                                                    "assignment")}
    gen["freq"] = env.freq_sampler.sample((b, env.n_products, 1))
    gen["picklist"] = env.picklist([b])
    gen = TD(gen, [b])
    times, load0 = [], _loadavg()
    for _ in range(episodes + 1):
        td = env.reset(TD({k: v.clone() for k, v in gen.items()}, [b]))
        t0 = time.perf_counter()
        rollout(env, td, slap_closest_free_action)
        times.append(time.perf_counter() - t0)
    return {**_spread(times, b * 20, load0), "unit": "env-steps/s", "cores": cpu_threads(),
            "kind": "port",
            "sample": f"oracle SLAP rollout (closest-free policy, per-batch Python loop of "
                      f"slap/env.py:61-62 kept), B={b}, median (min / max) of {episodes} "
                      f"episodes after 1 warm-up"}


def cpu_baseline_cvrp(b=32768, n=100, episodes=5):
    """The oracle's CVRP-100 rollout with the nearest-feasible policy (config 3 recipe and
    batch), including get_reward's Python capacity loop."""
    from oracle.envs import CVRPOracle, cvrp_nearest_action
    from oracle.rollout import rollout
    from oracle.td import TD

    threads = cpu_threads()
    torch.set_num_threads(threads)
    torch.manual_seed(1234)
    locs_all = torch.rand(b, n + 1, 2)
    demand = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
    env = CVRPOracle(num_loc=n, seed=1234)
    times, steps, load0 = [], 0, _loadavg()
    for _ in range(episodes + 1):
        td = env.reset(TD({"depot": locs_all[:, 0].clone(), "locs": locs_all[:, 1:].clone(),
                           "demand": demand.clone(),
                           "capacity": torch.full((b, 1), 50.0)}, [b]))
        t0 = time.perf_counter()
        _, _, acts = rollout(env, td, cvrp_nearest_action)
        times.append(time.perf_counter() - t0)
        steps = acts.shape[1]
    return {**_spread(times, b * steps, load0), "unit": "env-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"oracle CVRP-{n} rollout, nearest-feasible policy, B={b} (config 3, the "
                      f"GPU batch), T={steps} steps, get_reward with the validity + capacity "
                      f"loop, median (min / max) of {episodes} episodes after 1 warm-up"}


def cpu_baseline_pomo(b=256, n=100, episodes=5):
    """The oracle's POMO TSP-100 episode (the restated multistart loop on
    CPU, a stated subset of config 5's 8,192 x 100 envs): ``constructive_forward`` with
    multistart greedy decoding (``decoding.py:265-313``: batchify x S, the start step,
    N-1 decode steps of tanh clip 10 -> mask -> log_softmax -> argmax on fixed step-major
    logits, as the GPU mode feeds them), the reward with its validity check, then the
    shared-baseline REINFORCE loss (``pomo/model.py:87-144``, ``reinforce.py:97-115``).
    B = 256 instances x S = 100 starts = 25,600 envs (the GPU mode: 1,024 x 100 per GPU)."""
    from oracle.envs import TSPOracle
    from oracle.rollout import constructive_forward, pomo_loss
    from oracle.td import TD

    threads = cpu_threads()
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(1234)
    locs = torch.rand(b, n, 2, generator=g)
    logits = torch.randn(n - 1, n * b, n, generator=g)
    env = TSPOracle(num_loc=n, seed=1234)
    times, load0 = [], _loadavg()
    for _ in range(episodes + 1):
        td = env.reset(TD({"locs": locs.clone()}, [b]))
        it = iter(range(n - 1))
        t0 = time.perf_counter()
        out = constructive_forward(td, env, lambda t: logits[next(it)],
                                   decode_type="multistart_greedy", tanh_clipping=10.0)
        pomo_loss(out["reward"], out["log_likelihood"], n)
        times.append(time.perf_counter() - t0)
    return {**_spread(times, b * n * n, load0), "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle POMO TSP-{n} episode: constructive_forward multistart greedy "
                      f"(batchify x {n} starts, start step + {n - 1} decode steps, tanh clip 10, "
                      f"fixed step-major logits) + reward with validity + shared-baseline loss, "
                      f"B={b} instances x {n} starts = {b * n} envs (config 5 subset; the GPU "
                      f"mode runs 1,024 x {n} per GPU), median (min / max) of {episodes} "
                      f"episodes after 1 warm-up"}


def pmc_traffic(target, kernel_prefix):
    """HBM bytes per launch measured by rocprofv3 PMC passes (scripts/gpu_pmc.sh ->
    tools/pmc_summarize.py -> profiles/*_pmc_traffic.json, newest round first)."""
    import glob

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json")), reverse=True):
        try:
            data = json.load(open(f))
        except (OSError, ValueError):
            continue
        for e in data.get("kernels", {}).values():
            if e.get("target") == target and e.get("kernel", "").startswith(kernel_prefix) \
                    and "hbm_bytes_per_launch" in e:
                return e["hbm_bytes_per_launch"], os.path.basename(f)
    return None, None


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    world, rank, dev = setup_dist(args)
    if args.dry_run:
        return dry_run(args, world, rank, dev)
    from rl4co_slap_amd import _native
    from rl4co_slap_amd.rollout.engine import TSPFusedEpisode, TSPStepwiseEpisode

    _native.load()
    b, n = args.batch, args.num_loc
    locs_cpu, acts_cpu = tsp_inputs(b, n, rank)
    locs, acts = locs_cpu.to(dev), acts_cpu.to(dev)

    # ---- headline: fused one-launch episode, eager back-to-back launches ---------------
    # distinct batches cycled (16 B of inputs per node and instance): every launch reads
    # its inputs from HBM, not from the Infinity Cache after the previous launch
    n_rot = rotation(b * n * 16)
    eps = [TSPFusedEpisode(locs, acts, policy="teacher", check=True)]
    for r in range(1, n_rot):
        lr, ar = tsp_inputs(b, n, rank, salt=r)
        eps.append(TSPFusedEpisode(lr.to(dev), ar.to(dev), policy="teacher", check=True))
    sh = torch.cuda.current_stream(dev).cuda_stream  # launch stream, looked up once
    cyc = itertools.cycle([e._bound for e in eps])
    s = lambda: next(cyc)(sh)  # noqa: E731
    wall, ev = timed(s, args.steps, args.warmup, world, dev)
    assert all(int(e.status.item()) == 0 for e in eps), "invalid tour in the benchmark episode"
    del eps
    t = max_over_ranks(wall, world, dev)
    value = world * b * n * args.steps / t
    per_launch = ev / args.steps
    bytes_per_launch = b * (17 * n + 30)  # co_tsp_rollout algorithmic bytes
    achieved = bytes_per_launch / per_launch / 1e9
    traffic, traffic_src = (None, None)
    if (b, n) == (65536, 100):
        traffic, traffic_src = pmc_traffic("tsp_fused_teacher", "tsp_teacher_rows_kernel<")

    out = {
        "metric": "env-steps/sec (batch×decode) SLAP & TSP-100 at 1/2/4/8 MI355X",
        "value": value, "unit": "env-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": t / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8+i64+f32",
        "data": "synthetic: seeded torch.rand TSP instances, teacher-forced argsort actions",
        "config": {"workload": f"TSP-{n} B={b}/GPU teacher-forced episode (reset + {n} env steps + "
                               "reward + validity) as one fused launch (co_tsp_rollout_ex on the "
                               "reference's row-major [B, N] actions; BASELINE config 2). A "
                               "final-state-only episode: the per-step TensorDict states are not "
                               "written to HBM, so its env-steps/s is not comparable with a "
                               "per-step loop -- that figure is `tsp_stepwise`",
                   "episode_kind": "fused, final state only",
                   "batch_per_gpu": b, "num_loc": n, "env_steps_per_episode": n,
                   "parallelism": f"dp{world}: disjoint instance shards, no data-path collective"},
        "roofline": {"bound": "hbm",
                     "kernel": "tsp_teacher_rows_kernel<16,7,2,true> (co_tsp_rollout_ex, "
                               "row-major [B, N] actions; 16 lanes x 7 steps per instance)",
                     "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     # the same bytes over the wall time `value` uses (launch gaps included)
                     "achieved_wall": bytes_per_launch / (t / args.steps) / 1e9,
                     "frac_wall": bytes_per_launch / (t / args.steps) / 1e9 / HBM_PEAK_GBS,
                     "traffic_source": traffic_src,
                     "bytes_per_launch": bytes_per_launch, "launch_us": per_launch * 1e6,
                     "copy_probe": copy_probe(bytes_per_launch, dev, args.steps)},
    }
    out["config"]["input_batches_cycled"] = n_rot

    # ---- the contract-faithful per-step TSP loop: one launch per env step,
    # every step's TensorDict state written to and re-read from HBM (2N+50 B per env-step,
    # + the episode reward's 16N+4 B amortised), HIP graph of reset + N steps + reward
    k = max(3, args.steps // 5)
    sw = TSPStepwiseEpisode(locs, acts, policy="teacher", check=True).capture()
    wall_s, ev_s = timed(sw.replay, k, 2, world, dev)
    assert int(sw.status.item()) == 0, "TSP stepwise episode status"
    del sw
    t_s = max_over_ranks(wall_s, world, dev)
    sw_bytes = 2 * n + 50 + (16 * n + 4) / n
    out["tsp_stepwise"] = {
        "value": world * b * n * k / t_s, "unit": "env-steps/s", "ms_per_episode": t_s / k * 1e3,
        "workload": f"TSP-{n} B={b}/GPU teacher-forced episode, one co_tsp_step launch per env "
                    "step (state in HBM between steps, as the reference loop), reset + reward "
                    "included, HIP graph",
        "launches_per_step": 1, "alg_bytes_per_env_step": sw_bytes,
        "achieved_GBps": b * n * sw_bytes * k / ev_s / 1e9,
        "frac": b * n * sw_bytes * k / ev_s / 1e9 / HBM_PEAK_GBS,
        "frac_wall": b * n * sw_bytes * k / wall_s / 1e9 / HBM_PEAK_GBS}
    # ---- the same per-step loop with the steps in chunks of 10 per launch (co_tsp_steps,
    # round 6): every step's state is still written to HBM (the ping-pong buffers, as the
    # one-launch-per-step loop writes them; bit-identical), the state is carried in
    # registers inside a chunk instead of re-read.  Bytes it moves per env-step: the mask
    # row N + action 8 + i / first / current 24 + done / reward 2, the chunk's state read
    # (N + 16) / 10, the reward's (16N + 4) / N -- not the one-launch contract's 2N + 50.
    kc = 10
    swc = TSPStepwiseEpisode(locs, acts, policy="teacher", check=True, chunk=kc).capture()
    wall_c, ev_c = timed(swc.replay, k, 2, world, dev)
    assert int(swc.status.item()) == 0, "TSP chunked stepwise episode status"
    del swc
    t_c = max_over_ranks(wall_c, world, dev)
    swc_bytes = n + 34 + (n + 16) / kc + (16 * n + 4) / n
    out["tsp_stepwise_chunked"] = {
        "value": world * b * n * k / t_c, "unit": "env-steps/s", "ms_per_episode": t_c / k * 1e3,
        "workload": f"TSP-{n} B={b}/GPU teacher-forced episode, {kc} env steps per co_tsp_steps "
                    "launch (every step's state written to HBM), reset + reward included, HIP "
                    "graph",
        "steps_per_launch": kc, "alg_bytes_per_env_step": swc_bytes,
        "contract_bytes_per_env_step_one_launch_loop": sw_bytes,
        # PMC (profiles/r*_pmc_traffic.json): inside a launch the L2 absorbs the ping-pong
        # rewrites (a row's buffer is rewritten every second step), so HBM sees less than
        # the bytes the kernel issues; the mode is bounded by store issue + launch count
        "pmc_hbm_bytes_per_env_step_steps_kernel": (
            lambda t: None if t is None else t / (b * kc))(
            pmc_traffic("tsp_stepwise_chunked", "tsp_steps_group_kernel<")[0]) if (b, n) == (65536, 100) else None,
        "achieved_GBps": b * n * swc_bytes * k / ev_c / 1e9,
        "frac": b * n * swc_bytes * k / ev_c / 1e9 / HBM_PEAK_GBS,
        "frac_wall": b * n * swc_bytes * k / wall_c / 1e9 / HBM_PEAK_GBS}
    # ---- SLAP at the north star's batch (B = 65,536; examples/slap.py instance)
    slap65 = bench_slap(65536, k, world, rank, dev)
    fc, sc = slap65["slap_fused_closest"], slap65["slap_stepwise_graph"]
    s_traffic, s_src = pmc_traffic("slap_fused_closest_b65536", "slap_group_kernel<16, 8, true>")
    out["slap_b65536"] = {
        "value": fc["value"], "unit": "env-steps/s", "ms_per_episode": fc["ms_per_episode"],
        "workload": "SLAP (examples/slap.py:75-76: L=100, P=20 products, O=20 orders x K=5) "
                    "B=65,536/GPU, closest-free policy: reset + 20 env steps + pick-tour reward "
                    "as one fused launch (co_slap_rollout); final state only, like the TSP "
                    "headline",
        "roofline": {"bound": "hbm", "kernel": "slap_group_kernel<16,8,true> (co_slap_rollout)",
                     "achieved": fc["achieved_GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": fc["achieved_GBps"] / HBM_PEAK_GBS, "traffic": s_traffic,
                     "traffic_source": s_src, "bytes_per_launch": 65536 * 2754,
                     "launch_us": fc["launch_us"]},
        "stepwise": {"value": sc["value"], "ms_per_episode": sc["ms_per_episode"],
                     "launches_per_step": 1, "policy": sc["policy"],
                     "alg_bytes_per_env_step": 234 + 1684 / 20,
                     "frac_wall": sc["value"] / world * (234 + 1684 / 20) / 1e9 / HBM_PEAK_GBS},
        "stepwise_chunked": {k_: slap65["slap_stepwise_chunked"][k_] for k_ in (
            "value", "ms_per_episode", "steps_per_launch", "alg_bytes_per_env_step", "frac",
            "frac_wall")}}

    if not args.no_modes:
        modes = {}
        modes["tsp_stepwise_graph"] = {
            "value": out["tsp_stepwise"]["value"], "ms_per_episode": t_s / k * 1e3,
            "bytes_per_env_step": 2 * n + 50,
            "achieved_GBps_incl_reset_reward": b * n * (2 * n + 50) * k / ev_s / 1e9}
        # in-kernel nearest-unvisited policy, fused
        ne = TSPFusedEpisode(locs, None, policy="nearest", check=True)
        sn = lambda: ne._launch(sh)  # noqa: E731
        wall_n, ev_n = timed(sn, k, 1, world, dev)
        t_n = max_over_ranks(wall_n, world, dev)
        modes["tsp_fused_nearest"] = {"value": world * b * n * k / t_n,
                                      "ms_per_episode": t_n / k * 1e3}
        del ne
        # the drop-in API path (ConstructivePolicy + TSPEnv, one decode + one env launch
        # per step, Python TensorDict plumbing)
        modes["dropin_tsp100"] = bench_dropin(b, n, k, world, rank, dev)
        modes["dropin_cvrp100"] = bench_dropin_cvrp(32768, 100, k, world, rank, dev)
        # the fork's SLAP policy path (examples/slap.py): config 4's batch and the north star's
        modes["dropin_slap_b16384"] = bench_dropin_slap(args.slap_batch, k, world, rank, dev)
        modes["dropin_slap_b65536"] = bench_dropin_slap(65536, k, world, rank, dev)
        # SLAP (examples/slap.py instance), closest-free policy: fused and stepwise
        modes.update(bench_slap(args.slap_batch, k, world, rank, dev))
        # the north star's "SLAP at batch 65,536": fused and stepwise (measured above)
        modes.update({k2 + "_b65536": v for k2, v in slap65.items()})
        # POMO TSP-100 (config 5): 1,024 instances x 100 starts per GPU, decode-fused steps
        # on HBM-resident logits, shared baseline + RCCL all-gather of per-instance results
        # default decode math = certified (exact greedy actions, logp within 1e-5)
        modes["pomo_tsp100"] = bench_pomo(1024, n, max(2, k // 2), world, rank, dev)
        # the ATen-exact math (log-probabilities bit for bit; opt-in, decode_math="exact")
        modes["pomo_tsp100_exact"] = bench_pomo(1024, n, max(2, k // 2), world, rank, dev,
                                                decode_math="exact")
        # the opt-in CO_DECODE_FAST math (not bit-exact; reported separately)
        modes["pomo_tsp100_fast_math"] = bench_pomo(1024, n, max(2, k // 2), world, rank, dev,
                                                    decode_math="fast")
        # CVRP-100 (config 3), nearest-feasible policy: fused episode and stepwise loop
        modes.update(bench_cvrp(32768, 100, k, world, rank, dev))
        # instance generation, timed separately (SURVEY.md 8d protocol; 8f rank 1)
        modes["slap_generate_b16384"] = bench_generate_slap(args.slap_batch, dev,
                                                            with_ref=(rank == 0 and world == 1))
        modes["tsp_cvrp_generate"] = bench_generate_uniform(b, n, dev)
        annotate_modes(modes, n, world)
        out["modes"] = modes
        out["step_kernels_vs_copy"] = step_kernels_vs_copy(dev)

    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline_tsp(locs_cpu, acts_cpu)
        out["cpu_baseline"]["host"] = host_cpu()
        if not args.no_modes:
            out["cpu_baseline_slap"] = cpu_baseline_slap()
            out["cpu_baseline_cvrp"] = cpu_baseline_cvrp()
            out["cpu_baseline_pomo"] = cpu_baseline_pomo()
    if rank == 0:
        out["build"] = _native.provenance()  # the sources the measured library came from
        out["summary"] = summarize(out)
        # contract keys first, the long mode tables next, and the short records a reader
        # (and the driver's stdout tail) needs LAST: the stepwise / SLAP-65,536 figures and
        # the summary of every mode end the line
        order = ["metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                 "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
                 "roofline", "cpu_baseline"]
        last = ["tsp_stepwise", "tsp_stepwise_chunked", "slap_b65536", "summary"]
        final = {key: out[key] for key in order if key in out}
        final.update({key: v for key, v in out.items() if key not in final and key not in last})
        final.update({key: out[key] for key in last if key in out})
        print(json.dumps(final), flush=True)
    if world > 1:
        dist.destroy_process_group()


def pmc_sq_issue(target, kernel):
    """(SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES, file) of `target`'s main kernel from the newest
    committed profiles/r*_pmc_sq.txt (scripts/gpu_pmc_sq.sh), or None."""
    import glob
    import re

    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_sq.txt")), reverse=True):
        try:
            lines = open(f).read().splitlines()
        except OSError:
            continue
        for i, line in enumerate(lines[:-1]):
            w = line.split()
            if len(w) >= 2 and w[0] == target and w[1].startswith(kernel):
                m = re.search(r"\bactive=([0-9.eE+-]+)", lines[i + 1])
                if m:
                    return float(m.group(1)), os.path.basename(f)
    return None


def summarize(out):
    """The figures a reader needs first, in one short record: every per-GPU rate with its
    HBM fraction, the drop-in loops' launches / GPU / host time per step."""
    r = lambda x, d=3: None if x is None else round(float(x), d)  # noqa: E731
    sm = {"tsp100_fused_final_state": {"env_steps_s": r(out["value"], 0),
                                       "frac": r(out["roofline"]["frac"]),
                                       "frac_wall": r(out["roofline"]["frac_wall"])}}
    if "tsp_stepwise" in out:
        t = out["tsp_stepwise"]
        sm["tsp100_stepwise"] = {"env_steps_s": r(t["value"], 0), "frac": r(t["frac"]),
                                 "frac_wall": r(t["frac_wall"])}
    if "tsp_stepwise_chunked" in out:
        t = out["tsp_stepwise_chunked"]
        sm["tsp100_stepwise_chunked"] = {"env_steps_s": r(t["value"], 0), "frac": r(t["frac"]),
                                         "frac_wall": r(t["frac_wall"]),
                                         "steps_per_launch": t["steps_per_launch"]}
    if "slap_b65536" in out:
        t = out["slap_b65536"]
        sm["slap_b65536_fused"] = {"env_steps_s": r(t["value"], 0),
                                   "frac": r(t["roofline"]["frac"])}
        sm["slap_b65536_stepwise"] = {"env_steps_s": r(t["stepwise"]["value"], 0),
                                      "frac_wall": r(t["stepwise"]["frac_wall"])}
        if "stepwise_chunked" in t:
            c = t["stepwise_chunked"]
            sm["slap_b65536_stepwise_chunked"] = {
                "env_steps_s": r(c["value"], 0), "frac": r(c["frac"]),
                "frac_wall": r(c["frac_wall"]), "steps_per_launch": c["steps_per_launch"]}
    # the same run's streaming ceiling (co_probe_copy of 2 GiB): each rate below also as a
    # fraction of it, so a box that streams slower shows up here, not as a regression
    cp = out["roofline"].get("copy_probe", {})
    copy_gbs = cp.get("2GiB", {}).get("GBps")
    sm["copy_GBps"] = r(copy_gbs, 1)
    sm["copy_same_bytes_GBps"] = r(cp.get("same_bytes", {}).get("GBps"), 1)
    foc = lambda gbs: r(gbs / copy_gbs) if gbs and copy_gbs else None  # noqa: E731
    sm["tsp100_fused_final_state"]["frac_of_copy"] = foc(out["roofline"]["achieved"])
    modes = out.get("modes", {})
    for name in ("dropin_tsp100", "dropin_cvrp100", "dropin_slap_b16384", "dropin_slap_b65536"):
        m = modes.get(name)
        if not m:
            continue
        steps = m.get("episode_steps") or m.get("env_steps_per_episode") or 100
        sm[name] = {"env_steps_s": r(m["value"], 0), "ms_per_episode": r(m["ms_per_episode"]),
                    "launches_per_step": m.get("launches_per_step"),
                    "gpu_us_per_step": r(m["gpu_ms_per_episode"] * 1e3 / steps, 2),
                    # host time per step at B = 64: the whole episode's (reset, reward,
                    # epilogue included) and the marginal loop step (episodes of P and 2P)
                    "host_us_per_step_b64_all_in": r(m.get("host_us_per_step_b64"), 2),
                    "host_us_per_loop_step_b64": r(m.get("host_us_per_loop_step_b64"), 2),
                    "decode_fused_kernel_us": r(m.get("decode_fused_kernel_us"), 2),
                    "hbm_frac": r(m.get("hbm_frac")),
                    "frac_of_copy": foc(m.get("achieved_GBps_per_gpu"))}
    for name in ("pomo_tsp100", "tsp_fused_nearest", "cvrp_fused_nearest", "cvrp_stepwise_graph"):
        m = modes.get(name)
        if m:
            sm[name] = {"env_steps_s": r(m["value"], 0), "ms_per_episode": r(m["ms_per_episode"]),
                        "hbm_frac": r(m.get("hbm_frac")),
                        "frac_of_copy": foc(m.get("achieved_GBps_per_gpu"))}
    sk = out.get("step_kernels_vs_copy", {})
    if sk:
        sm["step_kernels_frac_of_copy"] = {k2: r(v["frac_of_copy"]) for k2, v in sk.items()}
    for name in ("cpu_baseline", "cpu_baseline_slap", "cpu_baseline_cvrp", "cpu_baseline_pomo"):
        c = out.get(name)
        if c:
            sm[name] = {"value": r(c["value"], 0), "min": r(c.get("value_min"), 0),
                        "max": r(c.get("value_max"), 0), "threads": c["cores"],
                        "loadavg_1m": [(c.get("host_loadavg_before") or [None])[0],
                                       (c.get("host_loadavg_after") or [None])[0]]}
    # every other rate with an HBM fraction: the same fraction of this run's copy ceiling
    for v in sm.values():
        if isinstance(v, dict) and "frac_of_copy" not in v and copy_gbs:
            f = v.get("hbm_frac", v.get("frac", v.get("frac_wall")))
            if f is not None:
                v["frac_of_copy"] = r(f * HBM_PEAK_GBS / copy_gbs)
    return sm


def dry_run(args, world, rank, dev):
    """CPU rehearsal of the launch / reduction / JSON path (no GPU, no HIP library): each
    gloo rank runs the oracle's TSP teacher episode on its own instance shard as the
    step, ranks are timed with the same barrier + max-over-ranks protocol, and the POMO
    all-gather runs on the oracle's per-instance baseline values."""
    from oracle.envs import TSPOracle
    from oracle.rollout import rollout
    from oracle.td import TD
    from rl4co_slap_amd.rollout.pomo import global_metrics

    b, n = min(args.batch, 512), min(args.num_loc, 20)
    locs, acts = tsp_inputs(b, n, rank)
    env = TSPOracle(num_loc=n, seed=1234)

    def step():
        it = iter(range(n))
        rollout(env, env.reset(TD({"locs": locs}, [b])), lambda td: acts[:, next(it)])

    for _ in range(args.warmup):
        step()
    barrier(world)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    barrier(world)
    t = max_over_ranks(time.perf_counter() - t0, world, dev)
    g = torch.Generator().manual_seed(rank)
    rw = -torch.rand(b, n, generator=g) * 10
    m = global_metrics(rw.mean(1), rw.max(1).values, torch.zeros(b), n)
    out = {"metric": "env-steps/sec (batch×decode) SLAP & TSP-100 at 1/2/4/8 MI355X",
           "value": world * b * n * args.steps / t, "unit": "env-steps/s", "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": t / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "u8+i64+f32", "data": "dry run: CPU oracle episode per gloo rank, no GPU",
           "config": {"workload": f"TSP-{n} B={b}/rank oracle episode (dry run)",
                      "batch_per_gpu": b, "num_loc": n, "dry_run": True,
                      "parallelism": f"dp{world}: disjoint instance shards, no data-path "
                                     "collective"},
           "allgather_instances": m["instances"]}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def annotate_modes(modes, n, world):
    """Algorithmic HBM bytes per env-step of each mode (SURVEY.md 8d definitions; fused
    modes: their kernels' own input/output bytes) -> per-GPU achieved
    GB/s and the fraction of the 8 TB/s peak."""
    per_step = {
        "tsp_stepwise_graph": lambda m: 2 * n + 50 + (16 * n + 4) / n,
        "dropin_tsp100": lambda m: 2 * n + 50 + 5 * n + 16 + (16 * n + 4) / n,
        # decode: logits + mask read, action + logp written; the CVRP step as stepwise
        # the decode-fused CVRP step: logits 4(N+1) + mask N+1 read, logp out (the action
        # written instead of read), the env step's 7N+33 + the episode reward
        "dropin_cvrp100": lambda m: 5 * (n + 1) + 4 + 7 * n + 33 + (16 * m["episode_steps"] + 12)
        / m["episode_steps"],
        "dropin_slap_b16384": lambda m: 234 + 404 + 1684 / 20,
        "dropin_slap_b65536": lambda m: 234 + 404 + 1684 / 20,
        "tsp_fused_nearest": lambda m: (17 * n + 30) / n,
        "slap_fused_closest": lambda m: 2754 / 20,
        "slap_fused_closest_b65536": lambda m: 2754 / 20,
        "slap_fused_random": lambda m: 2354 / 20,
        "slap_fused_random_b65536": lambda m: 2354 / 20,
        "slap_stepwise_graph": lambda m: 234 + 1684 / 20,
        "slap_stepwise_graph_teacher": lambda m: 234 + 1684 / 20,
        "slap_stepwise_graph_b65536": lambda m: 234 + 1684 / 20,
        "slap_stepwise_graph_teacher_b65536": lambda m: 234 + 1684 / 20,
        "pomo_tsp100": lambda m: 6 * n + 54,
        "pomo_tsp100_fast_math": lambda m: 6 * n + 54,
        "pomo_tsp100_exact": lambda m: 6 * n + 54,
        "cvrp_fused_nearest": lambda m: (8 + 12 * n + 8 * m["episode_steps"] + 10 * (n + 1) + 25)
        / m["episode_steps"],
        # fused policy: locs 8(N+1) + mask, visited N+1 each + demand 4N + 16 B state read;
        # visited, mask N+1 each + 22 B state written -- plus the episode's reward kernel
        "cvrp_stepwise_graph": lambda m: 16 * n + 50 + (16 * m["episode_steps"] + 12)
        / m["episode_steps"],
        "cvrp_stepwise_graph_pair": lambda m: 7 * n + 33 + (16 * m["episode_steps"] + 12)
        / m["episode_steps"],
    }
    for name, f in per_step.items():
        if name in modes and "value" in modes[name]:
            m = modes[name]
            byts = f(m)
            gbs = m["value"] / world * byts / 1e9
            m.update({"alg_bytes_per_env_step": byts, "achieved_GBps_per_gpu": gbs,
                      "hbm_frac": gbs / HBM_PEAK_GBS, "bound": "hbm"})
    # the in-kernel nearest policies are O(N^2) vector ALU work on LDS / register-resident
    # coordinates, not HBM traffic: per env-step one squared distance
    # per candidate (2 sub + 2 mul + 1 add = 5 FLOP), against the 157.3 TFLOP/s FP32
    # vector peak (MI355X_MICROARCH.md).  The FLOP fraction is small because the bound is
    # VALU *issue*: the key / min / second-min bookkeeping (3 integer ops per candidate)
    # and the per-step group reduction are instructions too, and a wave64 instruction takes
    # ~5 SIMD cycles at 4 waves per SIMD (tools/valu_rates.py); DESIGN.md section 4 counts
    # the instructions per instance-step.
    for name, cand in (("tsp_fused_nearest", n), ("cvrp_fused_nearest", n + 1)):
        if name in modes and "value" in modes[name]:
            m = modes[name]
            tf = m["value"] / world * cand * 5 / 1e12
            m.update({"bound": "valu-issue (instructions per instance-step; not HBM)",
                      "distance_TFLOPs_per_gpu": tf})
            sq = pmc_sq_issue(name, name.split("_")[0] + "_nearest_lds_kernel")
            if sq is not None:  # issuing fraction of wave cycles, from the committed SQ pass
                m["sq_issue_frac"], m["sq_issue_source"] = sq


SLAP_CHUNK = 10


def slap_chunk_bytes(kc, L=100, P=20):
    """Algorithmic HBM bytes per env-step of the chunked closest-free SLAP episode: every
    step writes the mask row L, i 8, done + reward 2, its action 8 and assignment entry 4
    and reads its product 4; each launch reads the row's depot distances 4L, mask L and i
    8 once; the first step's out-of-place assignment row (read + write 8P) and the
    episode's reset + pick-tour reward (1684 B) amortised over the P steps."""
    return L + 26 + (5 * L + 8) / kc + (8 * P + 1684) / P


def bench_slap(b, k, world, rank, dev, stepwise=True):
    import numpy as np

    from rl4co_slap_amd.envs.slap import SLAPGenerator
    from rl4co_slap_amd.rollout.engine import SLAPStepwiseEpisode

    torch.manual_seed(1234 + rank)
    np.random.seed(1234 + rank)
    from rl4co_slap_amd.rollout.engine import SLAPFusedEpisode

    gen = SLAPGenerator(materialize_dist_mat=False)
    n_rot = rotation(b * 2000)  # locs 8L + picklist 8OK + depot distances 4L per instance
    tds = [gen(b).to(dev) for _ in range(n_rot)]
    td = tds[0]
    out = {}
    fus = [SLAPFusedEpisode(t, policy="closest") for t in tds]
    sh = torch.cuda.current_stream(dev).cuda_stream
    cyc = itertools.cycle([f._bound for f in fus])
    run = lambda: next(cyc)(sh)  # noqa: E731
    wall, ev = timed(run, 4 * k, 2, world, dev)
    assert all(int(f.status.item()) == 0 for f in fus)
    t = max_over_ranks(wall, world, dev)
    out["slap_fused_closest"] = {"value": world * b * 20 * 4 * k / t,
                                 "ms_per_episode": t / (4 * k) * 1e3, "batch_per_gpu": b,
                                 "launch_us": ev / (4 * k) * 1e6,
                                 "bytes_per_episode": 2754, "input_batches_cycled": n_rot,
                                 "achieved_GBps": b * 2754 / (ev / (4 * k)) / 1e9}
    del fus
    # random-feasible policy, teacher-forced like the TSP headline:
    # P distinct non-depot locations per instance from a seeded permutation
    torch.manual_seed(4321 + rank)
    frs = [SLAPFusedEpisode(t, actions=(torch.rand(b, 99).argsort(1)[:, :20] + 1).to(dev),
                            policy="teacher") for t in tds]
    cyc = itertools.cycle([f._bound for f in frs])
    run = lambda: next(cyc)(sh)  # noqa: E731
    wall, ev = timed(run, 4 * k, 2, world, dev)
    assert all(int(f.status.item()) == 0 for f in frs)
    t = max_over_ranks(wall, world, dev)
    out["slap_fused_random"] = {"value": world * b * 20 * 4 * k / t,
                                "ms_per_episode": t / (4 * k) * 1e3, "batch_per_gpu": b,
                                "launch_us": ev / (4 * k) * 1e6, "bytes_per_episode": 2354,
                                "input_batches_cycled": n_rot,
                                "achieved_GBps": b * 2354 / (ev / (4 * k)) / 1e9}
    del frs
    if not stepwise:
        return out
    # closest-free policy fused with each step (co_slap_closest_step: one launch per step)
    ep = SLAPStepwiseEpisode(td, policy="closest").capture()
    wall, ev = timed(ep.replay, k, 2, world, dev)
    assert int(ep.status.item()) == 0, "SLAP stepwise episode status"
    t = max_over_ranks(wall, world, dev)
    out["slap_stepwise_graph"] = {"value": world * b * 20 * k / t, "ms_per_episode": t / k * 1e3,
                                  "batch_per_gpu": b, "bytes_per_env_step": 234,
                                  "launches_per_step": 1, "policy": "closest-free (fused)"}
    del ep
    # the same policy and per-step state writes, SLAP_CHUNK steps per co_slap_closest_steps
    # launch (the row's distances and mask in registers across the chunk)
    ep = SLAPStepwiseEpisode(td, policy="closest", chunk=SLAP_CHUNK).capture()
    wall, ev = timed(ep.replay, k, 2, world, dev)
    assert int(ep.status.item()) == 0, "SLAP chunked stepwise episode status"
    t = max_over_ranks(wall, world, dev)
    out["slap_stepwise_chunked"] = {
        "value": world * b * 20 * k / t, "ms_per_episode": t / k * 1e3, "batch_per_gpu": b,
        "steps_per_launch": SLAP_CHUNK, "policy": "closest-free (fused)",
        "alg_bytes_per_env_step": slap_chunk_bytes(SLAP_CHUNK),
        "frac_wall": b * 20 * slap_chunk_bytes(SLAP_CHUNK) * k / wall / 1e9 / HBM_PEAK_GBS,
        "frac": b * 20 * slap_chunk_bytes(SLAP_CHUNK) * k / ev / 1e9 / HBM_PEAK_GBS}
    del ep
    # the env step alone (co_slap_step), teacher-forced random-feasible actions
    torch.manual_seed(4321 + rank)
    acts = (torch.rand(b, 99).argsort(1)[:, :20] + 1).to(dev)
    ep = SLAPStepwiseEpisode(td, actions=acts, policy="teacher").capture()
    wall, ev = timed(ep.replay, k, 2, world, dev)
    assert int(ep.status.item()) == 0, "SLAP stepwise teacher episode status"
    t = max_over_ranks(wall, world, dev)
    out["slap_stepwise_graph_teacher"] = {"value": world * b * 20 * k / t,
                                          "ms_per_episode": t / k * 1e3, "batch_per_gpu": b,
                                          "bytes_per_env_step": 234, "launches_per_step": 1}
    return out


def bench_dropin(b, n, k, world, rank, dev):
    """The path an unchanged rl4co policy takes:
    ``ConstructivePolicy(None, decoder).forward(td, TSPEnv, greedy)`` at TSP-100
    B=65,536 -- per step the decode and the env step as one co_tsp_decode_step launch
    (TSPEnv.decode_and_step through the native step glue), the TensorDict plumbing in
    Python, the done poll only from step N on (env lower bound), then get_reward +
    validity and get_log_likelihood.  Decoders: a stub (logits from a fixed HBM-resident
    [B, N] tensor) and the AM-shaped pointer decoder of tests/am_pointer.py (glimpse +
    pointer over cached projections, random init).  Reported beside them: the host cost
    of the loop at B = 64, where the device work is negligible -- per step of a whole
    episode (reset, reward, log-likelihood amortised: host_us_per_step_b64) and the
    marginal cost of one more step (episodes of N and 2N steps:
    host_us_per_loop_step_b64) -- and the GPU time of the decode-fused kernel alone at B
    (HIP events)."""
    from rl4co_slap_amd import _native
    from rl4co_slap_amd.envs import TSPEnv
    from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder
    from rl4co_slap_amd.td import TensorDict

    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests"))
    from am_pointer import PointerDecoder

    out = {}
    for dec_name in ("stub", "am"):
        for bb, kk in ((b, k), (64, 3 * k)):
            locs, _ = tsp_inputs(bb, n, rank)
            locs = locs.to(dev)
            g = torch.Generator().manual_seed(7 + rank)
            logits = torch.randn(bb, n, generator=g).to(dev)
            env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
            dec = (LogitsDecoder(lambda td, lg=logits: lg) if dec_name == "stub"
                   else PointerDecoder(locs, dev, cache=True))
            pol = ConstructivePolicy(None, dec, env_name="tsp",
                                     tanh_clipping=0.0 if dec_name == "stub" else 10.0)

            def run():
                td = env.reset(TensorDict({"locs": locs}, [bb]))
                return pol(td, env, phase="test", decode_type="greedy")

            wall, ev = timed(run, kk, 2, world, dev)
            t = max_over_ranks(wall, world, dev)
            key = "" if dec_name == "stub" else "am_"
            if bb == b:
                m = {"value": world * bb * n * kk / t, "ms_per_episode": t / kk * 1e3,
                     "gpu_ms_per_episode": ev / kk * 1e3}
                if dec_name == "stub":
                    out.update(m)
                    out.update({"batch_per_gpu": bb, "launches_per_step": 1,
                                "done_polls_per_episode": 1,
                                "path": "ConstructivePolicy.forward + TSPEnv"})
                else:
                    out["am_decoder"] = m
            else:
                out[key + "host_us_per_step_b64"] = t / kk / n * 1e6
            del env, pol, dec
    # the marginal host cost of one loop step: episodes of N and 2N steps at B = 64 (the
    # per-episode reset / reward / log-likelihood / done poll cancel out)
    te = {}
    for nn in (n, 2 * n):
        locs, _ = tsp_inputs(64, nn, rank)
        locs = locs.to(dev)
        logits = torch.randn(64, nn, generator=torch.Generator().manual_seed(7)).to(dev)
        env = TSPEnv(generator_params=dict(num_loc=nn), device=dev)
        pol = ConstructivePolicy(None, LogitsDecoder(lambda td, lg=logits: lg), env_name="tsp")
        run = lambda: pol(env.reset(TensorDict({"locs": locs}, [64])), env,  # noqa: E731
                          phase="test", decode_type="greedy")
        wall, _ = timed(run, 3 * k, 2, world, dev)
        te[nn] = max_over_ranks(wall, world, dev) / (3 * k)
    out["host_us_per_loop_step_b64"] = (te[2 * n] - te[n]) / n * 1e6
    out["decode_fused_kernel_us"] = tsp_decode_step_kernel_us(b, n, dev)
    out["host_below_kernel"] = out["host_us_per_loop_step_b64"] < out["decode_fused_kernel_us"]
    out["native_step_glue"] = _native.torchstep() is not None
    return out


def tsp_decode_step_kernel_us(b, n, dev, reps=50):
    """GPU time of one co_tsp_decode_step launch (certified greedy, the drop-in default)
    at B x N: a mid-episode state (half the nodes visited), HIP events over reps
    launches on the launching stream."""
    from rl4co_slap_amd import _native

    g = torch.Generator().manual_seed(3)
    logits = torch.randn(b, n, generator=g).to(dev)
    mask = (torch.rand(b, n, generator=g) < 0.5).to(dev)
    mask[:, 0] = True
    i = torch.full((b, 1), n // 2, dtype=torch.int64, device=dev)
    first = torch.zeros(b, dtype=torch.int64, device=dev)
    outs = [torch.empty(b, dtype=torch.int64, device=dev), torch.empty(b, device=dev),
            torch.empty((b, n), dtype=torch.bool, device=dev),
            torch.empty((b, 1), dtype=torch.int64, device=dev),
            torch.empty(b, dtype=torch.int64, device=dev),
            torch.empty(b, dtype=torch.bool, device=dev), torch.empty(b, dtype=torch.bool,
                                                                        device=dev)]
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    launch = _native.bind("co_tsp_decode_step", b, n, logits.data_ptr(), n, mask.data_ptr(),
                          0.0, 1.0, _native.DECODE_CERTIFIED, None, outs[0].data_ptr(),
                          outs[1].data_ptr(), 0, 0, outs[2].data_ptr(), i.data_ptr(),
                          outs[3].data_ptr(), first.data_ptr(), outs[4].data_ptr(), 0,
                          outs[5].data_ptr(), outs[6].data_ptr(), None, st.data_ptr())
    _, ev = timed(lambda: launch(sh), reps, 5, 1, dev)
    return ev / reps * 1e6


def bench_dropin_cvrp(b, n, k, world, rank, dev):
    """The drop-in path on CVRP-100 (SURVEY.md 8d config 3 data): ConstructivePolicy +
    CVRPEnv, greedy on a stub decoder (a fixed HBM-resident [B, N+1] logits tensor whose
    masked argmax is the decoded action), per step one co_cvrp_decode_step launch (decode +
    env step) through the native step glue; the episode length is data dependent (polls
    resume once the env's lower bound N+1 is reached).  Plus the host cost per step at
    B = 64, the per-step GPU time (HIP events over the episode) and the fused kernel alone
    (decode_fused_kernel_us, a mid-episode state)."""
    from rl4co_slap_amd.envs import CVRPEnv
    from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder
    from rl4co_slap_amd.td import TensorDict

    out = {}
    for bb, kk in ((b, k), (64, 3 * k)):
        torch.manual_seed(1234 + rank)
        la = torch.rand(bb, n + 1, 2)
        dm = ((torch.rand(bb, n) * 9).int() + 1).float() / 50.0
        data = {"depot": la[:, 0].contiguous().to(dev), "locs": la[:, 1:].contiguous().to(dev),
                "demand": dm.to(dev)}
        g = torch.Generator().manual_seed(17 + rank)
        logits = torch.randn(bb, n + 1, generator=g).to(dev)
        env = CVRPEnv(generator_params=dict(num_loc=n), device=dev)
        pol = ConstructivePolicy(None, LogitsDecoder(lambda td: logits), env_name="cvrp")
        steps, calls = [], []

        def run():
            td = env.reset(TensorDict(dict(data), [bb]))
            r = pol(td, env, phase="test", decode_type="greedy", return_actions=True)
            steps.append(r["actions"].shape[1])
            return r

        count_fused_calls(env, calls)  # one untimed episode counts the fused launches
        run()
        uncount_fused_calls(env)
        steps.clear()
        wall, ev = timed(run, kk, 2, world, dev)
        t = max_over_ranks(wall, world, dev)
        T = steps[-1]
        if bb == b:
            out.update({"value": world * bb * T * kk / t, "ms_per_episode": t / kk * 1e3,
                        "gpu_ms_per_episode": ev / kk * 1e3, "episode_steps": T,
                        "gpu_us_per_step": ev / kk / T * 1e6, "batch_per_gpu": bb,
                        "launches_per_step": 1 if len(calls) == T else 2,
                        "path": "ConstructivePolicy.forward + CVRPEnv "
                                "(co_cvrp_decode_step per step)"})
        else:
            out["host_us_per_step_b64"] = t / kk / T * 1e6
    out["host_below_kernels"] = out["host_us_per_step_b64"] < out["gpu_us_per_step"]
    out["decode_fused_kernel_us"] = cvrp_decode_step_kernel_us(b, n, dev)
    return out


def cvrp_decode_step_kernel_us(b, n, dev, reps=50):
    """GPU time of one co_cvrp_decode_step launch (certified greedy, clip 10) on a CVRP-n
    state five steps into an episode (config 3 data), HIP events on the launch stream."""
    from rl4co_slap_amd import _native
    from rl4co_slap_amd.envs import CVRPEnv
    from rl4co_slap_amd.td import TensorDict

    torch.manual_seed(1)
    la = torch.rand(b, n + 1, 2)
    dm = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
    env = CVRPEnv(generator_params=dict(num_loc=n), device=dev)
    td = env.reset(TensorDict({"depot": la[:, 0].to(dev), "locs": la[:, 1:].contiguous().to(dev),
                               "demand": dm.to(dev)}, batch_size=[b]))
    for t in range(5):
        td.set("action", torch.full((b,), 1 + t, dtype=torch.int64, device=dev))
        td = env.step(td)["next"]
    logits = torch.randn(b, n + 1, device=dev)
    act = torch.empty(b, dtype=torch.int64, device=dev)
    lp = torch.empty(b, device=dev)
    used = torch.empty_like(td["used_capacity"])
    vis = torch.empty_like(td["visited"])
    cur = torch.empty((b, 1), dtype=torch.int64, device=dev)
    done, rew = (torch.empty(b, dtype=torch.bool, device=dev) for _ in range(2))
    mask = torch.empty_like(td["action_mask"])
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    p = _native.ptr
    launch = _native.bind("co_cvrp_decode_step", b, n, p(logits), n + 1, p(td["action_mask"]),
                          10.0, 1.0, _native.DECODE_CERTIFIED, None, p(act), p(lp), 0, 0,
                          p(td["demand"]), p(td["used_capacity"]), p(used),
                          p(td["vehicle_capacity"]), p(td["visited"]), p(vis), p(cur), p(done),
                          p(rew), p(mask), None, p(st))
    sh = torch.cuda.current_stream(dev).cuda_stream
    _, ev = timed(lambda: launch(sh), reps, 5, 1, dev)
    return ev / reps * 1e6


def count_fused_calls(env, calls):
    """Count the env's fused decode + step calls (the native step glue or the Python
    decode_and_step) by wrapping them on the instance; `uncount_fused_calls(env)` removes
    the wrappers.  Counting runs one untimed episode: the wrappers add a Python call per
    step, which the timed episodes must not pay."""
    real = (env.decode_and_step, env.native_decode_and_step)
    env.decode_and_step = lambda *a, **kw: calls.append(1) or real[0](*a, **kw)
    native = real[1]()
    if native is not None:
        counted = lambda *a, **kw: calls.append(1) or native(*a, **kw)  # noqa: E731
        env.native_decode_and_step = lambda: counted
    return real


def uncount_fused_calls(env):
    for name in ("decode_and_step", "native_decode_and_step"):
        env.__dict__.pop(name, None)


def bench_dropin_slap(b, k, world, rank, dev):
    """The fork's own user path (examples/slap.py:74-93 -> constructive/base.py:229-251):
    ``ConstructivePolicy.forward(td, SLAPEnv, greedy)`` on the config-4 instance recipe
    (``examples/slap.py:75-76``: 10 aisles x 10 locations, 20 products / orders, 5 picks per
    order; ``torch.manual_seed(1234 + rank)``, ``np.random.seed(1234 + rank)``), per step
    the decode and the SLAP env step as ONE co_slap_decode_step launch (SLAPEnv.
    decode_and_step), certified greedy with tanh clipping 10, P = 20 steps, then the pick-
    tour reward and get_log_likelihood.  Decoders: a stub (a fixed HBM-resident [B, L]
    logits tensor) and the SLAP pointer decoder of tests/am_pointer.py (examples/slap.py's
    init embedding + zero context, glimpse + pointer over cached projections).  Beside
    them: the host cost per loop step at B = 64 and the GPU time of the fused kernel at B."""
    import numpy as np

    from rl4co_slap_amd import _native
    from rl4co_slap_amd.envs import SLAPEnv
    from rl4co_slap_amd.envs.slap import SLAPGenerator
    from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder
    from rl4co_slap_amd.td import TensorDict

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from am_pointer import SLAPPointerDecoder

    out = {}
    P = 20
    for dec_name in ("stub", "am"):
        for bb, kk in ((b, k), (64, 3 * k)):
            torch.manual_seed(1234 + rank)
            np.random.seed(1234 + rank)
            data = SLAPGenerator(materialize_dist_mat=False)(bb).to(dev)
            l = data["locs"].shape[1]
            g = torch.Generator().manual_seed(11 + rank)
            logits = torch.randn(bb, l, generator=g).to(dev)
            env = SLAPEnv(device=dev)
            dec = (LogitsDecoder(lambda td, lg=logits: lg) if dec_name == "stub"
                   else SLAPPointerDecoder(data["locs"], dev))
            pol = ConstructivePolicy(None, dec, env_name="slap", tanh_clipping=10.0)
            calls = []

            def run():
                td = env.reset(TensorDict(dict(data.items()), [bb]))
                return pol(td, env, phase="test", decode_type="greedy")

            count_fused_calls(env, calls)  # one untimed episode counts the fused launches
            run()
            uncount_fused_calls(env)
            fused_steps = len(calls)
            wall, ev = timed(run, kk, 2, world, dev)
            t = max_over_ranks(wall, world, dev)
            key = "" if dec_name == "stub" else "am_"
            if bb == b:
                m = {"value": world * bb * P * kk / t, "ms_per_episode": t / kk * 1e3,
                     "gpu_ms_per_episode": ev / kk * 1e3,
                     "launches_per_step": 1 if fused_steps == P else 2}
                if dec_name == "stub":
                    out.update(m)
                    out.update({"batch_per_gpu": bb, "env_steps_per_episode": P,
                                "done_polls_per_episode": 1,
                                "path": "ConstructivePolicy.forward + SLAPEnv "
                                        "(co_slap_decode_step per step)"})
                else:
                    out["am_decoder"] = m
            else:
                out[key + "host_us_per_step_b64"] = t / kk / P * 1e6
            del env, pol, dec, data
    # the marginal host cost of one loop step: episodes of P = 20 and 40 products at B = 64
    # (the per-episode reset / reward / log-likelihood / status read cancel out)
    te = {}
    for pp in (P, 2 * P):
        torch.manual_seed(1234 + rank)
        np.random.seed(1234 + rank)
        data = SLAPGenerator(n_products=pp, materialize_dist_mat=False)(64).to(dev)
        logits = torch.randn(64, data["locs"].shape[1],
                             generator=torch.Generator().manual_seed(11)).to(dev)
        env = SLAPEnv(device=dev)
        pol = ConstructivePolicy(None, LogitsDecoder(lambda td, lg=logits: lg), env_name="slap",
                                 tanh_clipping=10.0)
        run = lambda: pol(env.reset(TensorDict(dict(data.items()), [64])), env,  # noqa: E731
                          phase="test", decode_type="greedy")
        wall, _ = timed(run, 3 * k, 2, world, dev)
        te[pp] = max_over_ranks(wall, world, dev) / (3 * k)
    out["host_us_per_loop_step_b64"] = (te[2 * P] - te[P]) / P * 1e6
    out["decode_fused_kernel_us"] = slap_decode_step_kernel_us(b, dev)
    out["host_below_kernel"] = out["host_us_per_loop_step_b64"] < out["decode_fused_kernel_us"]
    # the SLAP step 2L+34 B + the decode's logits 4L + logp 4 per env-step
    out["bytes_per_env_step"] = 2 * 100 + 34 + 4 * 100 + 4
    return out


def slap_decode_step_kernel_us(b, dev, reps=50, l=100, p=20):
    """GPU time of one co_slap_decode_step launch (certified greedy, clip 10, the drop-in
    default) at B x L: a mid-episode state (10 products placed) with the operands the step
    glue passes (the assignment written in place, to_choose's uniform product: no per-row
    column read), HIP events over reps launches on the launching stream."""
    from rl4co_slap_amd import _native

    g = torch.Generator().manual_seed(5)
    logits = torch.randn(b, l, generator=g).to(dev)
    mask = (torch.rand(b, l, generator=g) < 0.9).to(dev)
    mask[:, 0] = False
    mask[:, 1] = True
    asg = torch.randint(0, l, (b, p), dtype=torch.int32).to(dev)
    i = torch.full((b, 1), p // 2, dtype=torch.int64, device=dev)
    act = torch.empty(b, dtype=torch.int64, device=dev)
    lp = torch.empty(b, dtype=torch.float32, device=dev)
    m_o = torch.empty_like(mask)
    i_o = torch.empty_like(i)
    done, rw = (torch.empty((b, 1), dtype=torch.bool, device=dev) for _ in range(2))
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    launch = _native.bind("co_slap_decode_step", b, l, p, logits.data_ptr(), l, mask.data_ptr(),
                          10.0, 1.0, _native.DECODE_CERTIFIED, None, act.data_ptr(),
                          lp.data_ptr(), 0, 0, None, p // 2, asg.data_ptr(),
                          asg.data_ptr(), m_o.data_ptr(), i.data_ptr(), i_o.data_ptr(),
                          done.data_ptr(), rw.data_ptr(), None, st.data_ptr())
    _, ev = timed(lambda: launch(sh), reps, 5, 1, dev)
    return ev / reps * 1e6


def bench_cvrp(b, n, k, world, rank, dev):
    """torch.manual_seed(1234 + rank); locs_all = rand(B, N+1, 2),
    depot = locs_all[:, 0]; demand = ((rand(B, N) * 9).int() + 1) / 50 (CAPACITIES[100]).
    env-steps = B x T, T = the batch-wide episode length the reference loop runs."""
    from rl4co_slap_amd.rollout.engine import CVRPFusedEpisode, CVRPStepwiseEpisode

    torch.manual_seed(1234 + rank)
    locs_all = torch.rand(b, n + 1, 2)
    demand = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
    td = {"depot": locs_all[:, 0].contiguous().to(dev), "locs": locs_all[:, 1:].contiguous().to(dev),
          "demand": demand.to(dev)}
    out = {}
    # batches cycled past the Infinity Cache, each launched equally often (T differs per batch)
    n_rot = rotation(b * (12 * n + 8))
    tds = [td]
    for _ in range(1, n_rot):
        la = torch.rand(b, n + 1, 2)
        dm = ((torch.rand(b, n) * 9).int() + 1).float() / 50.0
        tds.append({"depot": la[:, 0].contiguous().to(dev), "locs": la[:, 1:].contiguous().to(dev),
                    "demand": dm.to(dev)})
    fus = [CVRPFusedEpisode(x) for x in tds]
    sh = torch.cuda.current_stream(dev).cuda_stream
    cyc = itertools.cycle([f._bound for f in fus])
    run = lambda: next(cyc)(sh)  # noqa: E731
    kk = n_rot * max(1, (4 * k) // n_rot)
    wall, ev = timed(run, kk, n_rot, world, dev)
    assert all(int(f.status.item()) == 0 for f in fus), "CVRP fused episode status"
    Ts = [f.final_state()["steps"] for f in fus]
    T = Ts[0]
    t = max_over_ranks(wall, world, dev)
    # env-steps = B x T per launch, T the batch-wide length of that batch's episode
    steps_all = sum_over_ranks(b * sum(Ts) * (kk // n_rot), world, dev)
    out["cvrp_fused_nearest"] = {"value": steps_all / t,
                                 "ms_per_episode": t / kk * 1e3, "batch_per_gpu": b,
                                 "num_loc": n, "episode_steps": T,
                                 "episode_steps_mean": sum(Ts) / n_rot,
                                 "input_batches_cycled": n_rot,
                                 "launch_us": ev / kk * 1e6}
    del fus
    steps_one = sum_over_ranks(b * T, world, dev)
    # nearest policy fused with each step (co_cvrp_nearest_step, one launch per step), then
    # the co_cvrp_nearest_action + co_cvrp_step pair (the env step as any policy drives it)
    for name, fused, byts in (("cvrp_stepwise_graph", True, 16 * n + 50),
                              ("cvrp_stepwise_graph_pair", False, 7 * n + 33)):
        sw = CVRPStepwiseEpisode(td, fused_policy=fused).capture()
        wall, ev = timed(sw.replay, k, 1, world, dev)
        t = max_over_ranks(wall, world, dev)
        assert sw.T == T and int(sw.status.item()) == 0, "CVRP stepwise episode status"
        out[name] = {"value": steps_one * k / t, "ms_per_episode": t / k * 1e3,
                     "batch_per_gpu": b, "episode_steps": T, "bytes_per_env_step": byts,
                     "launches_per_step": 1 if fused else 2}
        del sw
    return out


def bench_generate_slap(b, dev, reps=3, with_ref=True):
    """SLAP instance generation incl. the [B, 100, 100] dist_mat: co_slap_generate on the
    device (freq/picklists from the host RNG streams; device_rng: from co_uniform_fill /
    co_randint_fill too) vs the host generator (vectorised) + copy; the oracle's restatement of the
    reference's B x L Python loop is timed on a small sample and scaled per instance."""
    from rl4co_slap_amd.envs.slap import SLAPGenerator

    gd, gh = SLAPGenerator(device=dev), SLAPGenerator()
    gd(b)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        gd(b)
    torch.cuda.synchronize(dev)
    t_dev = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    gh(b).to(dev)
    torch.cuda.synchronize(dev)
    t_host = time.perf_counter() - t0
    gr = SLAPGenerator(device=dev, device_rng=True)
    gr(b)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(reps):
        gr(b)
    torch.cuda.synchronize(dev)
    t_rng = (time.perf_counter() - t0) / reps
    out = {"device_ms": t_dev * 1e3, "device_rng_ms": t_rng * 1e3,
           "host_vectorised_plus_copy_ms": t_host * 1e3, "dist_mat_MB": b * 100 * 100 * 4 / 1e6}
    if with_ref:
        from oracle.envs import SLAPOracle

        nb = 64
        t0 = time.perf_counter()
        SLAPOracle(seed=1).generate([nb])
        out["reference_loop_ms_scaled"] = (time.perf_counter() - t0) / nb * b * 1e3
    return out


def bench_generate_uniform(b, n, dev, reps=5):
    """TSP-100 / CVRP-100 instance generation (co_uniform_fill, Philox on the device) vs the
    reference's host sampling (torch CPU RNG) + copy.  Device kernel timed with HIP events
    (write-only: 4 B per element)."""
    from rl4co_slap_amd import _native as nat
    from rl4co_slap_amd.envs.cvrp import CVRPGenerator
    from rl4co_slap_amd.envs.tsp import TSPGenerator

    out = {}
    for name, gd, gh in (("tsp", TSPGenerator(num_loc=n, device=dev), TSPGenerator(num_loc=n)),
                         ("cvrp", CVRPGenerator(num_loc=n, device=dev), CVRPGenerator(num_loc=n))):
        gd([b])
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            gd([b])
        e1.record()
        torch.cuda.synchronize(dev)
        t_dev = e0.elapsed_time(e1) / 1e3 / reps
        t0 = time.perf_counter()
        gh([b]).to(dev)
        torch.cuda.synchronize(dev)
        t_host = time.perf_counter() - t0
        out[name] = {"batch": b, "num_loc": n, "device_ms": t_dev * 1e3,
                     "host_sample_plus_copy_ms": t_host * 1e3}
    # the kernel alone: TSP locs fill, launches back to back on one stream
    buf = torch.empty(b * n * 2, dtype=torch.float32, device=dev)
    f = nat.bind("co_uniform_fill", nat.ptr(buf), buf.numel(), 0.0, 1.0, 1.0, 0, 1234, 0)
    s = torch.cuda.current_stream(dev).cuda_stream
    f(s)
    e0.record()
    for _ in range(20):
        f(s)
    e1.record()
    torch.cuda.synchronize(dev)
    t = e0.elapsed_time(e1) / 1e3 / 20
    # write-only ceiling beside it: torch's fill of the same buffer
    e0.record()
    for _ in range(20):
        buf.fill_(0.5)
    e1.record()
    torch.cuda.synchronize(dev)
    t_fill = e0.elapsed_time(e1) / 1e3 / 20
    out["tsp"].update(kernel_us=t * 1e6, kernel_GBps_written=buf.numel() * 4 / t / 1e9,
                      same_bytes_fill_us=t_fill * 1e6)
    return out


def bench_pomo(b, n, k, world, rank, dev, decode_math=None):
    from rl4co_slap_amd.rollout.pomo import POMOEpisode, global_metrics
    from rl4co_slap_amd.utils.decoding import default_decode_math

    torch.manual_seed(1234 + rank)
    locs = torch.rand(b, n, 2).to(dev)
    e = b * n
    g = torch.Generator(device=dev).manual_seed(99 + rank)
    logits = torch.randn((n - 1, e, n), generator=g, device=dev)  # policy-network stand-in
    ep = POMOEpisode(locs, logits, tanh_clipping=10.0, decode_math=decode_math).capture()
    decode_math = ep.decode_math

    def run():
        ep.replay()

    wall, ev = timed(run, k, 1, world, dev)
    assert int(ep.status.item()) == 0
    t = max_over_ranks(wall, world, dev)
    total = world * b  # every rank holds b instances: shard sizes known, one all-gather
    m = global_metrics(ep.bl, ep.max_reward, ep.loss_terms, n,
                       total_instances=total)  # warm-up (communicator setup)
    ag = []
    for _ in range(10):  # the RCCL exchange itself (no collective at world size 1)
        torch.cuda.synchronize(dev)
        barrier(world)
        t0 = time.perf_counter()
        m = global_metrics(ep.bl, ep.max_reward, ep.loss_terms, n, total_instances=total)
        torch.cuda.synchronize(dev)
        ag.append(time.perf_counter() - t0)
    t_ag = sorted(ag)[len(ag) // 2]
    return {"value": world * e * n * k / t, "ms_per_episode": t / k * 1e3,
            "instances_per_gpu": b, "starts": n, "envs_per_gpu": e,
            "bytes_per_env_step_decode_fused": 6 * n + 54,
            "decode_math": {
                "fast": "fast (CO_DECODE_FAST, opt-in, not bit-exact)",
                "certified": "certified (the default; CO_DECODE_CERTIFIED: greedy actions = the "
                             "exact path's by a per-row error bound + exact recomputation of "
                             "uncertified waves; logp from the fast math, within 1e-5)",
                "exact": "exact (opt-in; ATen log_softmax bits, correctly rounded tanh)",
            }[decode_math],
            "allgather_ms": t_ag * 1e3,
            "allgather_note": "median of 10 after a warm-up call" + (
                "" if world > 1 else "; world size 1: no collective runs, host bookkeeping only"),
            "global_instances": m["instances"],
            "loss": float(m["loss"]), "max_reward_mean": float(m["max_reward_mean"])}


if __name__ == "__main__":
    main()
