"""How much of a one-round step kernel is launch + ramp and how much is memory
(diagnostic, not part of the product).  Times, on the launch stream
with HIP events (median of 5 x 50 launches), and -- under ``rocprofv3 --kernel-trace
--stats`` -- per dispatch:
  * ceiling_empty_kernel: the step kernels' grid (2,048 x 256) with an empty body;
  * ceiling_touch_kernel: the same grid, one dword load + store per thread (4 MB);
  * co_tsp_step (TSP-100, B = 65,536) and co_cvrp_step (CVRP-100, B = 32,768);
  * co_probe_copy of each step kernel's bytes (the same-byte copy).
Usage: python tools/launch_ceiling.py -> one JSON line.  Needs tools/diag/liblaunch_ceiling.so
(hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/diag/launch_ceiling.hip -o ...)."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rl4co_slap_amd import _native as nat  # noqa: E402

dev = torch.device("cuda:0")
nat.load()
lc = ctypes.CDLL(os.path.join(ROOT, "tools", "diag", "liblaunch_ceiling.so"))
lc.ceiling_empty.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_void_p]
lc.ceiling_touch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                             ctypes.c_void_p, ctypes.c_void_p]
s = torch.cuda.current_stream(dev)
sh = s.cuda_stream


def ev_us(launch, reps=50, rounds=5):
    """median over rounds of (HIP-event time of `reps` back-to-back launches) / reps"""
    launch()
    torch.cuda.synchronize()
    out = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            launch()
        e1.record(s)
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1) * 1e3 / reps)
    return round(statistics.median(out), 3)


res = {}
sink = torch.zeros(256, dtype=torch.int32, device=dev)
src = torch.ones(2048 * 256, dtype=torch.int32, device=dev)
dst = torch.empty_like(src)
# the same 512K threads as 2,048 x 256 (the step kernels' grid) and in other workgroup sizes:
# how much of a one-round launch is the workgroup dispatch
for blocks, threads in ((2048, 256), (8192, 64), (4096, 128), (1024, 512), (512, 1024)):
    res[f"empty_{blocks}x{threads}"] = ev_us(
        lambda: lc.ceiling_empty(blocks, threads, 1, sink.data_ptr(), sh))
    res[f"touch_{blocks}x{threads}_4MB"] = ev_us(
        lambda: lc.ceiling_touch(blocks, threads, 1, src.data_ptr(), dst.data_ptr(), sh))
res["empty_256x256"] = ev_us(lambda: lc.ceiling_empty(256, 256, 1, sink.data_ptr(), sh))
res["empty_1x64"] = ev_us(lambda: lc.ceiling_empty(1, 64, 1, sink.data_ptr(), sh))
# the same launches issued from C in one call (no Python / ctypes per launch) and replayed
# from a HIP graph: what the GPU side costs per kernel boundary once the host is not the
# bottleneck
for blocks, threads in ((1, 64), (2048, 256)):
    res[f"empty_{blocks}x{threads}_c_loop"] = round(ev_us(
        lambda: lc.ceiling_empty(blocks, threads, 50, sink.data_ptr(), sh), reps=4) / 50, 3)
    gs = torch.cuda.Stream(dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(gs):
        lc.ceiling_empty(blocks, threads, 1, sink.data_ptr(), gs.cuda_stream)  # warm
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=gs):
            lc.ceiling_empty(blocks, threads, 50, sink.data_ptr(), gs.cuda_stream)
    res[f"empty_{blocks}x{threads}_graph"] = round(ev_us(lambda: g.replay(), reps=4) / 50, 3)


def copy_us(nbytes):
    n = (nbytes // 2) // 16 * 16
    a = torch.ones(n, dtype=torch.uint8, device=dev)
    c = torch.empty(n, dtype=torch.uint8, device=dev)
    f = nat.bind("co_probe_copy", a.data_ptr(), c.data_ptr(), n)
    return ev_us(lambda: f(sh))


b, n = 65536, 100
act = torch.randint(0, n, (b,), device=dev)
mask = torch.ones(b, n, dtype=torch.bool, device=dev)
i = torch.zeros(b, 1, dtype=torch.int64, device=dev)
first, cur = (torch.zeros(b, dtype=torch.int64, device=dev) for _ in range(2))
done, rw = (torch.empty(b, dtype=torch.bool, device=dev) for _ in range(2))
st = torch.zeros(1, dtype=torch.int32, device=dev)
f = nat.bind("co_tsp_step", b, n, act.data_ptr(), mask.data_ptr(), mask.data_ptr(), i.data_ptr(),
             i.data_ptr(), first.data_ptr(), first.data_ptr(), cur.data_ptr(), done.data_ptr(),
             rw.data_ptr(), 0, None, st.data_ptr())
res["tsp_step_b65536"] = ev_us(lambda: f(sh))
res["copy_tsp_bytes"] = copy_us(b * (2 * n + 50))
del act, mask, i, first, cur, done, rw
b = 32768
act = torch.randint(0, n + 1, (b,), device=dev)
dem = torch.rand(b, n, device=dev) * 0.1
used, used2 = torch.zeros(b, 1, device=dev), torch.zeros(b, 1, device=dev)
vcap = torch.ones(b, 1, device=dev)
vis = torch.zeros(b, n + 1, dtype=torch.uint8, device=dev)
cur = torch.empty(b, dtype=torch.int64, device=dev)
done, rw = (torch.empty(b, dtype=torch.bool, device=dev) for _ in range(2))
m = torch.empty(b, n + 1, dtype=torch.bool, device=dev)
f2 = nat.bind("co_cvrp_step", b, n, act.data_ptr(), dem.data_ptr(), used.data_ptr(),
              used2.data_ptr(), vcap.data_ptr(), vis.data_ptr(), vis.data_ptr(), cur.data_ptr(),
              done.data_ptr(), rw.data_ptr(), m.data_ptr(), st.data_ptr(), None)
res["cvrp_step_b32768"] = ev_us(lambda: f2(sh))
res["copy_cvrp_bytes"] = copy_us(b * (7 * n + 33))
print(json.dumps(res), flush=True)
