"""Diagnostic timing of the decode kernels (not part of the product)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rl4co_slap_amd import _native as nat  # noqa: E402

if os.environ.get("DIAG_LIB"):
    nat.LIB_PATH = os.environ["DIAG_LIB"]
print("lib:", nat.LIB_PATH)
nat.load()
dev = torch.device("cuda:0")
BASE_MODE = int(os.environ.get("DIAG_DECODE_MODE", "0"))  # 0 greedy, 1 sampling, 2 evaluate
SIZES = [(102400, 100), (65536, 100), (102400, 20), (102400, 50), (16384, 200)]
if os.environ.get("DIAG_SIZES") == "tsp100":
    SIZES = [(102400, 100)]
for B, N in SIZES:
    logits = torch.randn(B, N, device=dev)
    mask = torch.rand(B, N, device=dev) > 0.3
    mask[:, 0] = True
    out_a = torch.empty(B, dtype=torch.int64, device=dev)
    lp = torch.empty(B, device=dev)
    m2 = torch.empty_like(mask)
    i0 = torch.zeros(B, 1, dtype=torch.int64, device=dev)
    i1 = torch.empty_like(i0)
    f0 = torch.zeros(B, dtype=torch.int64, device=dev)
    f1 = torch.empty_like(f0)
    done = torch.empty(B, dtype=torch.bool, device=dev)
    sr = torch.empty_like(done)
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    for clip, fast in [(c, f) for c in ((0.0, 10.0)) for f in (0, nat.DECODE_FAST)]:
        for name in ("decode", "tsp_decode"):
            def run():
                if name == "decode":
                    nat.call("co_decode_step", B, N, nat.ptr(logits), N, nat.ptr(mask), clip, 1.0, BASE_MODE | fast,
                             None, nat.ptr(out_a), nat.ptr(lp), None, 0, 0, nat.ptr(st), s)
                else:
                    nat.call("co_tsp_decode_step", B, N, nat.ptr(logits), N, nat.ptr(mask), clip, 1.0, BASE_MODE | fast,
                             None, nat.ptr(out_a), nat.ptr(lp), 0, 0, nat.ptr(m2), nat.ptr(i0),
                             nat.ptr(i1), nat.ptr(f0), nat.ptr(f1), 0, nat.ptr(done), nat.ptr(sr),
                             None, nat.ptr(st), s)
            # launches captured in a graph: the replay times the kernels, not ctypes
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                s = side.cuda_stream
                for _ in range(3):
                    run()
            torch.cuda.current_stream().wait_stream(side)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                s = torch.cuda.current_stream().cuda_stream
                for _ in range(50):
                    run()
            g.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / 50
            byts = B * (5 * N + 16) if name == "decode" else B * (6 * N + 54)
            print(f"mode={BASE_MODE} B={B} N={N} clip={clip} fast={bool(fast)} {name}: {us:.1f} us  "
                  f"{byts / us / 1e3:.0f} GB/s", flush=True)
