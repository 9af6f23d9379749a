"""SIMD cycles per wave-instruction of the VALU forms the nearest scan uses (diagnostic, not
part of the product), at 1, 2 and 4 waves per SIMD: independent chains (throughput) and
one chain (dependent latency).  Needs tools/diag/libvalu_rates.so
(hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/diag/valu_rates.hip -o ...).
Usage: python tools/valu_rates.py -> one JSON line."""
import ctypes
import json
import os

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
lib = ctypes.CDLL(os.path.join(ROOT, "tools", "diag", "libvalu_rates.so"))
lib.valu_probe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                           ctypes.c_void_p, ctypes.c_void_p]
names = ["sub", "mul", "fma", "pk_add", "pk_mul", "pk_fma", "min_u32", "med3_u32", "and_or",
         "cndmask", "min_dpp", "min_dep", "med3_dep", "pk_add_dep", "sub_dep", "min_dpp_dep"]
dev = torch.device("cuda:0")
sink = torch.zeros(1024, device=dev)
s = torch.cuda.current_stream(dev)
CUS, CLK = 256, 2.4e9
ITERS = 4096
out = {}
for w in (1, 2, 4):
    for i, n in enumerate(names):
        blocks = CUS * w  # 256 threads = 4 waves = one per SIMD, w blocks per CU
        lib.valu_probe(i, blocks, 256, 16, sink.data_ptr(), s.cuda_stream)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        lib.valu_probe(i, blocks, 256, ITERS, sink.data_ptr(), s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) * 1e-3
        # per SIMD: w waves x ITERS x 8 instructions
        out[f"{n}_w{w}"] = round(t * CLK / (w * ITERS * 8), 2)
print(json.dumps(out), flush=True)
