"""Host-side cost (us per call) of the pieces of the drop-in decode step at B = 64, where
the device work is negligible (diagnostic, not part of the product)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rl4co_slap_amd import _native as nat  # noqa: E402
from rl4co_slap_amd.envs import TSPEnv  # noqa: E402
from rl4co_slap_amd.rollout.constructive import ConstructivePolicy, LogitsDecoder  # noqa: E402
from rl4co_slap_amd.td import TensorDict  # noqa: E402

dev = torch.device("cuda:0")
b, n = 64, 100
nat.load()


def us(f, reps=3000):
    for _ in range(100):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    t = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    return round(t, 3)


out = {}
out["torch.empty"] = us(lambda: torch.empty((b, n), dtype=torch.bool, device=dev))
env = TSPEnv(generator_params=dict(num_loc=n), device=dev)
td = env.reset(TensorDict({"locs": torch.rand(b, n, 2, device=dev)}, [b]))
logits = torch.randn(b, n, device=dev)
st = torch.zeros(1, dtype=torch.int32, device=dev)
mask, i = td["action_mask"], td["i"]
first = torch.zeros(b, dtype=torch.int64, device=dev)
outs = [torch.empty(b, dtype=torch.int64, device=dev), torch.empty(b, device=dev),
        torch.empty((b, n), dtype=torch.bool, device=dev),
        torch.empty((b, 1), dtype=torch.int64, device=dev),
        torch.empty(b, dtype=torch.int64, device=dev),
        torch.empty(b, dtype=torch.bool, device=dev), torch.empty(b, dtype=torch.bool, device=dev)]
p = [t.data_ptr() for t in outs]
s = nat.stream_of(mask)
args = (b, n, logits.data_ptr(), n, mask.data_ptr(), 0.0, 1.0, nat.DECODE_CERTIFIED, None,
        p[0], p[1], 0, 0, p[2], i.data_ptr(), p[3], first.data_ptr(), p[4], 0, p[5], p[6], None,
        st.data_ptr(), s)
out["nat.call (fastcall, preallocated)"] = us(lambda: nat.call("co_tsp_decode_step", *args))
launch = nat.bind("co_tsp_decode_step", *args[:-1])
out["bind launch (ctypes, preconverted)"] = us(lambda: launch(s))
ts = nat.torchstep()
if ts is not None:
    out["glue tsp_decode_step"] = us(lambda: ts.tsp_decode_step(
        logits, mask, i, first, None, st, 0.0, 1.0, nat.DECODE_CERTIFIED, 0, 0, 0))
    out["glue decode_step"] = us(lambda: ts.decode_step(
        logits, mask, None, st, 0.0, 1.0, nat.DECODE_CERTIFIED, 0, 0, False))
lib = nat.load()
side = torch.cuda.Stream(dev)
args_side = args[:-1] + (side.cuda_stream,)
out["nat.call on a side stream"] = us(lambda: nat.call("co_tsp_decode_step", *args_side))
flag = torch.zeros(1, dtype=torch.int32, device=dev)
out["nat.call co_any_eq_i64 (5 args)"] = us(lambda: nat.call(
    "co_any_eq_i64", i.data_ptr(), b, 0, flag.data_ptr(), s))
small = torch.zeros(64, device=dev)
out["torch add_ (aten launch)"] = us(lambda: small.add_(1.0))
out["co_probe (no kernel: B=0 call)"] = us(lambda: nat.call(
    "co_tsp_decode_step", 0, n, *args[2:]))


def reset():
    return env.reset(TensorDict({"locs": td["locs"]}, [b]))


out["env.reset"] = us(reset, 1000)


def reset_step():
    t = reset()
    return env.decode_and_step(t, logits, nat.DECODE_CERTIFIED, 1.0, 0.0, None, 0, 0, st)


out["env.reset + decode_and_step"] = us(reset_step, 1000)
dec = LogitsDecoder(lambda t: logits)
out["decoder module call"] = us(lambda: dec(td, None, 0))
pol = ConstructivePolicy(None, dec, env_name="tsp")


def episode():
    t = reset()
    return pol(t, env, phase="test", decode_type="greedy")


out["episode (reset + N steps + reward), per step"] = round(us(episode, 100) / n, 3)
print(json.dumps(out))

if os.environ.get("CO_HOST_PROFILE"):
    import cProfile
    import pstats

    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        episode()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)

# launch cost by argument shape (tools/diag/launch_cost.hip)
_lc = os.path.join(ROOT, "tools", "diag", "liblaunch_cost.so")
if os.path.exists(_lc):
    import ctypes

    lc = ctypes.CDLL(_lc)
    res = {}
    for name in ("launch19", "launch_struct", "launch_module"):
        fn = getattr(lc, name)
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fn(s, 100)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = fn(s, 5000)
        res[name] = round((time.perf_counter() - t0) / 5000 * 1e6, 3)
        torch.cuda.synchronize()
        res[name + "_rc"] = rc
    for name in ("launch19_err", "get_error_only"):
        fn = getattr(lc, name)
        fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
        t0 = time.perf_counter()
        res[name + "_rc"] = fn(s, 5000)
        res[name] = round((time.perf_counter() - t0) / 5000 * 1e6, 3)
        torch.cuda.synchronize()
    fn = lc.call_tsp_decode_step
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_int64] + \
        [ctypes.c_void_p] * 13
    addr = ctypes.cast(nat.load().co_tsp_decode_step, ctypes.c_void_p).value
    cargs = [addr, 5000, b, n, logits.data_ptr(), mask.data_ptr(), p[0], p[1], p[2], i.data_ptr(),
             p[3], first.data_ptr(), p[4], p[5], p[6], st.data_ptr(), s]
    t0 = time.perf_counter()
    res["co_tsp_decode_step from C_rc"] = fn(*cargs)
    res["co_tsp_decode_step from C"] = round((time.perf_counter() - t0) / 5000 * 1e6, 3)
    torch.cuda.synchronize()
    res["launch19 side stream"] = None
    fn = lc.launch19
    t0 = time.perf_counter()
    fn(side.cuda_stream, 5000)
    res["launch19 side stream"] = round((time.perf_counter() - t0) / 5000 * 1e6, 3)
    torch.cuda.synchronize()
    print(json.dumps(res))
