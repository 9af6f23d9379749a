"""Host time per phase of the SLAP drop-in episode (diagnostic, not part of the product):
``env.reset`` + ``ConstructivePolicy.forward`` (greedy, stub decoder, clip 10) at a small
batch, where the device work is negligible, with every phase of the episode wrapped in a
host timer; plus the unit costs of the torch / HIP operations the phases are made of.
Usage: python tools/slap_dropin_phases.py [B] -> one JSON line (us per episode / per call)."""
import json
import os
import sys
import time
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from rl4co_slap_amd import _native as nat  # noqa: E402
from rl4co_slap_amd.envs import SLAPEnv  # noqa: E402
from rl4co_slap_amd.envs.slap import SLAPGenerator  # noqa: E402
from rl4co_slap_amd.rollout import constructive as C  # noqa: E402
from rl4co_slap_amd.td import TensorDict  # noqa: E402
from rl4co_slap_amd.utils import decoding as D  # noqa: E402

dev = torch.device(os.environ.get("CO_DEV", "cuda:0"))
b = int(sys.argv[1]) if len(sys.argv) > 1 else 64
nat.load()
torch.manual_seed(1234)
np.random.seed(1234)
data = SLAPGenerator(materialize_dist_mat=False)(b).to(dev)
logits = torch.randn(b, data["locs"].shape[1], device=dev)
env = SLAPEnv(device=dev)
pol = C.ConstructivePolicy(None, C.LogitsDecoder(lambda td: logits), env_name="slap",
                           tanh_clipping=10.0)
acc = defaultdict(float)
cnt = defaultdict(int)


def wrap(obj, name, label):
    f = getattr(obj, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        acc[label] += time.perf_counter() - t0
        cnt[label] += 1
        return r

    setattr(obj, name, w)


def episode():
    t0 = time.perf_counter()
    td = env.reset(TensorDict(dict(data.items()), [b]))
    acc["reset (all)"] += time.perf_counter() - t0
    t1 = time.perf_counter()
    r = pol(td, env, phase="test", decode_type="greedy")
    acc["forward (all)"] += time.perf_counter() - t1
    return r


def run(k):
    for _ in range(k):
        episode()
    torch.cuda.synchronize()


run(20)
t0 = time.perf_counter()
run(200)
plain = (time.perf_counter() - t0) / 200 * 1e6

wrap(env, "_reset", "reset: _reset")
wrap(D.DecodingStrategy, "pre_decoder_hook", "pre_decoder_hook")
wrap(D.DecodingStrategy, "post_decoder_hook", "post_decoder_hook (1 host read)")
wrap(D.DecodingStrategy, "step_env_fused", "step_env_fused (x20)")
wrap(env, "get_reward", "get_reward (1 host read)")
wrap(env, "min_steps_to_done", "min_steps_to_done")
wrap(env, "poll_done", "poll_done")
wrap(C, "get_log_likelihood", "get_log_likelihood")
wrap(C, "get_decoding_strategy", "get_decoding_strategy")
wrap(pol.decoder, "forward", "decoder.forward (x20)")
wrap(pol.encoder, "forward", "encoder")
acc.clear()
cnt.clear()
run(200)
res = {"batch": b, "episode_us_unwrapped": round(plain, 2)}
for k, v in sorted(acc.items(), key=lambda kv: -kv[1]):
    res[k] = round(v / 200 * 1e6, 2)
res["forward other (loop + dict)"] = round(
    res["forward (all)"] - sum(v for k, v in res.items() if k not in (
        "batch", "episode_us_unwrapped", "forward (all)", "reset (all)", "reset: _reset")), 2)


def us(f, reps=2000):
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        f()
    t = (time.perf_counter() - t0) / reps * 1e6
    torch.cuda.synchronize()
    return round(t, 3)


x = torch.zeros(b, device=dev)
xs = [torch.randn(b, device=dev) for _ in range(20)]
unit = {
    "torch.empty": us(lambda: torch.empty((b, 100), dtype=torch.bool, device=dev)),
    "torch.zeros": us(lambda: torch.zeros((b, 1), dtype=torch.bool, device=dev)),
    "torch.stack x20": us(lambda: torch.stack(xs, 1)),
    "(x > -1000).all()": us(lambda: (x > -1000).all()),
    "x.sum()": us(lambda: x.sum()),
    "int(w.item()) (sync, idle GPU)": us(lambda: int(x[0].item()), 500),
    "stack2.tolist() (sync)": us(lambda: torch.stack([x[0], x[1]]).tolist(), 500),
    "TensorDict(dict(data), [b])": us(lambda: TensorDict(dict(data.items()), [b])),
    "env.reset": us(lambda: env.reset(TensorDict(dict(data.items()), [b])), 500),
}
st = torch.zeros(1, dtype=torch.int32, device=dev)
unit["nat.call co_zero_i32-like (scratch_status)"] = us(lambda: nat.scratch_status(dev))
res["unit_us"] = unit
print(json.dumps(res), flush=True)

# ---- the loop step's pieces at this batch (us per call) -----------------------------
from rl4co_slap_amd.utils.decoding import Greedy  # noqa: E402

ts = nat.torchstep()
st2 = nat.scratch_status(dev, 2)


def steps_us(make_step, episodes=100, steps=19):
    """host us per call of make_step(td)() over `steps` calls per fresh reset (the reset
    itself outside the timed region)"""
    tot = 0.0
    for e in range(episodes + 5):
        t_ = env.reset(TensorDict(dict(data.items()), [b]))
        f = make_step(t_)
        t0 = time.perf_counter()
        for _ in range(steps):
            f()
        if e >= 5:
            tot += time.perf_counter() - t0
    torch.cuda.synchronize()
    return round(tot / episodes / steps * 1e6, 3)


piece = {}
piece["glue slap_step_td"] = steps_us(lambda t_: (lambda: ts.slap_step_td(
    env._lb_attr, t_, logits, nat.DECODE_CERTIFIED, 1.0, 10.0, None, 0, 1, st2, "action")))


def fused_step(t_):
    sg = Greedy(tanh_clipping=10.0)
    sg._status = st2
    sg._step_idx = 1  # past the episode start
    return lambda: sg.step_env_fused(logits, t_["action_mask"], t_, env)


piece["strategy.step_env_fused"] = steps_us(fused_step)
td = env.reset(TensorDict(dict(data.items()), [b]))
dec = pol.decoder
piece["decoder(td)"] = us(lambda: dec(td, None, 0), 2000)
m, i_t = td["action_mask"], td["i"]
a_out = torch.empty(b, dtype=torch.int64, device=dev)
lp_out = torch.empty(b, dtype=torch.float32, device=dev)
asg = td["assignment"]
outs = [torch.empty_like(m), torch.empty_like(i_t), torch.empty((b, 1), dtype=torch.bool, device=dev),
        torch.empty((b, 1), dtype=torch.bool, device=dev)]
args = (b, 100, 20, logits.data_ptr(), 100, m.data_ptr(), 10.0, 1.0, nat.DECODE_CERTIFIED, None,
        a_out.data_ptr(), lp_out.data_ptr(), 0, 1, None, 5, asg.data_ptr(), asg.data_ptr(),
        outs[0].data_ptr(), i_t.data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(),
        outs[3].data_ptr(), None, st2.data_ptr())
launch = nat.bind("co_slap_decode_step", *args)
sh = nat.stream_of(m)
piece["bind launch (ctypes, preconverted)"] = us(lambda: launch(sh), 2000)
piece["nat.call co_slap_decode_step B=0 (no launch)"] = us(
    lambda: nat.call("co_slap_decode_step", 0, *args[1:], sh), 2000)
piece["nat.call co_slap_decode_step"] = us(lambda: nat.call("co_slap_decode_step", *args, sh), 2000)
print(json.dumps({"batch": b, "pieces_us": piece}), flush=True)
