"""Host cost of one launch on the paths the drop-in loop takes (B = 64: the device work is
negligible).  Each figure is host wall time per call over many calls, the queue kept
short by a synchronize every 64 calls (not timed):

* ``entry_no_launch``: the fast-call path into a C entry that returns before launching
  (B = 0): Python -> C argument conversion alone;
* ``slap_decode_step``: the same entry at B = 64 -- validation + hipLaunchKernelGGL +
  the launch status check;
* ``probe_copy_1KiB``: the smallest kernel of the library (one workgroup, 3 arguments);
* ``torch_fill``: a torch elementwise launch (``x.fill_(1)``) for comparison;
* ``torch_empty``: a caching-allocator tensor (no launch);
* ``slap_step_td``: the whole native step glue (td dict reads, state block handling,
  the launch, three tensor wraps, td dict writes) as the drop-in loop calls it.

    python tools/launch_cost.py
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402


def per_call(f, n=4096):
    for _ in range(64):
        f()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(n // 64):
        t0 = time.perf_counter()
        for _ in range(64):
            f()
        tot += time.perf_counter() - t0
        torch.cuda.synchronize()
    return round(tot / n * 1e6, 3)


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from rl4co_slap_amd import _native as nat
    from rl4co_slap_amd.envs import SLAPEnv
    from rl4co_slap_amd.envs.slap import SLAPGenerator
    from rl4co_slap_amd.td import TensorDict

    nat.load()
    fast = nat._fastcall()
    fn, kinds = fast.table("dev")["co_slap_decode_step"]
    inv = fast.invoke
    b, l, p = 64, 100, 20
    g = torch.Generator().manual_seed(5)
    logits = torch.randn(b, l, generator=g).to(dev)
    mask = (torch.rand(b, l, generator=g) < 0.9).to(dev)
    mask[:, 1] = True
    asg = torch.randint(0, l, (b, p), dtype=torch.int32).to(dev)
    i = torch.full((b, 1), 3, dtype=torch.int64, device=dev)
    act = torch.empty(b, dtype=torch.int64, device=dev)
    lp = torch.empty(b, device=dev)
    m_o = torch.empty_like(mask)
    i_o = torch.empty_like(i)
    done, rw = (torch.empty((b, 1), dtype=torch.bool, device=dev) for _ in range(2))
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    ptr = [x.data_ptr() for x in (logits, mask, act, lp, asg, m_o, i, i_o, done, rw, st)]

    def args(bb):
        return (bb, l, p, ptr[0], l, ptr[1], 10.0, 1.0, nat.DECODE_CERTIFIED, None, ptr[2],
                ptr[3], 0, 0, None, 3, ptr[4], ptr[4], ptr[5], ptr[6], ptr[7], ptr[8], ptr[9],
                None, ptr[10], sh)

    a0, a1 = args(0), args(b)
    out = {"entry_no_launch": per_call(lambda: inv(fn, kinds, *a0)),
           "slap_decode_step": per_call(lambda: inv(fn, kinds, *a1))}
    fnc, kc = fast.table("dev")["co_probe_copy"]
    src, dst = torch.empty(256, device=dev), torch.empty(256, device=dev)
    pc = (src.data_ptr(), dst.data_ptr(), 1024, sh)
    out["probe_copy_1KiB"] = per_call(lambda: inv(fnc, kc, *pc))
    x = torch.empty(64, device=dev)
    out["torch_fill"] = per_call(lambda: x.fill_(1.0))
    out["torch_empty"] = per_call(lambda: torch.empty(64, device=dev))
    assert int(st.item()) == 0
    # the step glue on a live td: reset once, then step it (the state block and the
    # assignment are rewritten in place; i past P - 1 only sets done)
    data = SLAPGenerator(materialize_dist_mat=False)(b).to(dev)
    env = SLAPEnv(device=dev)
    td = env.reset(TensorDict(dict(data.items()), [b]))
    ts = nat.torchstep()
    step = env.native_decode_and_step()
    tc = td["to_choose"]

    def glue():
        td["to_choose"] = tc  # keep a product column to choose
        return step(td, logits, nat.DECODE_CERTIFIED, 1.0, 10.0, None, 0, 0, st, "action")

    out["slap_step_td"] = per_call(glue) if ts is not None else None
    print(json.dumps(out))


if __name__ == "__main__":
    main()
