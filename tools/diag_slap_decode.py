"""Diagnostic: GPU time of one co_slap_decode_step launch (certified greedy, tanh clip 10:
the drop-in loop's settings) at L = 100, P = 20 on a mid-episode state, HIP events over
100 launches, inputs cycled over 4 copies (HBM reads).  Two operand forms: "dropin" = what
the step glue passes (to_choose NULL with the uniform product, the assignment written in
place), "clone" = to_choose read per row and the assignment copied out of place (the
reference's clone).  CO_LIB picks a variant library (tools/build_variants.sh)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
from rl4co_slap_amd import _native  # noqa: E402

if os.environ.get("CO_LIB"):
    _native.LIB_PATH = os.environ["CO_LIB"]
_native.load()
dev = torch.device("cuda:0")
l, p = 100, 20
res = {}
for b in (16384, 65536):
    g = torch.Generator().manual_seed(5)
    sets = []
    for _ in range(4):
        mask = torch.rand(b, l, generator=g) < 0.9
        mask[:, 0] = False
        mask[:, 1] = True
        sets.append({"logits": torch.randn(b, l, generator=g).to(dev), "mask": mask.to(dev),
                     "asg": torch.randint(0, l, (b, p), dtype=torch.int32, generator=g).to(dev),
                     "tc": torch.arange(p, dtype=torch.float32).repeat(b, 1).to(dev),
                     "i": torch.full((b, 1), p // 2, dtype=torch.int64, device=dev)})
    act = torch.empty(b, dtype=torch.int64, device=dev)
    lp = torch.empty(b, dtype=torch.float32, device=dev)
    asg_o = torch.empty(b, p, dtype=torch.int32, device=dev)
    m_o = torch.empty(b, l, dtype=torch.bool, device=dev)
    i_o = torch.empty(b, 1, dtype=torch.int64, device=dev)
    done, rw = (torch.empty((b, 1), dtype=torch.bool, device=dev) for _ in range(2))
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    for form in ("dropin", "clone"):
        launches = []
        for s in sets:
            tc = None if form == "dropin" else s["tc"][:, p // 2:].data_ptr()
            tcs = p // 2 if form == "dropin" else p
            ao = s["asg"].data_ptr() if form == "dropin" else asg_o.data_ptr()
            launches.append(_native.bind(
                "co_slap_decode_step", b, l, p, s["logits"].data_ptr(), l, s["mask"].data_ptr(),
                10.0, 1.0, _native.DECODE_CERTIFIED, None, act.data_ptr(), lp.data_ptr(), 0, 0,
                tc, tcs, s["asg"].data_ptr(), ao, m_o.data_ptr(), s["i"].data_ptr(),
                i_o.data_ptr(), done.data_ptr(), rw.data_ptr(), None, st.data_ptr()))
        it = [0]

        def run():
            launches[it[0] % 4](sh)
            it[0] += 1

        _, ev = bench.timed(run, 100, 8, 1, dev)
        res[f"{form}_b{b}_us"] = round(ev / 100 * 1e6, 3)
print(json.dumps(res))
