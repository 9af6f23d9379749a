"""Diagnostic: how many waves of the certified greedy TSP decode step take the exact
fallback at the POMO timing shape (tools/run_mode.py decode_kernels inputs), with a
library built with -DCO_DIAG_CERT_COUNT (tier-1 rows' logp -23456, tier-2 rows' -12345)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from rl4co_slap_amd import _native  # noqa: E402

_native.LIB_PATH = os.environ["CO_LIB"]
_native.load()
dev = torch.device("cuda:0")
b, n = 102400, 100
for seed, clip in ((3, 10.0), (3, 0.0), (4, 10.0)):
    g = torch.Generator().manual_seed(seed)
    logits = torch.randn(b, n, generator=g).to(dev)
    mask = (torch.rand(b, n, generator=g) < 0.5).to(dev)
    mask[:, 0] = True
    i = torch.full((b, 1), n // 2, dtype=torch.int64, device=dev)
    first = torch.zeros(b, dtype=torch.int64, device=dev)
    outs = [torch.empty(b, dtype=torch.int64, device=dev), torch.empty(b, device=dev),
            torch.empty((b, n), dtype=torch.bool, device=dev),
            torch.empty((b, 1), dtype=torch.int64, device=dev),
            torch.empty(b, dtype=torch.int64, device=dev),
            torch.empty(b, dtype=torch.bool, device=dev), torch.empty(b, dtype=torch.bool, device=dev)]
    st = torch.zeros(1, dtype=torch.int32, device=dev)
    rc = _native.call("co_tsp_decode_step", b, n, logits.data_ptr(), n, mask.data_ptr(), clip, 1.0,
                      _native.DECODE_CERTIFIED, None, outs[0].data_ptr(), outs[1].data_ptr(), 0, 0,
                      outs[2].data_ptr(), i.data_ptr(), outs[3].data_ptr(), first.data_ptr(),
                      outs[4].data_ptr(), 0, outs[5].data_ptr(), outs[6].data_ptr(), None,
                      st.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    t1 = int((outs[1] == -23456.0).sum())
    t2 = int((outs[1] == -12345.0).sum())
    print(f"seed {seed} clip {clip}: {t1} rows resolved by tier 1 (exact z of the candidates), "
          f"{t2} rows in tier-2 waves (the exact row), of {b} rows")

# the POMO TSP-100 episode (1,024 x 100 starts, 99 decode-fused steps, clip 10): the markers
# land in the per-env log-likelihood sums; count the envs whose sum holds any
from rl4co_slap_amd.rollout.pomo import POMOEpisode  # noqa: E402

torch.manual_seed(1234)
locs = torch.rand(1024, 100, 2).to(dev)
g = torch.Generator(device=dev).manual_seed(99)
logits = torch.randn((99, 102400, 100), generator=g, device=dev)
ep = POMOEpisode(locs, logits, tanh_clipping=10.0)
ep.run_eager()
torch.cuda.synchronize()
ll = ep.ll.double()
marked = ll < -5000.0
print(f"POMO episode: {int(marked.sum())} of {ll.numel()} envs hold a marked step; "
      f"about {float((-ll[marked]).sum() / 23456.0):.0f} tier-1-equivalent marks "
      f"(a tier-2 mark counts 0.53)")
