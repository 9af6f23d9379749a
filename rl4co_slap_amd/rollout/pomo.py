"""POMO multistart greedy decode on the device (BASELINE config 5).

``POMOEpisode`` runs ``ConstructivePolicy.forward`` with multistart greedy decoding
(``rl4co/models/common/constructive/base.py:196-276``, ``decoding.py:265-313``) for
B instances x S starts as a fixed launch sequence on one stream (HIP-graph capturable):

* reset of the S*B envs (``co_tsp_reset``) in the reference's ``[S, B]`` layout
  (env ``e = s*B + b``); instance coordinates are NOT replicated -- the reward reads
  row ``e % B`` (``batchify``'s copy, ``ops.py:16``, is the cost this removes);
* the start step (``select_start_nodes``: start ``s % N``, ``ops.py:150-154``) through
  ``co_tsp_step``;
* N-1 decode-fused steps (``co_tsp_decode_step``): logits -> tanh clip -> mask ->
  log_softmax -> greedy argmax -> logp (accumulated: ``get_log_likelihood``) -> env step;
* the reward + validity (``co_tsp_reward``) and the shared baseline / REINFORCE terms
  (``co_pomo_shared_baseline``).

The logits come from the policy network in real use; the benchmark feeds a fixed
step-major logits tensor ``[N-1, S*B, N]`` resident in HBM (the network's output
stand-in), so every step reads 4N bytes of logits per env like the real decoder path.

Multi-GPU: each rank owns whole instances with all their starts, so the
shared baseline is rank-local; ``global_metrics`` all-gathers the per-instance
``[baseline, max_reward, loss_term]`` triples over RCCL (or gloo on CPU tensors).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .. import _native as nat
from ..utils.decoding import default_decode_math, math_flags
from .engine import _GraphEpisode


class POMOEpisode(_GraphEpisode):
    def __init__(self, locs: torch.Tensor, logits: torch.Tensor, num_starts: int = None,
                 tanh_clipping: float = 10.0, check: bool = True, fast_math: bool = False,
                 certified: bool = None, decode_math: str = None):
        super().__init__(locs.device)
        b, n, _ = locs.shape
        s = n if num_starts is None else num_starts
        e = s * b
        assert logits.shape == (n - 1, e, n) and logits.dtype == torch.float32
        d = locs.device
        self.b, self.n, self.s, self.e = b, n, s, e
        self.clip, self.check = float(tanh_clipping), check
        # decode math (utils/decoding.py _MATH): "certified" by default, as the decoding
        # strategies (greedy actions = the exact path's, log-probs within 1e-5);
        # "exact" = ATen bit for bit; "fast" (or fast_math=True) = opt-in approximate.
        # certified=True / False is the older spelling of "certified" / "exact".
        if decode_math is None:
            decode_math = ("fast" if fast_math else "certified" if certified
                           else "exact" if certified is False else default_decode_math())
        self.decode_math = decode_math
        self.mode = math_flags(decode_math)
        self.locs, self.logits = locs.contiguous(), logits.contiguous()
        self.acts = torch.empty((n, e), dtype=torch.int64, device=d)
        self.acts[0] = torch.arange(s, device=d).repeat_interleave(b) % n  # ops.py:150-154
        self.logp = torch.zeros((n, e), dtype=torch.float32, device=d)  # step 0: logp = 0
        self.ll = torch.empty(e, dtype=torch.float32, device=d)
        self.mask = [torch.empty((e, n), dtype=torch.bool, device=d) for _ in range(2)]
        self.i = [torch.empty((e, 1), dtype=torch.int64, device=d) for _ in range(2)]
        self.first = [torch.empty(e, dtype=torch.int64, device=d) for _ in range(2)]
        self.cur = torch.empty(e, dtype=torch.int64, device=d)
        self.done = torch.empty(e, dtype=torch.bool, device=d)
        self.step_reward = torch.empty(e, dtype=torch.bool, device=d)
        self.reset_reward = torch.empty((e, 1), dtype=torch.float32, device=d)
        self.reward = torch.empty(e, dtype=torch.float32, device=d)
        self.bl = torch.empty(b, dtype=torch.float32, device=d)
        self.max_reward = torch.empty(b, dtype=torch.float32, device=d)
        self.best_start = torch.empty(b, dtype=torch.int64, device=d)
        self.adv = torch.empty(e, dtype=torch.float32, device=d)
        self.loss_terms = torch.empty(b, dtype=torch.float32, device=d)
        self.status = torch.zeros(1, dtype=torch.int32, device=d)

    def _launch(self, st):
        b, n, e = self.b, self.n, self.e
        nat.call("co_tsp_reset", e, n, nat.ptr(self.mask[0]), nat.ptr(self.first[0]),
                 nat.ptr(self.cur), nat.ptr(self.i[0]), nat.ptr(self.reset_reward), st)
        self.ll.zero_()
        nat.call("co_tsp_step", e, n, nat.ptr(self.acts[0]), nat.ptr(self.mask[0]),
                 nat.ptr(self.mask[1]), nat.ptr(self.i[0]), nat.ptr(self.i[1]),
                 nat.ptr(self.first[0]), nat.ptr(self.first[1]), nat.ptr(self.cur),
                 nat.ptr(self.done), nat.ptr(self.step_reward), 1, None, nat.ptr(self.status), st)
        for t in range(1, n):
            src, dst = t & 1, (t + 1) & 1
            lg = self.logits[t - 1]
            nat.call("co_tsp_decode_step", e, n, nat.ptr(lg), lg.stride(0), nat.ptr(self.mask[src]),
                     self.clip, 1.0, self.mode, None, nat.ptr(self.acts[t]), nat.ptr(self.logp[t]),
                     0, t,
                     nat.ptr(self.mask[dst]), nat.ptr(self.i[src]), nat.ptr(self.i[dst]),
                     nat.ptr(self.first[src]), nat.ptr(self.first[dst]), 0, nat.ptr(self.done),
                     nat.ptr(self.step_reward), nat.ptr(self.ll), nat.ptr(self.status), st)
        nat.call("co_tsp_reward", e, n, n, nat.ptr(self.locs), b, nat.ptr(self.acts), 1, e,
                 int(self.check), nat.ptr(self.reward), nat.ptr(self.status), st)
        nat.call("co_pomo_shared_baseline", b, self.s, nat.ptr(self.reward), nat.ptr(self.ll),
                 nat.ptr(self.bl), nat.ptr(self.max_reward), nat.ptr(self.best_start),
                 nat.ptr(self.adv), nat.ptr(self.loss_terms), st)

    def final_state(self):
        k = self.n & 1
        return {"actions": self.acts.t(), "logprobs": self.logp.t(), "log_likelihood": self.ll,
                "reward": self.reward, "action_mask": self.mask[k], "done": self.done,
                "bl_val": self.bl, "max_reward": self.max_reward, "best_start": self.best_start,
                "advantage": self.adv, "loss_terms": self.loss_terms}


def shard_range(total: int, world: int, rank: int):
    """Instances [lo, hi) owned by `rank` (contiguous, balanced)."""
    base, rem = divmod(total, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def global_metrics(bl: torch.Tensor, max_reward: torch.Tensor, loss_terms: torch.Tensor,
                   num_starts: int, group=None, total_instances: int = None):
    """All-gather the per-instance shared-baseline results of every rank (RCCL on device
    tensors, gloo on CPU tensors) and form the global POMO metrics: the REINFORCE loss
    ``-(adv * ll).mean()`` over all envs (``reinforce.py:103-105``), the mean reward
    and the mean multistart max reward (``pomo/model.py:113-114``).

    With ``total_instances`` (the instances over all ranks, sharded by ``shard_range``)
    every rank knows every shard's size: the exchange is ONE padded all-gather and no host
    read.  Without it the shard sizes are all-gathered first (a second collective and a
    host read per rank)."""
    local = torch.stack([bl, max_reward, loss_terms])  # [3, B_local]
    # with a process group the exchange always runs (at world size 1 too: the same RCCL /
    # gloo call path, a copy of the local values); without one the values are local
    grouped = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if grouped else 1
    if grouped:
        if total_instances is not None:
            rank = dist.get_rank(group)
            sizes = [hi - lo for lo, hi in (shard_range(total_instances, world, r)
                                            for r in range(world))]
            if sizes[rank] != local.shape[1]:
                raise ValueError(f"global_metrics: rank {rank} holds {local.shape[1]} "
                                 f"instances, shard_range({total_instances}, {world}) gives "
                                 f"{sizes[rank]}")
        else:
            n_local = torch.tensor([local.shape[1]], device=local.device)
            all_sizes = [torch.zeros_like(n_local) for _ in range(world)]
            dist.all_gather(all_sizes, n_local, group=group)
            sizes = [int(x) for x in torch.cat(all_sizes).tolist()]
        mx = max(sizes)
        pad = torch.zeros((3, mx), dtype=local.dtype, device=local.device)
        pad[:, :local.shape[1]] = local
        bufs = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(bufs, pad, group=group)
        allv = torch.cat([buf[:, :n] for buf, n in zip(bufs, sizes)], dim=1)
    else:
        allv = local
    total_inst = allv.shape[1]
    return {"loss": -allv[2].sum() / (total_inst * num_starts), "reward_mean": allv[0].mean(),
            "max_reward_mean": allv[1].mean(), "instances": total_inst,
            "per_instance": allv}
