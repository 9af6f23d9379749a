"""Tensor helpers of ``rl4co/utils/ops.py`` for the HIP path.

``gather_by_index`` and ``get_tour_length`` run the gfx950 kernels; the batch
reshapes (``batchify``/``unbatchify``) and the multistart index generation are
view / index ops with the reference semantics (layout index ``s*B + b``).
"""
from __future__ import annotations

from typing import Union

import torch
from torch import Tensor

from .. import _native as nat
from ..td import TensorDict

# CO_EAGER_BATCHIFY=1: batchify TensorDicts with the reference's eager copy (no lazy rows)
_EAGER_BATCHIFY = bool(__import__("os").environ.get("CO_EAGER_BATCHIFY"))


def _batchify_single(x, repeats: int):
    s = x.shape
    return x.expand(repeats, *s).contiguous().view(s[0] * repeats, *s[1:])


def _batchify_td_lazy(td, repeats: int):
    """The stand-in TensorDict: every entry becomes a ``RepeatedRows`` (no copy until it
    is read, see ``td.RepeatedRows``); same keys, shapes and values as the reference's
    ``expand(...).contiguous().view(...)``."""
    from ..td import RepeatedRows

    out = TensorDict({}, batch_size=[td.batch_size[0] * repeats, *td.batch_size[1:]])
    for k in list(td.keys()):
        v = td.get_raw(k)
        if isinstance(v, RepeatedRows):  # nested batchify: materialise the inner one
            v = v.materialize()
        dict.__setitem__(out, k, RepeatedRows(v, repeats))
    return out


def batchify(x: Union[Tensor, TensorDict], shape):
    """``ops.py:19-34``: ``b ... -> (r b) ...`` (repeat-major layout).  A tensor is
    copied as in the reference; a (stand-in) TensorDict keeps its entries as lazy
    ``RepeatedRows`` (zero-copy multistart: the row-index scheme of the POMO episode)."""
    shape = [shape] if isinstance(shape, int) else shape
    for s in reversed(shape):
        if s <= 0:
            continue
        if hasattr(x, "get_raw") and len(x.batch_size) >= 1 and not _EAGER_BATCHIFY:
            x = _batchify_td_lazy(x, s)
        else:
            x = _batchify_single(x, s)
    return x


def _unbatchify_single(x, repeats: int):
    s = x.shape
    return x.view(repeats, s[0] // repeats, *s[1:]).permute(1, 0, *range(2, len(s) + 1))


def unbatchify(x: Union[Tensor, TensorDict], shape):
    """``ops.py:45-62``: ``(r b) ... -> b r ...``."""
    shape = [shape] if isinstance(shape, int) else shape
    for s in reversed(shape):
        x = _unbatchify_single(x, s) if s > 0 else x
    return x


def gather_by_index(src: Tensor, idx: Tensor, dim: int = 1, squeeze: bool = True) -> Tensor:
    """``ops.py:65-77`` on the gfx950 gather kernel.

    ``src`` is viewed as ``[outer, src.shape[dim], inner]`` (``inner`` = the product of
    the trailing dims, which must be contiguous); ``idx`` must have shape
    ``src.shape[:dim] + (M,)`` (trailing singleton dims allowed), which covers every
    call site on the hot path (rewards, CVRP demand, context embeddings, logprob
    gather, POMO best actions).
    """
    nat.require_device(src, idx)
    dim = dim % src.dim()
    if idx.dtype != torch.int64:
        idx = idx.long()
    while idx.dim() > dim + 1 and idx.shape[-1] == 1:
        idx = idx.squeeze(-1)
    lead = tuple(src.shape[:dim])
    if idx.dim() == dim:  # e.g. idx [B] for dim=1 -> one index per row
        idx = idx.unsqueeze(-1)
    if tuple(idx.shape[:dim]) != lead:
        raise RuntimeError(f"gather_by_index: index leading shape {tuple(idx.shape[:dim])} "
                           f"does not match source {lead}")
    trail = tuple(src.shape[dim + 1:])
    inner = 1
    for t in trail:
        inner *= t
    # the trailing block must be dense; leading dims must flatten to one stride
    if inner > 1 and not src[(0,) * (dim + 1)].is_contiguous():
        src = src.contiguous()
    outer = 1
    for t in lead:
        outer *= t
    if dim > 0:
        try:
            flat = src.view(outer, src.shape[dim], *trail) if outer > 0 else src
        except RuntimeError:
            src = src.contiguous()
            flat = src.view(outer, src.shape[dim], *trail)
    else:
        flat = src.unsqueeze(0)
        outer = 1
    idx2 = idx.reshape(outer, idx.shape[-1])
    m = idx2.shape[1]
    es = src.element_size()
    out = torch.empty((*lead, m, *trail), dtype=src.dtype, device=src.device)
    # out-of-range indices: the device's deferred status word, raised at the next status
    # read (torch.gather on a HIP tensor raises a device-side assert that likewise
    # surfaces at the next sync); on the CPU (host build) the check is immediate
    host = src.device.type == "cpu"
    status = nat.scratch_status(src.device) if host else nat.deferred_status(src.device)
    nat.call("co_gather_by_index", nat.ptr(flat), outer, flat.shape[1], inner * es,
             flat.stride(0) * es, flat.stride(1) * es, nat.ptr(idx2), m, idx2.stride(0),
             idx2.stride(1), nat.ptr(out), nat.ptr(status), nat.stream_of(src))
    if host:
        nat.raise_deferred(int(status.item()), None)
    elif nat.SYNC_CHECKS:
        nat.check_deferred(src.device)
    if squeeze and m == 1:
        out = out.squeeze(dim)
    return out


def unbatchify_and_gather(x: Tensor, idx: Tensor, n: int):
    """``ops.py:80-85``."""
    x = unbatchify(x, n)
    return gather_by_index(x, idx, dim=idx.dim())


def get_distance(x: Tensor, y: Tensor):
    """``ops.py:88-90`` (elementwise helper, not on the timed path)."""
    return (x - y).norm(p=2, dim=-1)


def get_tour_length(ordered_locs: Tensor) -> Tensor:
    """``ops.py:93-101`` on the TSP reward kernel: closed tour over the given order."""
    nat.require_device(ordered_locs)
    b, m, _ = ordered_locs.shape
    locs = ordered_locs.contiguous().float()
    ident = torch.arange(m, device=locs.device, dtype=torch.int64)
    out = torch.empty(b, dtype=torch.float32, device=locs.device)
    nat.call("co_tsp_reward", b, m, m, nat.ptr(locs), b, nat.ptr(ident), 0, 1, 0,
             nat.ptr(out),
             None, nat.stream_of(locs))
    return -out


def get_distance_matrix(locs: Tensor) -> Tensor:
    """``ops.py:104-111``: ``[..., N, 2] -> [..., N, N]`` Euclidean distances (gfx950
    kernel, one launch)."""
    nat.require_device(locs)
    lead, n = locs.shape[:-2], locs.shape[-2]
    flat = locs.reshape(-1, n, 2).contiguous().float()
    out = torch.empty((flat.shape[0], n, n), dtype=torch.float32, device=locs.device)
    nat.call("co_distance_matrix", flat.shape[0], n, nat.ptr(flat), nat.ptr(out),
             nat.stream_of(flat))
    return out.reshape(*lead, n, n)


def get_num_starts(td, env_name=None):
    """``ops.py:126-136``."""
    n = td["action_mask"].shape[-1]
    if env_name == "pdp":
        n = (n - 1) // 2
    elif env_name in ["cvrp", "cvrptw", "sdvrp", "mtsp", "op", "pctsp", "spctsp"]:
        n = n - 1
    return n


def select_start_nodes(td, env, num_starts):
    """``ops.py:139-163``: start action of env ``s*B + b`` is ``s % num_loc`` (TSP) or
    ``s % num_loc + 1`` (depot envs).  Envs without ``generator.num_loc`` (SLAP)
    keep the reference's ``0xFFFFFFFF`` sentinel and its off-by-one."""
    num_loc = env.generator.num_loc if hasattr(env.generator, "num_loc") else 0xFFFFFFFF
    sel = torch.arange(num_starts, device=td.device).repeat_interleave(td.shape[0]) % num_loc
    if env.name in ["tsp", "atsp", "flp", "mcp"]:
        return sel
    if env.name in ["jssp", "fjsp"]:
        raise NotImplementedError("Multistart not yet supported for FJSP/JSSP")
    return sel + 1


def get_best_actions(actions, max_idxs):
    """``ops.py:186-188``."""
    actions = unbatchify(actions, max_idxs.shape[0])
    return actions.gather(0, max_idxs[..., None, None])


def calculate_entropy(logprobs: Tensor):
    """``ops.py:114-122``: entropy of per-step log-probabilities ``[B, steps, n]``,
    summed over steps (torch ops on the device tensors; not on the timed path)."""
    logprobs = torch.nan_to_num(logprobs, nan=0.0)
    entropy = -(logprobs.exp() * logprobs).sum(dim=-1)
    entropy = entropy.sum(dim=1)
    assert entropy.isfinite().all(), "Entropy is not finite"
    return entropy
