"""Restatement of ``rl4co/utils/ops.py`` (test infrastructure only)."""
from __future__ import annotations

import torch


def batchify(x, shape):
    """``ops.py:19-34``: repeat along dim 0, layout index = r*B + b."""
    shape = [shape] if isinstance(shape, int) else shape
    for s in reversed(shape):
        if s > 0:
            sz = x.shape
            x = x.expand(s, *sz).contiguous().view(sz[0] * s, *sz[1:])
    return x


def unbatchify(x, shape):
    """``ops.py:45-62``: ``(r b) ... -> b r ...``."""
    shape = [shape] if isinstance(shape, int) else shape
    for s in reversed(shape):
        if s > 0:
            sz = x.shape
            x = x.view(s, sz[0] // s, *sz[1:]).permute(1, 0, *range(2, len(sz) + 1))
    return x


def gather_by_index(src, idx, dim=1, squeeze=True):
    """``ops.py:65-77``: expand idx over src's trailing dims, gather, optional squeeze."""
    shape = list(src.shape)
    shape[dim] = -1
    idx = idx.view(idx.shape + (1,) * (src.dim() - idx.dim())).expand(shape)
    out = src.gather(dim, idx)
    if squeeze and idx.size(dim) == 1:
        return out.squeeze(dim)
    return out


def unbatchify_and_gather(x, idx, n):
    """``ops.py:80-85``."""
    x = unbatchify(x, n)
    return gather_by_index(x, idx, dim=idx.dim())


def get_distance(x, y):
    """``ops.py:88-90``."""
    return (x - y).norm(p=2, dim=-1)


def get_tour_length(ordered_locs):
    """``ops.py:93-101``: closed tour (roll by -1 along the node dim)."""
    nxt = torch.roll(ordered_locs, -1, dims=-2)
    return get_distance(nxt, ordered_locs).sum(-1)


def get_num_starts(td, env_name=None):
    """``ops.py:126-136`` (only the branches reachable by tsp/cvrp/slap matter here)."""
    n = td["action_mask"].shape[-1]
    if env_name == "pdp":
        n = (n - 1) // 2
    elif env_name in ("cvrp", "cvrptw", "sdvrp", "mtsp", "op", "pctsp", "spctsp"):
        n = n - 1
    return n


def select_start_nodes(td, env_name, num_loc, num_starts):
    """``ops.py:139-163``.  ``num_loc`` is ``env.generator.num_loc`` or ``0xFFFFFFFF``
    when the generator has none (SLAP: the fork quirk that yields start index
    ``num_loc`` for the last start)."""
    b = td.batch_size[0]
    base = torch.arange(num_starts).repeat_interleave(b) % num_loc
    if env_name in ("tsp", "atsp", "flp", "mcp"):
        return base
    return base + 1
