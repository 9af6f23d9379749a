"""An AM-shaped pointer decoder for the drop-in tests (test helper, not product code):
``am/decoder.py:162-200`` (query from the context embedding, multi-head glimpse over the
node embeddings under ``action_mask``, single-head pointer logits) with the TSP context of
``context.py:102-137`` (first + current node embeddings, a learned placeholder at
``i == 0``).  It reads ``first_node`` / ``current_node`` / ``i`` / ``action_mask`` from the
env's TensorDict exactly as the AM does.  ``oracle_logits_fn`` evaluates the same network
from the oracle's own state (on ``dev``), so identical states give identical logits."""
import math

import torch
from torch import nn

H, HEADS = 32, 4


class PointerDecoder(nn.Module):
    """A small attention-model decoder (random init, eval mode, on the device)."""

    def __init__(self, locs_bn2, dev, depot_env=False, cache=False):
        super().__init__()
        self.cache = cache  # precompute the key / value / logit-key projections once (the
        self._kvl = None    # AM's _precompute_cache, am/decoder.py:138-160)
        g = torch.Generator().manual_seed(5)

        def lin(i, o):
            m = nn.Linear(i, o, bias=False)
            with torch.no_grad():
                m.weight.copy_(torch.randn(o, i, generator=g) / math.sqrt(i))
            return m

        self.init_embed = lin(2, H)
        self.wq, self.wk, self.wv, self.wo, self.wl = (lin(2 * H, H), lin(H, H), lin(H, H),
                                                       lin(H, H), lin(H, H))
        self.placeholder = nn.Parameter(torch.randn(2 * H, generator=g))
        self.depot_env = depot_env
        self.to(dev).eval()
        with torch.no_grad():  # "encoder": node embeddings of the B instances
            self.h = self.init_embed(locs_bn2.to(dev))
        self.b = locs_bn2.shape[0]

    @torch.no_grad()
    def logits(self, first, cur, i, mask):
        """am/decoder.py:162-200 shaped: glimpse + pointer; rows e of a multistart batch
        use instance e % B's embeddings (the AM batchifies its cached embeddings)."""
        e = first.shape[0]
        n = self.h.shape[1]
        if self.cache and self._kvl is not None and self._kvl[0].shape[0] == e:
            rows = self._rows  # the cached projections stand for h: gather the two rows only
            hf, hc = self.h[rows, first.reshape(e)], self.h[rows, cur.reshape(e)]
            h = None
        else:
            self._rows = torch.arange(e, device=self.h.device) % self.b
            h = self.h[self._rows]  # [E, N, H]
            hf = h.gather(1, first.reshape(e, 1, 1).expand(e, 1, H)).squeeze(1)
            hc = h.gather(1, cur.reshape(e, 1, 1).expand(e, 1, H)).squeeze(1)
        ctx = torch.cat([hf, hc], -1)
        if not self.depot_env:  # TSP context: the placeholder before the first step
            ctx = torch.where((i.reshape(e, 1) == 0), self.placeholder.expand(e, -1), ctx)
        q = self.wq(ctx).view(e, HEADS, 1, H // HEADS)
        if self.cache:
            if self._kvl is None or self._kvl[0].shape[0] != e:
                self._kvl = (self.wk(h).view(e, n, HEADS, H // HEADS).permute(0, 2, 3, 1),
                             self.wv(h).view(e, n, HEADS, H // HEADS).transpose(1, 2),
                             self.wl(h).transpose(1, 2).contiguous())
            kt, v, lt = self._kvl
        else:
            kt = self.wk(h).view(e, n, HEADS, H // HEADS).permute(0, 2, 3, 1)
            v = self.wv(h).view(e, n, HEADS, H // HEADS).transpose(1, 2)
            lt = self.wl(h).transpose(1, 2)
        att = (q @ kt) / math.sqrt(H // HEADS)
        att = att.masked_fill(~mask.view(e, 1, 1, n), float("-inf"))
        glimpse = self.wo((att.softmax(-1) @ v).reshape(e, H))
        return (glimpse.unsqueeze(1) @ lt).squeeze(1) / math.sqrt(H)

    # ConstructiveDecoder interface (constructive/base.py:43-86)
    def forward(self, td, hidden=None, num_starts: int = 0):
        first = td["first_node"] if not self.depot_env else td["current_node"]
        i = td["i"] if "i" in td else torch.ones_like(td["current_node"])
        return self.logits(first, td["current_node"], i, td["action_mask"]), td["action_mask"]

    def pre_decoder_hook(self, td, env, hidden=None, num_starts: int = 0):
        return td, env, hidden


def _oracle_logits_fn(dec, dev):
    def fn(td):  # the same network on the device, from the ORACLE's state
        first = td["first_node"] if not dec.depot_env else td["current_node"]
        i = td["i"] if "i" in td.keys() else torch.ones_like(td["current_node"])
        return dec.logits(first.to(dev), td["current_node"].to(dev), i.to(dev),
                          td["action_mask"].to(dev)).cpu()
    return fn


def oracle_logits_fn(dec, dev):
    def fn(td):  # the same network on `dev`, from the ORACLE's state
        first = td["first_node"] if not dec.depot_env else td["current_node"]
        i = td["i"] if "i" in td.keys() else torch.ones_like(td["current_node"])
        return dec.logits(first.to(dev), td["current_node"].to(dev), i.to(dev),
                          td["action_mask"].to(dev)).cpu()
    return fn


class SLAPPointerDecoder(nn.Module):
    """The fork's SLAP policy (``examples/slap.py:11-93``) in the AM decoder's shape
    (``am/decoder.py:134-200``): node features ``cat(locs, dist_mat[:, 0, :])`` (the
    Manhattan distance of every location to the depot) through ``Linear(3, H)``
    (``SLAPInitEmbedding``), a zero step context (``SLAPContext``), a static dynamic
    embedding (``StaticEmbedding``), so the query is the projected graph context
    ``project_fixed_context(mean(h))`` alone; glimpse + pointer over ``action_mask``.
    Random init, eval mode, on the device; key / value / logit projections precomputed
    (``_precompute_cache``).  Rows e of a multistart batch use instance e % B."""

    def __init__(self, locs_bl2, dev):
        super().__init__()
        g = torch.Generator().manual_seed(9)

        def lin(i, o, bias=False):
            m = nn.Linear(i, o, bias=bias)
            with torch.no_grad():
                m.weight.copy_(torch.randn(o, i, generator=g) / math.sqrt(i))
                if bias:
                    m.bias.copy_(0.1 * torch.randn(o, generator=g))
            return m

        self.init_embed = lin(3, H, bias=True)
        self.wfix, self.wk, self.wv, self.wo, self.wl = (lin(H, H), lin(H, H), lin(H, H),
                                                         lin(H, H), lin(H, H))
        self.to(dev).eval()
        locs = locs_bl2.to(dev)
        with torch.no_grad():
            dist0 = (locs[:, :1, :] - locs).abs().sum(-1)  # dist_mat[:, 0, :] (Manhattan)
            h = self.init_embed(torch.cat((locs, dist0[..., None]), -1))  # [B, L, H]
            b, n = h.shape[0], h.shape[1]
            self.q = self.wfix(h.mean(1))  # graph context + zero step context
            self.kt = self.wk(h).view(b, n, HEADS, H // HEADS).permute(0, 2, 3, 1)
            self.v = self.wv(h).view(b, n, HEADS, H // HEADS).transpose(1, 2)
            self.lt = self.wl(h).transpose(1, 2).contiguous()
        self.b = b

    @torch.no_grad()
    def logits(self, mask):
        e, n = mask.shape
        rows = torch.arange(e, device=mask.device) % self.b
        q = self.q[rows].view(e, HEADS, 1, H // HEADS)
        att = (q @ self.kt[rows]) / math.sqrt(H // HEADS)
        att = att.masked_fill(~mask.view(e, 1, 1, n), float("-inf"))
        glimpse = self.wo((att.softmax(-1) @ self.v[rows]).reshape(e, H))
        return (glimpse.unsqueeze(1) @ self.lt[rows]).squeeze(1) / math.sqrt(H)

    def forward(self, td, hidden=None, num_starts: int = 0):
        return self.logits(td["action_mask"]), td["action_mask"]

    def pre_decoder_hook(self, td, env, hidden=None, num_starts: int = 0):
        return td, env, hidden


def slap_oracle_logits_fn(dec, dev, rows_total=None):
    """The SLAP decoder on `dev` from the ORACLE's mask.  ``rows_total``: evaluate the
    oracle's rows as the first rows of a batch of that many (the rest all-feasible), so
    every GEMM has the device run's shapes and the rows get the device run's bits."""
    def fn(td):
        m = td["action_mask"].to(dev)
        if rows_total is not None and rows_total > m.shape[0]:
            pad = torch.ones((rows_total - m.shape[0], m.shape[1]), dtype=torch.bool, device=dev)
            return dec.logits(torch.cat((m, pad), 0))[: m.shape[0]].cpu()
        return dec.logits(m).cpu()
    return fn
