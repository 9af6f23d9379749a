"""Restatement of the per-step decode math of ``rl4co/utils/decoding.py``
(test infrastructure only)."""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .ops import batchify, gather_by_index


def top_k_filter(logits, top_k):  # decoding.py:112-117
    remove = logits < torch.topk(logits, top_k)[0][..., -1, None]
    return logits.masked_fill(remove, float("-inf"))


def top_p_filter(logits, top_p):  # decoding.py:120-138
    if top_p <= 0.0 or top_p >= 1.0:
        return logits
    sorted_logits, sorted_indices = torch.sort(logits, descending=False, stable=True)
    cumulative_probs = sorted_logits.softmax(dim=-1).cumsum(dim=-1)
    sorted_remove = cumulative_probs <= (1 - top_p)
    remove = sorted_remove.scatter(-1, sorted_indices, sorted_remove)
    return logits.masked_fill(remove, float("-inf"))


def process_logits(logits, mask=None, temperature=1.0, tanh_clipping=0.0, mask_logits=True,
                   top_k=0, top_p=0.0):
    """``decoding.py:141-191`` (ties of the top-p sort in index order: stable sort)."""
    if tanh_clipping > 0:
        logits = torch.tanh(logits) * tanh_clipping
    if mask_logits:
        assert mask is not None, "mask must be provided if mask_logits is True"
        logits = logits.clone()
        logits[~mask] = float("-inf")
    logits = logits / temperature
    if top_k > 0:
        logits = top_k_filter(logits, min(top_k, logits.size(-1)))
    if top_p > 0:
        assert top_p <= 1.0, "top-p should be in (0, 1]."
        logits = top_p_filter(logits, top_p)
    return F.log_softmax(logits, dim=-1)


def greedy(logprobs, mask=None):  # decoding.py:371-381
    sel = logprobs.argmax(dim=-1)
    if mask is not None:
        assert not (~mask).gather(1, sel.unsqueeze(-1)).data.any(), "infeasible action selected"
    return sel


def sampling(logprobs, mask=None, generator=None):  # decoding.py:383-397
    probs = logprobs.exp()
    sel = torch.multinomial(probs, 1, generator=generator).squeeze(1)
    if mask is not None:
        while (~mask).gather(1, sel.unsqueeze(-1)).data.any():
            sel = probs.multinomial(1, generator=generator).squeeze(1)
    return sel


def get_log_likelihood(logprobs, actions=None, mask=None, return_sum=True):  # decoding.py:39-65
    if actions is not None and logprobs.dim() == 3:
        logprobs = logprobs.gather(-1, actions.unsqueeze(-1)).squeeze(-1)
    if mask is not None:
        logprobs[~mask] = 0
    assert (logprobs > -1000).data.all(), "Logprobs should not be -inf, check sampling procedure!"
    return logprobs.sum(1) if return_sum else logprobs


class Decoding:
    """``DecodingStrategy`` (``decoding.py:194-369``) for greedy / sampling /
    evaluate, with multistart (``pre_decoder_hook`` ``:265-313``)."""

    def __init__(self, kind="greedy", temperature=1.0, tanh_clipping=0.0, mask_logits=True,
                 multistart=False, num_starts=None, store_all_logp=False):
        self.kind = kind.replace("multistart_", "")
        self.multistart = multistart or kind.startswith("multistart")
        self.temperature, self.tanh_clipping, self.mask_logits = temperature, tanh_clipping, mask_logits
        self.num_starts, self.store_all_logp = num_starts, store_all_logp
        self.actions, self.logprobs = [], []

    def pre_decoder_hook(self, td, env, action=None):
        from .td import batchify_td
        if self.multistart:
            if self.num_starts is None:
                self.num_starts = env.get_num_starts(td)
        else:
            self.num_starts = 0
        if self.num_starts >= 1 and self.multistart:
            if action is None:
                action = env.select_start_nodes(td, num_starts=self.num_starts)
            td = batchify_td(td, self.num_starts)
            td["action"] = action
            td = env.step(td)["next"]
            lp = torch.zeros_like(td["action_mask"]) if self.store_all_logp else torch.zeros_like(action)
            self.logprobs.append(lp)
            self.actions.append(action)
        return td, env, self.num_starts

    def step(self, logits, mask, td, action=None):  # decoding.py:327-369
        m = mask if self.mask_logits else None
        logp = process_logits(logits, m, self.temperature, self.tanh_clipping, self.mask_logits)
        if self.kind == "greedy":
            sel = greedy(logp, m)
        elif self.kind == "sampling":
            sel = sampling(logp, m)
        elif self.kind == "evaluate":
            sel = action
        else:
            raise ValueError(self.kind)
        if not self.store_all_logp:
            logp = gather_by_index(logp, sel, dim=1)
        td["action"] = sel
        self.actions.append(sel)
        self.logprobs.append(logp)
        return td

    def post_decoder_hook(self, td, env):  # decoding.py:315-325 (select_best off)
        assert len(self.logprobs) > 0
        return torch.stack(self.logprobs, 1), torch.stack(self.actions, 1), td, env


__all__ = ["process_logits", "greedy", "sampling", "get_log_likelihood", "Decoding", "batchify"]
