"""The constructive decode loop of ``rl4co/models/common/constructive/base.py:158-276``
(``ConstructivePolicy``) over the MI355X env and decoding kernels.

The encoder / decoder networks are the consumers of this API and stay PyTorch modules
(or plain callables): ``encoder(td) -> (hidden, init_embeds)`` and ``decoder(td, hidden,
num_starts) -> (logits, mask)`` with an optional ``decoder.pre_decoder_hook(td, env,
hidden, num_starts)``.  Everything between them is the hot path: the decoding step
(``co_decode_step``: tanh clip, mask, temperature, log-softmax, greedy / sampling /
evaluate selection in one launch), ``env.step`` on the env kernels, the multistart
hooks and the episode reward.  ``while not td["done"].all()`` (a host sync) is read
only from the step on which the env's host-side lower bound
(``env.min_steps_to_done``: e.g. N unvisited TSP nodes after reset) allows every
instance to be done -- the same stopping step as the reference's per-step poll.
"""
from __future__ import annotations

import logging
from typing import Callable, Optional, Union

import torch
from torch import nn

from ..envs import get_env
from ..envs.base import RL4COEnvBase
from ..utils.decoding import DecodingStrategy, get_decoding_strategy, get_log_likelihood
from ..utils.ops import calculate_entropy

log = logging.getLogger(__name__)


def _direct_call(m):
    """``m.forward`` when calling the module would go straight to it (nn.Module's own fast
    path: no hooks of any kind, not compiled, not tracing), so the decode loop skips the call wrapper's
    per-step checks; else ``m`` itself.  Decided once per ``forward``."""
    from torch.nn.modules import module as M

    if (not isinstance(m, nn.Module) or getattr(m, "_compiled_call_impl", None) is not None
            or torch._C._get_tracing_state()):
        return m
    if (m._backward_hooks or m._backward_pre_hooks or m._forward_hooks or m._forward_pre_hooks
            or M._global_backward_pre_hooks or M._global_backward_hooks
            or M._global_forward_hooks or M._global_forward_pre_hooks):
        return m
    return m.forward


class NoEncoder(nn.Module):
    """``constructive/base.py:36-40``: no encoder, hidden = initial embeddings = None."""

    def forward(self, td):
        return None, None


class ConstructiveDecoder(nn.Module):
    """``constructive/base.py:43-86`` interface: ``forward(td, hidden, num_starts)``
    returns ``(logits, mask)``; ``pre_decoder_hook`` passes through by default."""

    def forward(self, td, hidden=None, num_starts: int = 0):
        raise NotImplementedError

    def pre_decoder_hook(self, td, env, hidden=None, num_starts: int = 0):
        return td, env, hidden


class LogitsDecoder(ConstructiveDecoder):
    """Adapter for a plain ``logits_fn(td) -> logits [B, n_actions]`` (the mask is the
    env's ``action_mask``), e.g. a heuristic or a network head evaluated elsewhere."""

    def __init__(self, logits_fn: Callable):
        super().__init__()
        self.logits_fn = logits_fn

    def forward(self, td, hidden=None, num_starts: int = 0):
        return self.logits_fn(td), td["action_mask"]


class ConstructivePolicy(nn.Module):
    """``constructive/base.py:88-276``: same constructor and ``forward`` arguments."""

    def __init__(self, encoder: Union[nn.Module, Callable, None],
                 decoder: Union[nn.Module, Callable], env_name: str = "tsp",
                 temperature: float = 1.0, tanh_clipping: float = 0, mask_logits: bool = True,
                 train_decode_type: str = "sampling", val_decode_type: str = "greedy",
                 test_decode_type: str = "greedy", **unused_kw):
        super().__init__()
        if len(unused_kw) > 0:
            log.error(f"Found {len(unused_kw)} unused kwargs: {unused_kw}")
        self.env_name = env_name
        if encoder is None:
            log.warning("`None` was provided as encoder. Using `NoEncoder`.")
            encoder = NoEncoder()
        self.encoder = encoder
        self.decoder = decoder
        self.temperature, self.tanh_clipping = temperature, tanh_clipping
        self.mask_logits = mask_logits
        self.train_decode_type = train_decode_type
        self.val_decode_type = val_decode_type
        self.test_decode_type = test_decode_type

    def forward(self, td, env: Optional[Union[str, RL4COEnvBase]] = None, phase: str = "train",
                calc_reward: bool = True, return_actions: bool = False,
                return_entropy: bool = False, return_hidden: bool = False,
                return_init_embeds: bool = False, return_sum_log_likelihood: bool = True,
                actions=None, max_steps=1_000_000, **decoding_kwargs) -> dict:
        hidden, init_embeds = self.encoder(td)
        if isinstance(env, str) or env is None:
            env_name = self.env_name if env is None else env
            log.info(f"Instantiated environment not provided; instantiating {env_name}")
            env = get_env(env_name, device=td.device)
        decode_type = decoding_kwargs.pop("decode_type", None)
        if actions is not None:
            decode_type = "evaluate"
        elif decode_type is None:
            decode_type = getattr(self, f"{phase}_decode_type")
        strategy = get_decoding_strategy(
            decode_type,
            temperature=decoding_kwargs.pop("temperature", self.temperature),
            tanh_clipping=decoding_kwargs.pop("tanh_clipping", self.tanh_clipping),
            mask_logits=decoding_kwargs.pop("mask_logits", self.mask_logits),
            store_all_logp=decoding_kwargs.pop("store_all_logp", return_entropy),
            **decoding_kwargs)
        # steps that must happen before every instance can be done: the `done` poll (a host
        # sync) is skipped until then, which cannot change where the loop stops
        lb = env.min_steps_to_done(td) if hasattr(env, "min_steps_to_done") else 0
        td, env, num_starts = strategy.pre_decoder_hook(td, env)
        lb -= len(strategy.actions)  # the multistart hook's first step
        strategy.steps_hint = lb
        hook = getattr(self.decoder, "pre_decoder_hook", None)
        if hook is not None:
            td, env, hidden = hook(td, env, hidden, num_starts)
        step = 0
        decode = _direct_call(self.decoder)
        poll = getattr(env, "poll_done", None) or (lambda t: (bool(t["done"].all()), 1))
        fast = None  # greedy through the env's native glue: the per-step decisions bound once
        while True:
            if step >= lb:  # the reference's `while not td["done"].all()` test
                done, k = poll(td)
                if done:
                    break
                lb = step + k  # cannot be all done before then: no host sync until
            logits, mask = decode(td, hidden, num_starts)
            if fast is None or not fast(td, logits, mask):
                act = actions[..., step] if actions is not None else None
                # decode + env step as one launch where the env provides it (TSP, CVRP, SLAP)
                nxt = strategy.step_env_fused(logits, mask, td, env, action=act)
                if nxt is None:
                    td = strategy.step(logits, mask, td, action=act)
                    td = env.step(td)["next"]
                else:
                    td = nxt
                    if step == 0 and actions is None:
                        fast = strategy.fast_stepper(env)
            step += 1
            if step > max_steps:
                log.error(f"Exceeded maximum number of steps ({max_steps}) duing decoding")
                break
        # the epilogue (stack + log-likelihood in one launch where it applies), then the
        # reward, then ONE host read for the decode step's and the reward's checks
        if type(strategy).post_decoder_hook is DecodingStrategy.post_decoder_hook:
            logprobs, actions, td, env = strategy._post(td, env, collect=True)
        else:  # a strategy with its own hook (beam search)
            logprobs, actions, td, env = strategy.post_decoder_hook(td, env)
        if getattr(strategy, "checks", None) is not None:
            env._checks = strategy.checks
            try:
                reward = env.get_reward(td, actions) if calc_reward else None
            except BaseException:
                env._checks = None
                strategy.read_checks(logprobs)  # a decode-step error came first
                raise
            env._checks = None
            strategy.read_checks(logprobs)
            if calc_reward:
                td.set("reward", reward)
        elif calc_reward:
            td.set("reward", env.get_reward(td, actions))
        out = {"reward": td["reward"],
               "log_likelihood": get_log_likelihood(logprobs, actions, td.get("mask", None),
                                                    return_sum_log_likelihood)}
        if return_actions:
            out["actions"] = actions
        if return_entropy:
            out["entropy"] = calculate_entropy(logprobs)
        if return_hidden:
            out["hidden"] = hidden
        if return_init_embeds:
            out["init_embeds"] = init_embeds
        return out
