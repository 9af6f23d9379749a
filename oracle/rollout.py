"""Decode loop, env-only rollout and POMO shared baseline, restated on CPU
(test infrastructure only)."""
from __future__ import annotations

import torch

from .decoding import Decoding, get_log_likelihood
from .ops import unbatchify


def rollout(env, td, policy, max_steps=None):
    """``rl4co/utils/decoding.py:88-109``: step until every instance is done."""
    max_steps = float("inf") if max_steps is None else max_steps
    actions, steps = [], 0
    while not td["done"].all():
        td["action"] = policy(td)
        actions.append(td["action"])
        td = env.step(td)["next"]
        steps += 1
        if steps > max_steps:
            break
    acts = torch.stack(actions, dim=1)
    return env.get_reward(td, acts), td, acts


def constructive_forward(td, env, logits_fn, decode_type="greedy", actions=None,
                         calc_reward=True, max_steps=1_000_000, **decoding_kwargs):
    """``rl4co/models/common/constructive/base.py:196-276`` with the policy network
    replaced by ``logits_fn(td) -> logits [B, n_actions]`` (the AM decoder is a
    consumer of the env API and out of scope)."""
    if actions is not None:
        decode_type = "evaluate"
    if decode_type == "beam_search":
        from .decoding import BeamSearchOracle
        strat = BeamSearchOracle(**decoding_kwargs)
    else:
        strat = Decoding(decode_type, **decoding_kwargs)
    td, env, num_starts = strat.pre_decoder_hook(td, env)
    step = 0
    while not td["done"].all():
        logits = logits_fn(td)
        td = strat.step(logits, td["action_mask"], td,
                        action=actions[..., step] if actions is not None else None)
        td = env.step(td)["next"]
        step += 1
        if step > max_steps:
            break
    logprobs, acts, td, env = strat.post_decoder_hook(td, env)
    if calc_reward:
        td["reward"] = env.get_reward(td, acts)
    return {"reward": td["reward"], "log_likelihood": get_log_likelihood(logprobs, acts, None),
            "actions": acts, "td": td}


def shared_baseline(reward, on_dim=1):
    """``rl4co/models/rl/reinforce/baselines.py:57-61``."""
    return reward.mean(dim=on_dim, keepdims=True)


def pomo_loss(reward_flat, ll_flat, num_starts):
    """``zoo/pomo/model.py:105-113`` + ``reinforce.py:97-115`` (no augmentation,
    identity advantage scaler)."""
    reward = unbatchify(reward_flat, num_starts)
    ll = unbatchify(ll_flat, num_starts)
    bl = shared_baseline(reward)
    adv = reward - bl
    loss = -(adv * ll).mean()
    max_reward, _ = reward.max(dim=-1)
    return {"loss": loss, "bl_val": bl, "max_reward": max_reward}
