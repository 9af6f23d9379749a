"""TSP env + generator on the gfx950 kernels (``rl4co/envs/routing/tsp/``)."""
from __future__ import annotations

from typing import Callable, Union

import torch
from torch.distributions import Uniform

from .. import _native as nat
from ..td import RepeatedRows, TensorDict, set_many
from .base import RL4COEnvBase
from .common import Generator, device_uniform, get_sampler


class TSPGenerator(Generator):
    """``tsp/generator.py:14-60``: ``locs ~ Uniform(min_loc, max_loc)`` drawn from
    torch's global CPU RNG (seeded by the env), shape ``[*B, num_loc, 2]``.  With
    ``device="cuda"`` a Uniform sampler draws on the GPU instead (``common.device_uniform``:
    same value grid, Philox stream keyed from the CPU RNG)."""

    def __init__(self, num_loc: int = 20, min_loc: float = 0.0, max_loc: float = 1.0,
                 init_sol_type: str = "random",
                 loc_distribution: Union[int, float, str, type, Callable] = Uniform, **kwargs):
        self.num_loc, self.min_loc, self.max_loc = num_loc, min_loc, max_loc
        self.init_sol_type = init_sol_type
        self.device = kwargs.get("device")
        self.loc_sampler = kwargs.get("loc_sampler") or get_sampler(
            "loc", loc_distribution, min_loc, max_loc, **kwargs)

    def _generate(self, batch_size) -> TensorDict:
        shape = (*batch_size, self.num_loc, 2)
        locs = device_uniform(self.loc_sampler, shape, self.device) if self.device else None
        if locs is None:
            locs = self.loc_sampler.sample(shape)
        return TensorDict({"locs": locs}, batch_size=batch_size)


class TSPEnv(RL4COEnvBase):
    """``tsp/env.py:29-173`` with ``_step``/``_reset``/``get_reward`` on the device."""

    name = "tsp"

    def __init__(self, generator: TSPGenerator = None, generator_params: dict = {}, **kwargs):
        super().__init__(**kwargs)
        self.generator = generator if generator is not None else TSPGenerator(**generator_params)

    def _reset(self, td=None, batch_size=None) -> TensorDict:
        """``tsp/env.py:95-120``: one fused reset kernel."""
        locs = td["locs"]
        nat.require_device(locs)
        b, n = locs.shape[0], locs.shape[-2]
        dev = locs.device
        cur = torch.empty(b, dtype=torch.int64, device=dev)  # first_node aliases it (env.py:113-114)
        mask = torch.empty((b, n), dtype=torch.bool, device=dev)
        i = torch.empty((b, 1), dtype=torch.int64, device=dev)
        reward = torch.empty((b, 1), dtype=torch.float32, device=dev)
        nat.call("co_tsp_reset", b, n, nat.ptr(mask), nat.ptr(cur), nat.ptr(cur), nat.ptr(i),
                 nat.ptr(reward), nat.stream_of(locs))
        self._remember_i(i, 0)
        self._remember_lb(mask, n)  # N ones; a step clears at most one
        return TensorDict({"locs": locs, "first_node": cur, "current_node": cur, "i": i,
                           "action_mask": mask, "reward": reward}, batch_size=batch_size)

    def _step(self, td: TensorDict) -> TensorDict:
        """``tsp/env.py:67-93`` in one kernel launch.  ``current_node`` aliases the
        action tensor exactly as the reference does."""
        action, mask, i = td["action"], td["action_mask"], td["i"]
        nat.require_device(action, mask, i)
        if action.dtype != torch.int64:
            action = action.long()
        action, mask, i = action.contiguous(), mask.contiguous(), i.contiguous()
        b, n = mask.shape
        dev = mask.device
        known = self._known_i(td["i"])
        first_in = td.get("first_node", None)
        flag = None
        if known is not None:
            mode = 1 if known == 0 else 0
        else:  # unknown provenance: batch-wide any(i == 0) on the device
            flag = torch.empty(1, dtype=torch.int32, device=dev)
            nat.call("co_any_eq_i64", nat.ptr(i), i.numel(), 0, nat.ptr(flag), nat.stream_of(i))
            mode = 2
        if first_in is None:
            first_in = action
        first_in = first_in.contiguous()
        s = nat.stream_of(mask)
        mask_out = self._out(mask.shape, mask.dtype, dev, s)
        i_out = self._out(i.shape, i.dtype, dev, s)
        first_out = self._out(action.shape, torch.int64, dev, s)
        done = self._out((b,), torch.bool, dev, s)
        reward = self._out((b,), torch.bool, dev, s)
        nat.call("co_tsp_step", b, n, nat.ptr(action), nat.ptr(mask), nat.ptr(mask_out),
                 nat.ptr(i), nat.ptr(i_out), nat.ptr(first_in), nat.ptr(first_out), None,
                 nat.ptr(done), nat.ptr(reward), mode, nat.ptr(flag), None, s)
        if known is not None:
            self._remember_i(i_out, known + 1)
        lb = self._known_lb(td["action_mask"])
        if lb is not None:
            self._remember_lb(mask_out, lb - 1)
        td.update({"first_node": first_out, "current_node": td["action"], "i": i_out,
                   "action_mask": mask_out, "reward": reward, "done": done})
        return td

    def decode_and_step(self, td, logits, mode, temperature, tanh_clipping, action_in, seed,
                        offset, status, key="action"):
        """``DecodingStrategy.step`` + ``_step`` (``decoding.py:327-369``, ``tsp/env.py:67-93``)
        in one ``co_tsp_decode_step`` launch: the same selection, log-probability, state
        and aliasing (``current_node`` is the action tensor) as the two calls.  Returns
        ``(action, logp)``, or None when it does not apply (CPU tensors, unknown ``i``
        provenance for the batch-wide first-node test, non-f32 logits)."""
        ts = nat.torchstep()
        if ts is not None:  # the whole step, bookkeeping included, in one native call
            r = ts.tsp_step_td(self._lb_attr, td, logits, mode, temperature, tanh_clipping,
                               action_in, seed, offset, status, key)
            if r is not None:
                if type(r) is int:
                    nat.check_rc("co_tsp_decode_step", r)
                return r
        return self._decode_and_step_py(td, logits, mode, temperature, tanh_clipping,
                                        action_in, seed, offset, status, key)

    def native_decode_and_step(self):
        """``decode_and_step``'s native call for a decoding strategy's loop: ``f(td,
        logits, mode, temperature, tanh_clipping, action_in, seed, offset, status, key)``
        returning ``(action, logp)``, an error code, or None (then call
        ``decode_and_step``); None when the step glue is unavailable."""
        ts = nat.torchstep()
        if ts is None:
            return None
        import functools

        return functools.partial(ts.tsp_step_td, self._lb_attr)

    def _decode_and_step_py(self, td, logits, mode, temperature, tanh_clipping, action_in,
                            seed, offset, status, key):
        mask, i = td["action_mask"], td["i"]
        known = self._known_i(i)
        if known is None:
            return None
        first_in = td.get("first_node", None)
        take = 1 if known == 0 else 0
        if not take and first_in is None:
            return None
        ts = nat.torchstep()
        if ts is not None:  # output allocation + launch in one native call
            r = ts.tsp_decode_step(logits, mask, i, None if take else first_in, action_in,
                                   status, float(tanh_clipping), float(temperature), mode, seed,
                                   offset, take)
            if r is not None:
                if type(r) is int:
                    nat.check_rc("co_tsp_decode_step", r)
                act, logp, mask_out, i_out, first_out, done, reward = r
                return self._after_decode_step(td, key, action_in, act, logp, mask, mask_out,
                                               i_out, first_out, done, reward, known)
        if logits.device.type != "cuda" or mask.device != logits.device:
            return None
        if logits.dtype != torch.float32 or logits.dim() != 2 or logits.stride(-1) != 1:
            return None
        b, n = mask.shape
        if logits.shape != (b, n) or n > 2048:  # long rows: co_decode_step's row kernel
            return None
        dev = mask.device
        m, i = mask.contiguous(), i.contiguous()
        first_in = first_in.contiguous() if (first_in is not None and not take) else None
        ain = action_in.long().contiguous() if action_in is not None else None
        s = nat.stream_of(m)
        # the decoding strategy keeps every action and log-probability: never pooled
        act = torch.empty(b, dtype=torch.int64, device=dev)
        logp = torch.empty(b, dtype=torch.float32, device=dev)
        mask_out = self._out(m.shape, m.dtype, dev, s)
        i_out = self._out(i.shape, i.dtype, dev, s)
        first_out = self._out((b,), torch.int64, dev, s)
        done = self._out((b,), torch.bool, dev, s)
        reward = self._out((b,), torch.bool, dev, s)
        nat.call("co_tsp_decode_step", b, n, nat.ptr(logits), logits.stride(0), nat.ptr(m),
                 float(tanh_clipping), float(temperature), mode, nat.ptr(ain), nat.ptr(act),
                 nat.ptr(logp), seed, offset, nat.ptr(mask_out), nat.ptr(i), nat.ptr(i_out),
                 nat.ptr(first_in), nat.ptr(first_out), take, nat.ptr(done), nat.ptr(reward),
                 None, nat.ptr(status), s)
        return self._after_decode_step(td, key, action_in, act, logp, mask, mask_out, i_out,
                                       first_out, done, reward, known)

    def _after_decode_step(self, td, key, action_in, act, logp, mask, mask_out, i_out,
                           first_out, done, reward, known):
        sel = action_in if action_in is not None else act
        self._remember_i(i_out, known + 1)
        lb = self._known_lb(mask)
        if lb is not None:
            self._remember_lb(mask_out, lb - 1)
        set_many(td, {key: sel, "first_node": first_out, "current_node": sel, "i": i_out,
                      "action_mask": mask_out, "reward": reward, "done": done})
        return sel, logp

    def _get_reward(self, td, actions, check: bool = False) -> torch.Tensor:
        """``tsp/env.py:157-173``: -tour length, fused with the permutation check.  A
        multistart td's un-replicated ``locs`` (``RepeatedRows``) is read in place: env
        ``e`` uses coordinate row ``e % B`` (the kernel's ``locs_batch``)."""
        raw = td.get_raw("locs") if hasattr(td, "get_raw") else td["locs"]
        locs = raw.source() if isinstance(raw, RepeatedRows) else raw
        nat.require_device(locs, actions)
        locs = locs.contiguous()
        if actions.dtype != torch.int64:
            actions = actions.long()
        b, t = actions.shape
        reward = torch.empty(b, dtype=torch.float32, device=locs.device)
        status = self.status_word(locs.device)
        nat.call("co_tsp_reward", b, locs.shape[-2], t, nat.ptr(locs), locs.shape[0],
                 nat.ptr(actions),
                 actions.stride(0), actions.stride(1), int(check), nat.ptr(reward),
                 nat.ptr(status), nat.stream_of(locs))
        msgs = [(nat.ST_INVALID_TOUR, AssertionError, "Invalid tour")] if check else []
        msgs.append((nat.ST_INDEX_RANGE, RuntimeError, "index out of range in gather (actions)"))
        self.raise_for_status(status, msgs)
        return reward

    def check_solution_validity(self, td, actions) -> None:
        """``tsp/env.py:165-173``."""
        self._get_reward(td, actions, check=True)

    def get_action_mask(self, td):
        return td["action_mask"]

    def min_steps_to_done(self, td) -> int:
        """done = no unvisited node (``tsp/env.py:78``), and a step clears one node."""
        return self._known_lb(td.get_raw("action_mask") if hasattr(td, "get_raw")
                              else td["action_mask"]) or 0

    def replace_selected_actions(self, cur_actions, new_actions, selection_mask):
        cur_actions[selection_mask] = new_actions[selection_mask]
        return cur_actions
