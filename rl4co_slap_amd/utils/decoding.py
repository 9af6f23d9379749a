"""Decoding strategies (``rl4co/utils/decoding.py``) on the fused gfx950 decode step.

``DecodingStrategy.step`` issues one ``co_decode_step`` launch per decode step:
tanh clipping, masking, temperature, ``log_softmax``, greedy argmax / Philox
sampling / evaluate, and the logprob gather.  The greedy/sampling feasibility
assertion (``decoding.py:376-379,393-395``) is recorded in a device status word
and raised once in ``post_decoder_hook`` instead of synchronising every step.
Top-k / top-p filtering runs inside the same launch (``co_decode_step_ex``); beam search
ranks the beams' candidates with ``co_beam_select`` and re-indexes the state rows with
the device gather.
"""
from __future__ import annotations

import abc
from typing import Optional, Tuple

import torch

from .. import _native as nat
from ..td import TensorDict
from .ops import batchify, gather_by_index, unbatchify, unbatchify_and_gather

_MODES = {"greedy": 0, "sampling": 1, "evaluate": 2}
_NO_FUSED = bool(__import__("os").environ.get("CO_NO_FUSED_STEP"))  # A/B switch (tests, diag)
# A/B switch: the greedy loop's per-step closure in Python instead of the glue's fast_step
_NO_FAST_STEP = bool(__import__("os").environ.get("CO_NO_FAST_STEP"))

# Decode math (the mode word's flag bits, include/co_env.h):
# * "exact": ATen's CPU log_softmax restated bit for bit (SLEEF expf/logf, map_reduce_all
#   order, correctly rounded tanh) for every mode;
# * "certified": greedy picks on the fast math, each row certified by an error bound and
#   any wave holding an uncertified row recomputed exactly -- the greedy ACTIONS are the
#   exact path's; the log-probabilities are the fast math's, within 1e-5 (measured ~1e-6)
#   of the exact ones.  Sampling / evaluate / top-k / top-p / beam ranking stay exact;
# * "fast": opt-in approximate math everywhere (not bit-exact; benchmarks only).
# The decoding strategies default to "certified" (CO_DECODE_MATH overrides it); the
# low-level ``decode_step`` defaults to "exact".
_MATH = {"exact": 0, "certified": nat.DECODE_CERTIFIED, "fast": nat.DECODE_FAST}


def default_decode_math() -> str:
    m = __import__("os").environ.get("CO_DECODE_MATH", "certified")
    if m not in _MATH:
        raise ValueError(f"CO_DECODE_MATH={m!r}: expected one of {sorted(_MATH)}")
    return m


def math_flags(math: str) -> int:
    try:
        return _MATH[math]
    except KeyError:
        raise ValueError(f"decode_math={math!r}: expected one of {sorted(_MATH)}") from None


def decode_step(logits, mask, mode: str, temperature=1.0, tanh_clipping=0.0, action=None,
                return_full=False, seed=None, offset=0, status=None, top_k: int = 0,
                top_p: float = 0.0, math: str = "exact"):
    """One fused decode step.  Returns ``(action[B], logp[B], full_logprobs or None)``.
    ``math`` selects the decode math (``_MATH`` above)."""
    flags = math_flags(math)
    mword = _MODES[mode] | flags
    if seed is None:
        seed = int(torch.randint(0, 2**62, ()).item()) if mode == "sampling" else 0
    ts = nat.torchstep() if top_k <= 0 and top_p <= 0 else None
    if ts is not None:  # output allocation + launch in one native call (device tensors)
        r = ts.decode_step(logits, mask, action, status, float(tanh_clipping),
                           float(temperature), mword, seed, offset, return_full)
        if r is not None:
            if type(r) is int:
                nat.check_rc("co_decode_step", r)
            return r
    nat.require_device(logits, mask, action)
    if logits.dtype != torch.float32:
        logits = logits.float()
    if logits.stride(-1) != 1:
        logits = logits.contiguous()
    b, n = logits.shape
    dev = logits.device
    if mask is not None:
        mask = mask.contiguous()
    act_out = torch.empty(b, dtype=torch.int64, device=dev)
    logp = torch.empty(b, dtype=torch.float32, device=dev)
    full = torch.empty((b, n), dtype=torch.float32, device=dev) if return_full else None
    if action is not None:
        action = action.long().contiguous()
    if top_k > 0 or top_p > 0:
        assert top_p <= 1.0, "top-p should be in (0, 1]."
        nat.call("co_decode_step_ex", b, n, nat.ptr(logits), logits.stride(0), nat.ptr(mask),
                 float(tanh_clipping), float(temperature), min(int(top_k), n), float(top_p),
                 _MODES[mode] | flags, nat.ptr(action), nat.ptr(act_out), nat.ptr(logp), nat.ptr(full),
                 seed, offset, nat.ptr(status), nat.stream_of(logits))
    else:
        nat.call("co_decode_step", b, n, nat.ptr(logits), logits.stride(0), nat.ptr(mask),
                 float(tanh_clipping), float(temperature), mword,
                 nat.ptr(action), nat.ptr(act_out), nat.ptr(logp), nat.ptr(full), seed, offset, nat.ptr(status),
                 nat.stream_of(logits))
    return act_out, logp, full


def process_logits(logits, mask=None, temperature: float = 1.0, top_p: float = 0.0,
                   top_k: int = 0, tanh_clipping: float = 0, mask_logits: bool = True):
    """``decoding.py:141-191`` -> full log-probabilities."""
    if mask_logits:
        assert mask is not None, "mask must be provided if mask_logits is True"
    _, _, full = decode_step(logits, mask if mask_logits else None, "greedy", temperature,
                             tanh_clipping, return_full=True, top_k=top_k, top_p=top_p)
    return full


def get_log_likelihood(logprobs, actions=None, mask=None, return_sum: bool = True):
    """``decoding.py:39-65``.  The ``> -1000`` assert needs a host sync; for logprobs
    that ``post_decoder_hook`` produced, the same test was folded into its single
    status read (``_co_logp_ok``), so no second sync happens here; and when its epilogue
    kernel (``co_episode_stack``) also summed them, that sum is returned (``_co_ll``)."""
    rec = getattr(logprobs, "_co_logp_ok", None)
    # the folded test is valid only while the tensor is unchanged since it was made
    checked = rec[0] if rec is not None and rec[1] == logprobs._version else None
    ll = getattr(logprobs, "_co_ll", None) if return_sum and mask is None else None
    if actions is not None and logprobs.dim() == 3:
        logprobs = logprobs.gather(-1, actions.unsqueeze(-1)).squeeze(-1)
    if mask is not None:
        logprobs[~mask] = 0
        checked = None  # the precomputed test saw the unmasked values
    if checked is None:
        checked = bool((logprobs > -1000).data.all())
    assert checked, "Logprobs should not be -inf, check sampling procedure!"
    if ll is not None and ll[1] == logprobs._version:
        return ll[0]
    return logprobs.sum(1) if return_sum else logprobs


def random_policy(td):
    """``decoding.py:81-85``."""
    action = torch.multinomial(td["action_mask"].float(), 1).squeeze(-1)
    td.set("action", action)
    return td


def _own_step(env) -> bool:
    """True when ``env``'s ``_step`` is the one its ``decode_and_step`` fuses: the class
    that defines ``decode_and_step`` (and ``native_decode_and_step``) must also be the one
    whose ``_step`` the env runs.  A subclass that overrides ``_step`` (a CVRPTW- or
    SDVRP-like env on top of CVRPEnv) inherits the fused call but not its transition, so
    it takes the two-call path."""
    cls = type(env)
    if "_step" in getattr(env, "__dict__", {}):  # replaced on the instance
        return False
    for name in ("decode_and_step", "native_decode_and_step"):
        owner = next((c for c in cls.__mro__ if name in c.__dict__), None)
        if owner is not None and getattr(cls, "_step", None) is not owner.__dict__.get("_step"):
            return False
    return True


def rollout(env, td, policy, max_steps: int = None):
    """``decoding.py:88-109``."""
    max_steps = float("inf") if max_steps is None else max_steps
    actions, steps = [], 0
    lb = env.min_steps_to_done(td) if hasattr(env, "min_steps_to_done") else 0
    poll = getattr(env, "poll_done", None) or (lambda t: (bool(t["done"].all()), 1))
    while True:  # same stop; polls only once every instance can be done
        if steps >= lb:
            done, k = poll(td)
            if done:
                break
            lb = steps + k
        td = policy(td)
        actions.append(td["action"])
        td = env.step(td)["next"]
        steps += 1
        if steps > max_steps:
            break
    acts = torch.stack(actions, dim=1)
    return env.get_reward(td, acts), td, acts


def _stack_device(actions, logprobs, status):
    """``torch.stack(actions, 1)`` / ``torch.stack(logprobs, 1)`` + the log-likelihood
    sum and the ``> -1000`` test through ``co_episode_stack`` on step-major stacks (the
    same kernel, so the same bits, as the step glue's slab path); int64 actions ride along,
    others (int32 evaluate actions) are stacked by torch.  None when the per-step
    log-probabilities are not [B] f32 tensors on the status word's device."""
    l0 = logprobs[0]
    if l0.dim() != 1 or l0.dtype != torch.float32 or l0.device != status.device:
        return None
    L = torch.stack(logprobs, 0)  # [T, B]: rows are the steps' tensors (checks shapes too)
    t, b = L.shape
    dev = L.device
    a0 = actions[0]
    A = None
    if a0.dim() == 1 and a0.dtype == torch.int64 and a0.device == dev:
        A = torch.stack(actions, 0)
        if A.shape != L.shape:
            return None
        acts = torch.empty((b, t), dtype=torch.int64, device=dev)
    else:
        acts = torch.stack(actions, 1)
    lps = torch.empty((b, t), dtype=torch.float32, device=dev)
    ll = torch.empty(b, dtype=torch.float32, device=dev)
    nat.call("co_episode_stack", b, t, nat.ptr(A), b, nat.ptr(L), b,
             nat.ptr(acts) if A is not None else None, nat.ptr(lps), nat.ptr(ll),
             nat.ptr(status), nat.stream_of(L))
    return acts, lps, ll


class _Checks:
    """The data-dependent checks of one decode episode, read in ONE host sync.

    Word 0 of the strategy's status tensor collects the decode steps' bits (infeasible
    selection, ``decoding.py:376-379,393-395``; out-of-range env indices) and the
    epilogue's ``> -1000`` test (``co_episode_stack``, ``decoding.py:57-58``); word 1 is
    the status word of the kernels an env runs while the collection is open (the reward
    and its validity asserts, ``base.py:182-188``).  ``read`` raises in the reference's
    order: the decode step's assertion, then the reward's, and records the
    log-probability test for ``get_log_likelihood`` (which raises it there)."""

    def __init__(self, status: torch.Tensor):
        self.status = status
        self._word1 = None
        self.env_msgs = []

    def env_word(self) -> torch.Tensor:
        if self._word1 is None:
            self._word1 = self.status[1:]
        return self._word1

    def owns(self, t) -> bool:
        return self._word1 is not None and t is self._word1

    def add(self, messages):
        self.env_msgs.extend(messages)

    def read(self):
        """-> the decode word's bits (the caller raises / records them); raises the env
        messages and the device's deferred gather errors."""
        st = self.status
        d = nat.pending_deferred(st.device) if st.device.type != "cpu" else None
        vals = [int(v) for v in (torch.cat([st, d]) if d is not None else st).tolist()]
        if d is not None:
            nat.raise_deferred(vals[2], st.device)
        w0, w1 = vals[0], vals[1]
        if w0 & nat.ST_INFEASIBLE:
            raise AssertionError("infeasible action selected")
        for bit, exc, msg in self.env_msgs:
            if w1 & bit:
                raise exc(msg)
        nat.release_status(st, vals[:2])
        return w0


class DecodingStrategy(metaclass=abc.ABCMeta):
    """``decoding.py:194-407``."""

    name = "base"

    def __init__(self, temperature: float = 1.0, top_p: float = 0.0, top_k: int = 0,
                 mask_logits: bool = True, tanh_clipping: float = 0, multistart: bool = False,
                 multisample: bool = False, num_starts: Optional[int] = None,
                 select_start_nodes_fn: Optional[callable] = None,
                 improvement_method_mode: bool = False, select_best: bool = False,
                 store_all_logp: bool = False, key: str = "action",
                 decode_math: Optional[str] = None, **kwargs):
        self.temperature, self.top_p, self.top_k = temperature, top_p, top_k
        # "certified" by default: exact greedy actions, log-probabilities within 1e-5
        self.decode_math = decode_math if decode_math is not None else default_decode_math()
        self._math_flags = math_flags(self.decode_math)
        self.mask_logits, self.tanh_clipping = mask_logits, tanh_clipping
        self.multistart, self.multisample = multistart, multisample
        self.num_starts, self.select_start_nodes_fn = num_starts, select_start_nodes_fn
        self.improvement_method_mode, self.select_best = improvement_method_mode, select_best
        self.store_all_logp, self.key = store_all_logp, key
        self.actions, self.logprobs = [], []
        self._status = None
        self._step_idx = 0
        self._fused = None  # (env, its decode_and_step or None, mode, mode word)

    def pre_decoder_hook(self, td, env, action=None):
        """``decoding.py:265-313``."""
        if self.multistart or self.multisample:
            if self.num_starts is None:
                self.num_starts = env.get_num_starts(td)
        else:
            self.num_starts = 0
        if self.num_starts >= 1:
            if self.multistart:
                if action is None:
                    if self.select_start_nodes_fn is not None:
                        action = self.select_start_nodes_fn(td, env, self.num_starts)
                    else:
                        action = env.select_start_nodes(td, num_starts=self.num_starts)
                td = batchify(td, self.num_starts)
                td.set("action", action)
                td = env.step(td)["next"]
                lp = torch.zeros_like(td["action_mask"]) if self.store_all_logp else \
                    torch.zeros_like(action, device=td.device)
                self.logprobs.append(lp)
                self.actions.append(action)
            else:
                td = batchify(td, self.num_starts)
        return td, env, self.num_starts

    def post_decoder_hook(self, td, env):
        """``decoding.py:315-325`` + the deferred feasibility assertion."""
        out = self._post(td, env, collect=False)
        return out

    def _post(self, td, env, collect: bool):
        """``post_decoder_hook``'s work.  On the device, per-step [B] actions (int64) and
        log-probabilities (f32) are stacked by ONE ``co_episode_stack`` launch that also
        sums the log-likelihood (``get_log_likelihood``) and tests ``> -1000`` into the
        status word -- straight from the step glue's slabs when the rows are one block
        (no torch.stack at all), else from a step-major torch.stack.  collect=True (the
        decode loop, which reads its checks once after the reward): the status read is
        left to ``self.checks`` (``_Checks.read``).  Other layouts (CPU tensors, full
        log-probabilities, int32 evaluate actions) take torch.stack and a read here."""
        assert len(self.logprobs) > 0, \
            "No logprobs were collected because all environments were done. Check your initial state"
        st = self._status
        r = None
        if (st is not None and st.device.type != "cpu" and st.shape[0] >= 2
                and not self.store_all_logp):
            ts = nat.torchstep()
            r = ts.episode_stack(self.actions, self.logprobs, st, True) if ts is not None else None
            if type(r) is int:
                nat.check_rc("co_episode_stack", r)
            if r is None:
                r = _stack_device(self.actions, self.logprobs, st)
        if r is not None:
            actions, logprobs, ll = r
            logprobs._co_ll = (ll, logprobs._version)
            if collect and not (self.num_starts > 0 and self.select_best):
                self.checks = _Checks(st)
                self._status = None
                return logprobs, actions, td, env
            w0 = _Checks(st).read()
            self._status = None
            self._finish_checks(logprobs, w0)
            if self.num_starts > 0 and self.select_best:
                logprobs, actions, td, env = self._select_best(logprobs, actions, td, env)
            return logprobs, actions, td, env
        logprobs = torch.stack(self.logprobs, 1)
        actions = torch.stack(self.actions, 1)
        # one host read for the deferred feasibility assert and get_log_likelihood's
        # `> -1000` test (decoding.py:57-58) on the same logprobs
        # (per-step selected logprobs only: full [B, steps, N] ones hold -inf at masked
        # entries, and get_log_likelihood tests them after its gather)
        flat = logprobs.dim() == 2
        ok = ((logprobs > -1000).all() if flat else torch.ones((), dtype=torch.bool,
                                                                device=logprobs.device))
        ok = ok.to(torch.int32)
        st = self._status[0] if self._status is not None else torch.zeros_like(ok)
        words = [st.reshape(()), ok]
        d = nat.pending_deferred(ok.device) if ok.device.type != "cpu" else None
        if d is not None:  # an out-of-range gather_by_index since the last read
            words.append(d.reshape(()))
        vals = [int(v) for v in torch.stack(words).tolist()]
        st_bits, lp_ok = vals[0], vals[1]
        if d is not None:
            nat.raise_deferred(vals[2], ok.device)
        if st_bits & nat.ST_INFEASIBLE:
            raise AssertionError("infeasible action selected")
        if flat:
            # the test result holds for these values only: keyed by the tensor's version
            logprobs._co_logp_ok = (bool(lp_ok), logprobs._version)
        if self.num_starts > 0 and self.select_best:
            logprobs, actions, td, env = self._select_best(logprobs, actions, td, env)
        return logprobs, actions, td, env

    @staticmethod
    def _finish_checks(logprobs, w0: int):
        """After the read: the epilogue's ``> -1000`` test, kept for get_log_likelihood
        (valid while the tensor is unchanged)."""
        logprobs._co_logp_ok = (not (w0 & nat.ST_LOGP_NEG_INF), logprobs._version)

    def read_checks(self, logprobs):
        """The decode loop's single host read (``_post(collect=True)`` left it pending):
        raises the decode step's and the reward's errors in the reference's order."""
        checks = getattr(self, "checks", None)
        if checks is None:
            return
        self.checks = None
        self._finish_checks(logprobs, checks.read())

    def _episode_start(self):
        """At an episode's first decode step: the step glue's next action / log-probability
        rows start a slab sized for the episode (``steps_hint``: the env's bound, set by
        the decode loop), so that ``co_episode_stack`` can take them as one block."""
        ts = nat.torchstep()
        if ts is not None:
            h = getattr(self, "steps_hint", 0)
            ts.slab_fresh(2 * h + 8 if h else 64)

    def _new_status(self, device):
        """The strategy's status words (0: the decode steps + epilogue, 1: the env kernels
        of the decode loop's checks, _Checks)."""
        return nat.scratch_status(device, 2)

    def step(self, logits, mask, td: TensorDict = None, action=None, env=None, **kwargs):
        """``decoding.py:327-369`` as one fused launch."""
        if not self.mask_logits:
            mask = None
        if self._status is None:
            self._status = self._new_status(logits.device)
        if self._step_idx == 0:
            self._episode_start()
        mode = self._mode()
        act_in = action if mode == "evaluate" else None
        seed = getattr(self, "_seed_carry", None)
        self._seed_carry = None
        sel, logp, full = decode_step(logits, mask, mode, self.temperature, self.tanh_clipping,
                                      action=act_in, return_full=self.store_all_logp,
                                      seed=seed, offset=self._step_idx, status=self._status,
                                      top_k=self.top_k, top_p=self.top_p,
                                      math=self.decode_math)
        self._step_idx += 1
        if mode == "evaluate":
            sel = action
        if self.improvement_method_mode:
            return (full if full is not None else logp), sel
        out_lp = full if self.store_all_logp else logp
        td.set(self.key, sel)
        self.actions.append(sel)
        self.logprobs.append(out_lp)
        return td

    def step_env_fused(self, logits, mask, td, env, action=None):
        """``self.step`` followed by ``env.step`` as ONE launch, when the env offers it
        (``decode_and_step``: ``co_tsp_decode_step`` / ``co_slap_decode_step`` /
        ``co_cvrp_decode_step``) and nothing in between could
        observe the difference: the env's own ``step``, the mask the env holds, no full
        log-probabilities / top-k / top-p.  Same outputs, same RNG use; returns the next
        td, or None when the fused path does not apply (the caller runs both steps)."""
        # the strategy-side conditions, decided once per env (the settings do not change
        # inside a decode loop)
        cached = self._fused
        if cached is None or cached[0] is not env:
            fused = getattr(env, "decode_and_step", None)
            mode = self._mode()
            if (fused is None or not _own_step(env) or _NO_FUSED or self.store_all_logp
                    or self.improvement_method_mode
                    or self.top_k > 0 or 0.0 < self.top_p < 1.0 or not self.mask_logits
                    or mode not in _MODES):
                fused = None
            # the env's native form of the same call (TSPEnv: csrc/pycall), tried first
            native = getattr(env, "native_decode_and_step", None)
            native = native() if (native is not None and fused is not None) else None
            cached = self._fused = (env, fused, native, mode,
                                    _MODES.get(mode, 0) | self._math_flags)
        _, fused, native, mode, mword = cached
        if fused is None or getattr(env, "_torchrl_mode", False):
            return None
        held = dict.get(td, "action_mask") if type(td) is TensorDict else td.get("action_mask")
        if mask is not held:
            return None
        if self._status is None:
            self._status = self._new_status(logits.device)
        if self._step_idx == 0:
            self._episode_start()
        seed = int(torch.randint(0, 2**62, ()).item()) if mode == "sampling" else 0
        ain = action if mode == "evaluate" else None
        out = None
        if native is not None:
            out = native(td, logits, mword, self.temperature, self.tanh_clipping, ain, seed,
                         self._step_idx, self._status, self.key)
            if type(out) is int:
                nat.check_rc("decode_and_step", out)
        if out is None:
            out = fused(td, logits, mword, self.temperature, self.tanh_clipping, ain, seed,
                        self._step_idx, self._status, self.key)
        if out is None:
            if mode == "sampling":  # the seed draw above stands in for decode_step's
                self._seed_carry = seed
            return None
        self._step_idx += 1
        sel, logp = out
        self.actions.append(sel)
        self.logprobs.append(logp)
        return td

    def fast_stepper(self, env):
        """After a greedy loop's first fused step through the env's native glue: a closure
        ``f(td, logits, mask) -> bool`` for the following steps with everything
        ``step_env_fused`` decides per call bound once (the glue, mode word, temperature,
        clipping, status word, the action / log-probability lists).  It returns False,
        having done nothing, whenever the fused path does not apply to a call (the caller
        then takes ``step_env_fused``); None when there is nothing to bind."""
        cached = self._fused
        if (cached is None or cached[0] is not env or cached[1] is None or cached[2] is None
                or cached[3] != "greedy" or getattr(env, "_torchrl_mode", False)
                or self._status is None or self._step_idx == 0):
            return None
        native, mword = cached[2], cached[4]
        temp, clip, key, st = self.temperature, self.tanh_clipping, self.key, self._status
        ts = nat.torchstep()
        fs = ts.fast_step if ts is not None and not _NO_FAST_STEP else None
        if fs is not None and type(self.actions) is list and type(self.logprobs) is list:
            # the closure below in C (csrc/pycall/co_torchstep.cpp: fast_step): the same
            # calls in the same order, without a Python frame per step
            import functools

            return functools.partial(fs, native, TensorDict, mword, temp, clip, st, key,
                                     self.actions, self.logprobs, self, "_step_idx",
                                     nat.check_rc)
        push_a, push_l = self.actions.append, self.logprobs.append
        dget, td_type = dict.get, TensorDict

        def stepper(td, logits, mask):
            if type(td) is not td_type or mask is not dget(td, "action_mask"):
                return False
            out = native(td, logits, mword, temp, clip, None, 0, self._step_idx, st, key)
            if out is None:
                return False
            if type(out) is int:
                nat.check_rc("decode_and_step", out)
            self._step_idx += 1
            push_a(out[0])
            push_l(out[1])
            return True

        return stepper

    @abc.abstractmethod
    def _mode(self) -> str:
        raise NotImplementedError

    def _select_best(self, logprobs, actions, td, env):
        """``decoding.py:399-407``."""
        rewards = env.get_reward(td, actions)
        _, max_idxs = unbatchify(rewards, self.num_starts).max(dim=-1)
        actions = unbatchify_and_gather(actions, max_idxs, self.num_starts)
        logprobs = unbatchify_and_gather(logprobs, max_idxs, self.num_starts)
        td = unbatchify(td, self.num_starts)
        td = TensorDict({k: gather_by_index(v, max_idxs, dim=1) for k, v in td.items()},
                        batch_size=max_idxs.shape)
        return logprobs, actions, td, env


class Greedy(DecodingStrategy):
    name = "greedy"

    def _mode(self):
        return "greedy"


class Sampling(DecodingStrategy):
    name = "sampling"

    def _mode(self):
        return "sampling"


class MultiSampling(Sampling):
    """``decoding.py:421-472``: sampling (with ``multisample=True`` the td is batchified
    ``num_starts`` times in ``pre_decoder_hook`` without start-node selection)."""

    name = "multisampling"


class Evaluate(DecodingStrategy):
    name = "evaluate"

    def _mode(self):
        return "evaluate"


def _take_rows(td, idx):
    """``td[idx]`` for a TensorDict whose columns all lead with the batch dim: one device
    gather per column."""
    out = {}
    for k, v in td.items():
        if not torch.is_tensor(v) or v.dim() == 0:
            out[k] = v
        elif v.dim() == 1:
            out[k] = gather_by_index(v[:, None], idx, dim=0).squeeze(-1)
        else:
            out[k] = gather_by_index(v, idx, dim=0, squeeze=False)
    return TensorDict(out, batch_size=[idx.shape[0]])


class BeamSearch(DecodingStrategy):
    """``decoding.py:500-641``: beam width defaults to the env's number of starts; the
    first step takes the start nodes, then every step ranks the BW x N (beam, node)
    candidates per instance on the device (``co_beam_select``)."""

    name = "beam_search"

    def __init__(self, beam_width=None, select_best=True, **kwargs):
        kwargs["store_all_logp"] = True
        # the beams are ranked on the full log-probabilities: only the exact math ranks
        # them as the reference does (certification covers the argmax alone)
        if kwargs.get("decode_math") is None:
            kwargs["decode_math"] = "exact"
        super().__init__(**kwargs)
        self.beam_width = beam_width
        self.select_best = select_best
        self.parent_beam_logprobs = None
        self.beam_path = []

    def _mode(self):
        return "greedy"

    def pre_decoder_hook(self, td, env, action=None):
        """``decoding.py:526-556``."""
        if self.beam_width is None:
            self.beam_width = env.get_num_starts(td)
        assert self.beam_width > 1, "beam width must be larger than 1"
        if self.select_start_nodes_fn is not None:
            action = self.select_start_nodes_fn(td, env, self.beam_width)
        else:
            action = env.select_start_nodes(td, num_starts=self.beam_width)
        td = batchify(td, self.beam_width)
        td.set("action", action)
        td = env.step(td)["next"]
        logprobs = torch.zeros(td["action_mask"].shape, dtype=torch.float32, device=td.device)
        self.logprobs.append(logprobs)
        self.actions.append(action)
        self.parent_beam_logprobs = torch.zeros((action.shape[0], 1), dtype=torch.float32,
                                                device=td.device)
        self.beam_path.append(torch.zeros(action.shape[0], dtype=torch.int32, device=td.device))
        self.num_starts = self.beam_width
        return td, env, self.beam_width

    def step(self, logits, mask, td: TensorDict = None, action=None, env=None, **kwargs):
        """``decoding.py:327-369`` with ``_step`` = ``decoding.py:512-524`` + ``:611-641``."""
        if not self.mask_logits:
            mask = None
        if self._status is None:
            self._status = self._new_status(logits.device)
        _, _, full = decode_step(logits, mask, "greedy", self.temperature, self.tanh_clipping,
                                 return_full=True, top_k=self.top_k, top_p=self.top_p)
        e, n = full.shape
        b = e // self.beam_width
        dev = full.device
        sel = torch.empty(e, dtype=torch.int64, device=dev)
        parent = torch.empty(e, dtype=torch.int32, device=dev)
        rows = torch.empty(e, dtype=torch.int64, device=dev)
        score = torch.empty(e, dtype=torch.float32, device=dev)
        par = self.parent_beam_logprobs.reshape(e).contiguous()
        m = mask.contiguous() if mask is not None else None
        nat.call("co_beam_select", b, self.beam_width, n, nat.ptr(full), full.stride(0),
                 nat.ptr(par), nat.ptr(m), nat.ptr(sel), nat.ptr(parent), nat.ptr(rows),
                 nat.ptr(score), nat.ptr(self._status), nat.stream_of(full))
        self.parent_beam_logprobs = score[:, None]
        self.beam_path.append(parent)
        td = _take_rows(td, rows)
        logprobs = gather_by_index(full, rows, dim=0, squeeze=False)
        td.set(self.key, sel)
        self.actions.append(sel)
        self.logprobs.append(logprobs)
        return td

    def post_decoder_hook(self, td, env):
        """``decoding.py:558-565``."""
        if self._status is not None and int(self._status[0].item()) & nat.ST_INFEASIBLE:
            raise AssertionError("infeasible action selected")
        actions, logprobs = self._backtrack()
        if self.select_best:
            return self._select_best_beam(logprobs, actions, td, env)
        return logprobs, actions, td, env

    def _backtrack(self):
        """``decoding.py:567-599``: follow the parents back from the last step."""
        actions = torch.stack(self.actions, 1)
        logprobs = torch.stack(self.logprobs, 1)
        assert actions.size(1) == len(self.beam_path), "action idx shape and beam path shape dont match"
        cur_parent = self.beam_path[-1].long()
        seqs, lps = [actions[:, -1]], [logprobs[:, -1]]
        e = actions.size(0)
        b = e // self.beam_width
        seq = torch.arange(0, b, device=actions.device).repeat(self.beam_width)
        for k in reversed(range(len(self.beam_path) - 1)):
            idx = seq + cur_parent * b
            seqs.append(gather_by_index(actions[:, k].contiguous()[:, None], idx, dim=0).squeeze(-1))
            lps.append(gather_by_index(logprobs[:, k].contiguous(), idx, dim=0, squeeze=False))
            cur_parent = gather_by_index(self.beam_path[k].long()[:, None], idx, dim=0).squeeze(-1)
        return (torch.stack(list(reversed(seqs)), dim=1),
                torch.stack(list(reversed(lps)), dim=1))

    def _select_best_beam(self, logprobs, actions, td, env):
        """``decoding.py:601-609``."""
        e = logprobs.size(0)
        b = e // self.beam_width
        rewards = env.get_reward(td, actions)
        _, idx = torch.cat(rewards.unsqueeze(1).split(b), 1).max(1)
        flat_idx = torch.arange(b, device=rewards.device) + idx * b
        return (gather_by_index(logprobs, flat_idx, dim=0, squeeze=False),
                gather_by_index(actions, flat_idx, dim=0, squeeze=False),
                _take_rows(td, flat_idx), env)


def get_decoding_strategy(decoding_strategy, **config):
    """``decoding.py:17-36``."""
    registry = {"greedy": Greedy, "sampling": Sampling, "multistart_greedy": Greedy,
                "multistart_sampling": Sampling, "evaluate": Evaluate, "beam_search": BeamSearch,
                "multisampling": MultiSampling}
    if "multistart" in decoding_strategy:
        config["multistart"] = True
    return registry.get(decoding_strategy, Sampling)(**config)
