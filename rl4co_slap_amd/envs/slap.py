"""SLAP (storage location assignment) env + generator on the gfx950 kernels
(``rl4co/envs/warehousing/slap/``, the fork's warehouse env)."""
from __future__ import annotations

import numpy as np
import torch

from .. import _native as nat
from ..td import TensorDict, set_many
from .base import RL4COEnvBase
from .common import Generator, device_uniform


class SLAPGenerator(Generator):
    """``slap/generator.py:21-155``.

    Same keys, dtypes and RNG streams as the reference: ``freq`` from torch's global
    RNG (``Uniform(min_freq, max_freq)``, shape ``[*B, P, 1]``), picklists from
    numpy's global RNG in the reference's draw order (per instance, per order, one
    ``randint(0, P, size=K)``; drawn here as one ``randint(0, P, size=(B, O, K))``,
    which consumes the stream identically -- checked in the tests).  The aisle grid
    and the Manhattan matrices are computed vectorised instead of the reference's
    ``B x L`` Python loop (values identical: ``x = aisle * inter_aisle_dist`` in
    double rounded to f32, ``y = loc * inter_loc_dist``).
    """

    def __init__(self, n_products: int = 20, n_aisles: int = 10, n_locs: int = 10,
                 inter_loc_dist: float = 1, inter_aisle_dist: float = 2.4, min_freq: int = 1,
                 max_freq: int = 20, max_orders: int = 20, max_products_in_order: int = 5,
                 materialize_dist_mat: bool = True, device=None, device_rng: bool = False):
        self.n_products, self.n_aisles, self.n_locs = n_products, n_aisles, n_locs
        self.max_orders, self.max_products_in_order = max_orders, max_products_in_order
        self.inter_loc_dist, self.inter_aisle_dist = inter_loc_dist, inter_aisle_dist
        self.min_freq, self.max_freq = min_freq, max_freq
        self.freq_sampler = torch.distributions.Uniform(low=min_freq, high=max_freq)
        self.materialize_dist_mat = materialize_dist_mat
        # device generation: the deterministic columns (grid, distance
        # matrices, assignment) are written by co_slap_generate on the device; freq and the
        # picklists keep the host RNG streams and are copied (1.3 + 13 MB at B = 16,384)
        self.device = None if device is None else torch.device(device)
        # device_rng (throughput runs only): freq and picklists drawn on the device too
        # (co_uniform_fill / co_randint_fill, Philox keyed by one torch CPU draw) -- the
        # same distributions, not the reference's torch/numpy streams
        self.device_rng = device_rng

    @staticmethod
    def _get_distance_matrix(locs: torch.Tensor):
        """``generator.py:51-65`` (Manhattan)."""
        if locs.dtype not in (torch.float32, torch.float64):
            locs = locs.to(torch.float32)
        return torch.sum(torch.abs(locs[..., :, None, :] - locs[..., None, :, :]), dim=-1)

    def grid(self) -> torch.Tensor:
        total = self.n_aisles * self.n_locs
        i = np.arange(total)
        xy = np.stack([(i // self.n_locs) * self.inter_aisle_dist,
                       (i % self.n_locs) * self.inter_loc_dist], axis=-1)
        return torch.tensor(xy, dtype=torch.float64).to(torch.float32)

    def _generate(self, batch_size) -> TensorDict:
        if self.device is not None and self.device.type == "cuda":
            return self._generate_device(batch_size)
        freq = self.freq_sampler.sample((*batch_size, self.n_products, 1))
        g = self.grid()
        locs = g.expand(*batch_size, *g.shape).contiguous()
        dist1 = self._get_distance_matrix(g)
        depot = dist1[0].expand(*batch_size, dist1.shape[-1]).contiguous()
        picklist = torch.from_numpy(np.random.randint(
            0, self.n_products, size=(batch_size[0], self.max_orders, self.max_products_in_order)
        ).astype(np.int64))
        data = {"freq": freq, "locs": locs,
                "assignment": torch.full((*batch_size, self.n_products), -1, dtype=torch.int),
                "picklist": picklist, "depot_loc_dist": depot}
        if self.materialize_dist_mat:
            data["dist_mat"] = dist1.expand(*batch_size, *dist1.shape).contiguous()
        return TensorDict(data, batch_size=batch_size)

    def _generate_device(self, batch_size) -> TensorDict:
        dev = self.device
        b, L, P = batch_size[0], self.n_aisles * self.n_locs, self.n_products
        if self.device_rng:
            freq = device_uniform(self.freq_sampler, (*batch_size, P, 1), dev)
            picklist = torch.empty((b, self.max_orders, self.max_products_in_order),
                                   dtype=torch.int64, device=dev)
            seed = int(torch.randint(0, 2 ** 62, (), dtype=torch.int64))
            nat.call("co_randint_fill", nat.ptr(picklist), picklist.numel(), 0, P, seed, 0,
                     nat.stream_of(picklist))
        else:
            freq = self.freq_sampler.sample((*batch_size, P, 1))  # host path's draw order
            picklist = torch.from_numpy(np.random.randint(
                0, P, size=(b, self.max_orders, self.max_products_in_order)).astype(np.int64))
        locs = torch.empty((b, L, 2), dtype=torch.float32, device=dev)
        depot = torch.empty((b, L), dtype=torch.float32, device=dev)
        assign = torch.empty((b, P), dtype=torch.int32, device=dev)
        dist = (torch.empty((b, L, L), dtype=torch.float32, device=dev)
                if self.materialize_dist_mat else None)
        nat.call("co_slap_generate", b, self.n_aisles, self.n_locs, float(self.inter_aisle_dist),
                 float(self.inter_loc_dist), P, nat.ptr(locs), nat.ptr(depot), nat.ptr(dist),
                 nat.ptr(assign), nat.stream_of(locs))
        data = {"freq": freq.to(dev, non_blocking=True), "locs": locs, "assignment": assign,
                "picklist": picklist.to(dev, non_blocking=True), "depot_loc_dist": depot}
        if dist is not None:
            data["dist_mat"] = dist
        return TensorDict(data, batch_size=batch_size)


class SLAPEnv(RL4COEnvBase):
    """``slap/env.py:17-152``."""

    name = "slap"

    def __init__(self, generator: SLAPGenerator = None, generator_params: dict = {},
                 check_solution=False, **kwargs):
        super().__init__(**kwargs)
        self.generator = generator if generator is not None else SLAPGenerator(**generator_params)
        self.check_solution = check_solution

    def _reset(self, td=None, batch_size=None) -> TensorDict:
        """``slap/env.py:95-129`` in one kernel (``to_choose``/``ratio`` on the device),
        which also writes the ``done`` / ``terminated`` zeros ``reset`` adds.  On a device
        stand-in TensorDict the step glue does it in one call (one storage for the seven
        outputs, set straight into ``td``)."""
        ts = nat.torchstep() if type(td) is TensorDict else None
        if ts is not None:
            r = ts.slap_reset_td(self._lb_attr, td)
            if type(r) is int:
                nat.check_rc("co_slap_reset", r)
            if r is not None:
                return td
        assignment = td["assignment"]
        nat.require_device(assignment)
        b = assignment.shape[0]
        p = td["freq"].shape[-2]
        l = td["locs"].shape[1]
        dev = assignment.device
        mask = torch.empty((b, l), dtype=torch.bool, device=dev)
        to_choose = torch.empty((b, p), dtype=torch.float32, device=dev)
        i = torch.empty((b, 1), dtype=torch.int64, device=dev)
        reward = torch.empty((b, 1), dtype=torch.float32, device=dev)
        ratio = torch.empty(td["depot_loc_dist"].shape, dtype=torch.float32, device=dev)
        dt = torch.empty((2, b, 1), dtype=torch.bool, device=dev)  # done, terminated
        nat.call("co_slap_reset", b, l, p, nat.ptr(mask), nat.ptr(to_choose), nat.ptr(i),
                 nat.ptr(reward), nat.ptr(ratio), nat.ptr(dt[0]), nat.ptr(dt[1]),
                 nat.stream_of(assignment))
        self._remember_lb(i, p)  # done = (i == P-1) before the step (slap/env.py:57)
        self._remember_i(i, 0)
        return TensorDict({"assignment": assignment, "to_choose": to_choose, "i": i,
                           "ratio": ratio, "action_mask": mask, "reward": reward,
                           "done": dt[0], "terminated": dt[1]}, batch_size=batch_size)

    def _step(self, td: TensorDict) -> TensorDict:
        """``slap/env.py:38-93``: one kernel replaces the clone + advanced-index write +
        the per-batch Python loop; ``to_choose`` shrinks as a zero-copy view."""
        action, tc, assign, mask, i = (td["action"], td["to_choose"], td["assignment"],
                                       td["action_mask"], td["i"])
        nat.require_device(action, tc, assign, mask, i)
        if action.dtype != torch.int64:
            action = action.long()
        action, assign, mask, i = (x.contiguous() for x in (action, assign, mask, i))
        b, l = mask.shape
        p = td["freq"].shape[-2]
        dev = mask.device
        s = nat.stream_of(mask)
        assign_out = self._out(assign.shape, assign.dtype, dev, s)
        mask_out = self._out(mask.shape, mask.dtype, dev, s)
        i_out = self._out(i.shape, i.dtype, dev, s)
        done = self._out((b, 1), torch.bool, dev, s)
        reward = self._out((b, 1), torch.bool, dev, s)
        nat.call("co_slap_step", b, l, p, nat.ptr(action), nat.ptr(tc), tc.stride(0),
                 nat.ptr(assign), nat.ptr(assign_out), nat.ptr(mask), nat.ptr(mask_out),
                 nat.ptr(i), nat.ptr(i_out), nat.ptr(done), nat.ptr(reward), None, s)
        self._step_records(td["i"], i_out, done, p)
        td.update({"assignment": assign_out, "to_choose": tc[..., 1:], "action_mask": mask_out,
                   "i": i_out, "reward": reward, "done": done})
        return td

    def _step_records(self, i_in, i_out, done, p):
        """Host-side knowledge carried to a step's outputs: the done lower bound, and --
        when every entry of ``i`` is known to hold one value (reset: 0; each step adds 1
        to every row, ``slap/env.py:57-58``) -- that value, and then ``done = (i == P-1)``
        is uniform too (recorded on ``done``: ``poll_done`` answers without a read)."""
        lb = self._known_lb(i_in)
        if lb is not None:
            self._remember_lb(i_out, lb - 1)
        k = self._known_i(i_in)
        if k is not None:
            self._remember_i(i_out, k + 1)
            self._remember_i(done, int(k == p - 1))

    def poll_done(self, td):
        """``td["done"].all()``: known on the host when the step that produced ``done``
        knew ``i`` (see ``_step_records``), else one device read."""
        d = td.get_raw("done") if hasattr(td, "get_raw") else td["done"]
        k = self._known_i(d) if isinstance(d, torch.Tensor) else None
        if k is not None:
            return bool(k), 1
        return super().poll_done(td)

    def native_decode_and_step(self):
        """``decode_and_step``'s native call for a decoding strategy's loop (the step glue
        ``csrc/pycall/co_torchstep.cpp``: slap_step_td): ``f(td, logits, mode, temperature,
        tanh_clipping, action_in, seed, offset, status, key)`` returning ``(action, logp)``,
        an error code, or None (then call ``decode_and_step``); None when the glue is
        unavailable."""
        ts = nat.torchstep()
        if ts is None:
            return None
        import functools

        return functools.partial(ts.slap_step_td, self._lb_attr)

    def decode_and_step(self, td, logits, mode, temperature, tanh_clipping, action_in, seed,
                        offset, status, key="action"):
        """``DecodingStrategy.step`` + ``_step`` (``decoding.py:327-369``,
        ``slap/env.py:38-93``) in one ``co_slap_decode_step`` launch: the same selection,
        log-probability, RNG use and state (assignment row written out of place, the
        mask minus the action, ``done = i == P-1``, ``to_choose`` shrunk as a view) as the
        two calls.  Returns ``(action, logp)``, or None when it does not apply (CPU
        tensors, non-f32 logits, rows past the register row engines, no product left)."""
        mask, i, tc, assign = td["action_mask"], td["i"], td["to_choose"], td["assignment"]
        dev = logits.device
        if dev.type != "cuda" or any(x.device != dev for x in (mask, i, tc, assign)):
            return None
        if logits.dtype != torch.float32 or logits.dim() != 2 or logits.stride(-1) != 1:
            return None
        b, l = mask.shape
        if (logits.shape != (b, l) or l > 2048 or assign.dtype != torch.int32 or tc.dim() != 2
                or tc.shape[-1] == 0 or tc.dtype != torch.float32):
            return None
        p = td["freq"].shape[-2]
        # the operands the kernel indexes: i [b] int64, assignment [b, P] (it writes r*P + c)
        if (i.dtype != torch.int64 or i.numel() != b or assign.dim() != 2
                or tuple(assign.shape) != (b, p) or tc.shape[0] != b):
            return None
        if action_in is not None and action_in.numel() != b:
            return None
        m, i, assign = mask.contiguous(), i.contiguous(), assign.contiguous()
        ain = action_in.long().contiguous() if action_in is not None else None
        s = nat.stream_of(m)
        # the decoding strategy keeps every action and log-probability: never pooled
        act = torch.empty(b, dtype=torch.int64, device=dev)
        logp = torch.empty(b, dtype=torch.float32, device=dev)
        assign_out = self._out(assign.shape, assign.dtype, dev, s)
        mask_out = self._out(m.shape, m.dtype, dev, s)
        i_out = self._out(i.shape, i.dtype, dev, s)
        done = self._out((b, 1), torch.bool, dev, s)
        reward = self._out((b, 1), torch.bool, dev, s)
        nat.call("co_slap_decode_step", b, l, p, nat.ptr(logits), logits.stride(0), nat.ptr(m),
                 float(tanh_clipping), float(temperature), mode, nat.ptr(ain), nat.ptr(act),
                 nat.ptr(logp), seed, offset, nat.ptr(tc), tc.stride(0), nat.ptr(assign),
                 nat.ptr(assign_out), nat.ptr(mask_out), nat.ptr(i), nat.ptr(i_out),
                 nat.ptr(done), nat.ptr(reward), None, nat.ptr(status), s)
        self._step_records(td["i"], i_out, done, p)
        sel = action_in if action_in is not None else act
        set_many(td, {key: sel, "assignment": assign_out, "to_choose": tc[..., 1:],
                      "action_mask": mask_out, "i": i_out, "reward": reward, "done": done})
        return sel, logp

    def _get_reward(self, td, actions=None, check: bool = False) -> torch.Tensor:
        """``slap/env.py:131-143``: sum over orders of the closed pick tour (``actions``
        is ignored, as in the reference)."""
        if check:
            raise NotImplementedError  # base.py:209-213: SLAP has no validity check
        assign, picklist, locs = td["assignment"], td["picklist"], td["locs"]
        nat.require_device(assign, picklist, locs)
        assign, picklist, locs = assign.contiguous(), picklist.contiguous(), locs.contiguous()
        b, o, k = picklist.shape
        reward = torch.empty(b, dtype=torch.float32, device=locs.device)
        status = self.status_word(locs.device)
        nat.call("co_slap_reward", b, locs.shape[1], assign.shape[1], o, k, nat.ptr(assign),
                 nat.ptr(picklist), nat.ptr(locs), nat.ptr(reward), nat.ptr(status),
                 nat.stream_of(locs))
        self.raise_for_status(status, [(nat.ST_INDEX_RANGE, IndexError,
                                        "index out of range in SLAP reward gather")])
        return reward

    def get_action_mask(self, td):
        return td["action_mask"]

    def min_steps_to_done(self, td) -> int:
        """done = (i == P - 1) at the step (``slap/env.py:57``): P - i steps."""
        return self._known_lb(td.get_raw("i") if hasattr(td, "get_raw") else td["i"]) or 0
