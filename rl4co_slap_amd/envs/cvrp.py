"""CVRP env + generator on the gfx950 kernels (``rl4co/envs/routing/cvrp/``)."""
from __future__ import annotations

from typing import Callable, Union

import torch
from torch.distributions import Uniform

from .. import _native as nat
from ..td import TensorDict, set_many
from .base import RL4COEnvBase
from .common import Generator, device_uniform, get_sampler

# cvrp/generator.py:15-30 (Kool et al. 2019, Hottung et al. 2022, Kim et al. 2023)
CAPACITIES = {10: 20.0, 15: 25.0, 20: 30.0, 30: 33.0, 40: 37.0, 50: 40.0, 60: 43.0, 75: 45.0,
              100: 50.0, 125: 55.0, 150: 60.0, 200: 70.0, 500: 100.0, 1000: 150.0}


class CVRPGenerator(Generator):
    """``cvrp/generator.py:33-143``: depot sampled with the customers when no depot
    distribution is given; ``demand = (Uniform(min-1, max-1).int() + 1) / capacity``.
    With ``device="cuda"`` Uniform samplers draw on the GPU (``common.device_uniform``)."""

    def __init__(self, num_loc: int = 20, min_loc: float = 0.0, max_loc: float = 1.0,
                 loc_distribution: Union[int, float, str, type, Callable] = Uniform,
                 depot_distribution: Union[int, float, str, type, Callable] = None,
                 min_demand: int = 1, max_demand: int = 10,
                 demand_distribution: Union[int, float, type, Callable] = Uniform,
                 vehicle_capacity: float = 1.0, capacity: float = None, **kwargs):
        self.num_loc, self.min_loc, self.max_loc = num_loc, min_loc, max_loc
        self.min_demand, self.max_demand = min_demand, max_demand
        self.vehicle_capacity = vehicle_capacity
        self.device = kwargs.get("device")
        self.loc_sampler = kwargs.get("loc_sampler") or get_sampler(
            "loc", loc_distribution, min_loc, max_loc, **kwargs)
        if kwargs.get("depot_sampler") is not None:
            self.depot_sampler = kwargs["depot_sampler"]
        else:
            self.depot_sampler = get_sampler("depot", depot_distribution, min_loc, max_loc, **kwargs) \
                if depot_distribution is not None else None
        self.demand_sampler = kwargs.get("demand_sampler") or get_sampler(
            "demand", demand_distribution, min_demand - 1, max_demand - 1, **kwargs)
        if capacity is None:
            capacity = CAPACITIES.get(num_loc)
        if capacity is None:
            capacity = CAPACITIES[min(CAPACITIES, key=lambda x: abs(x - num_loc))]
        self.capacity = capacity

    def _sample(self, sampler, shape, capacity=None):
        out = device_uniform(sampler, shape, self.device, capacity) if self.device else None
        if out is not None:
            return out
        out = sampler.sample(shape).to(self.device)
        return out if capacity is None else (out.int() + 1).float() / capacity

    def _generate(self, batch_size) -> TensorDict:
        if self.device:
            if self.depot_sampler is not None:
                depot = self._sample(self.depot_sampler, (*batch_size, 2))
                locs = self._sample(self.loc_sampler, (*batch_size, self.num_loc, 2))
            else:
                locs = self._sample(self.loc_sampler, (*batch_size, self.num_loc + 1, 2))
                depot, locs = locs[..., 0, :], locs[..., 1:, :]
            demand = self._sample(self.demand_sampler, (*batch_size, self.num_loc), self.capacity)
            capacity = torch.full((*batch_size, 1), self.capacity, device=demand.device)
            return TensorDict({"locs": locs, "depot": depot, "demand": demand,
                               "capacity": capacity}, batch_size=batch_size)
        if self.depot_sampler is not None:
            depot = self.depot_sampler.sample((*batch_size, 2))
            locs = self.loc_sampler.sample((*batch_size, self.num_loc, 2))
        else:
            locs = self.loc_sampler.sample((*batch_size, self.num_loc + 1, 2))
            depot, locs = locs[..., 0, :], locs[..., 1:, :]
        demand = self.demand_sampler.sample((*batch_size, self.num_loc))
        demand = (demand.int() + 1).float()
        capacity = torch.full((*batch_size, 1), self.capacity)
        return TensorDict({"locs": locs, "depot": depot, "demand": demand / self.capacity,
                           "capacity": capacity}, batch_size=batch_size)


class CVRPEnv(RL4COEnvBase):
    """``cvrp/env.py:29-199``: fused step + mask, fused reward + validity."""

    name = "cvrp"

    def __init__(self, generator: CVRPGenerator = None, generator_params: dict = {}, **kwargs):
        super().__init__(**kwargs)
        self.generator = generator if generator is not None else CVRPGenerator(**generator_params)

    def _reset(self, td=None, batch_size=None) -> TensorDict:
        """``cvrp/env.py:107-135``: cat(depot, locs), state zeros, capacity fill and the
        initial action mask in one kernel."""
        depot, locs, demand = td["depot"], td["locs"], td["demand"]
        nat.require_device(depot, locs, demand)
        depot, locs, demand = depot.contiguous(), locs.contiguous(), demand.contiguous()
        b, n = demand.shape
        dev = demand.device
        locs_out = torch.empty((b, n + 1, 2), dtype=torch.float32, device=dev)
        cur = torch.empty((b, 1), dtype=torch.int64, device=dev)
        used = torch.empty((b, 1), dtype=torch.float32, device=dev)
        vcap = torch.empty((b, 1), dtype=torch.float32, device=dev)
        visited = torch.empty((b, n + 1), dtype=torch.uint8, device=dev)
        mask = torch.empty((b, n + 1), dtype=torch.bool, device=dev)
        nat.call("co_cvrp_reset", b, n, nat.ptr(depot), nat.ptr(locs), nat.ptr(demand),
                 float(self.generator.vehicle_capacity), nat.ptr(locs_out), nat.ptr(cur),
                 nat.ptr(used), nat.ptr(vcap), nat.ptr(visited), nat.ptr(mask),
                 nat.stream_of(demand))
        self._remember_lb(visited, n + 1)  # done = all N+1 nodes visited (cvrp/env.py:95)
        return TensorDict({"locs": locs_out, "demand": demand, "current_node": cur,
                           "used_capacity": used, "vehicle_capacity": vcap, "visited": visited,
                           "action_mask": mask}, batch_size=batch_size)

    def _step(self, td: TensorDict) -> TensorDict:
        """``cvrp/env.py:73-105`` + ``get_action_mask`` (``:137-149``) in one kernel."""
        action = td["action"]
        demand, used, vcap, visited = (td["demand"], td["used_capacity"], td["vehicle_capacity"],
                                       td["visited"])
        ts = nat.torchstep()
        r = ts.cvrp_step(action, demand, used, vcap, visited) if ts is not None else None
        if r is not None:  # output allocation + launch in one native call
            if type(r) is int:
                nat.check_rc("co_cvrp_step", r)
            used_out, visited_out, cur, done, reward, mask = r
            return self._after_step(td, used_out, visited_out, cur, done, reward, mask)
        nat.require_device(action, demand, used, vcap, visited)
        if action.dtype != torch.int64:
            action = action.long()
        action, demand, used, vcap, visited = (x.contiguous() for x in
                                               (action, demand, used, vcap, visited))
        b, n = demand.shape
        dev = demand.device
        s = nat.stream_of(demand)
        used_out = self._out(used.shape, used.dtype, dev, s)
        visited_out = self._out(visited.shape, visited.dtype, dev, s)
        cur = self._out((b, 1), torch.int64, dev, s)
        done = self._out((b,), torch.bool, dev, s)
        reward = self._out((b,), torch.bool, dev, s)
        mask = self._out((b, n + 1), torch.bool, dev, s)
        nat.call("co_cvrp_step", b, n, nat.ptr(action), nat.ptr(demand), nat.ptr(used),
                 nat.ptr(used_out), nat.ptr(vcap), nat.ptr(visited), nat.ptr(visited_out),
                 nat.ptr(cur), nat.ptr(done), nat.ptr(reward), nat.ptr(mask), None, None, s)
        return self._after_step(td, used_out, visited_out, cur, done, reward, mask)

    def _after_step(self, td, used_out, visited_out, cur, done, reward, mask):
        lb = self._known_lb(td["visited"])
        if lb is not None:  # a step marks at most one more node visited
            self._remember_lb(visited_out, lb - 1)
        set_many(td, {"current_node": cur, "used_capacity": used_out, "visited": visited_out,
                      "reward": reward, "done": done, "action_mask": mask})
        return td

    def native_decode_and_step(self):
        """``decode_and_step``'s native call for a decoding strategy's loop (the step glue
        ``csrc/pycall/co_torchstep.cpp``: cvrp_step_td): ``f(td, logits, mode, temperature,
        tanh_clipping, action_in, seed, offset, status, key)`` returning ``(action, logp)``,
        an error code, or None (then call ``decode_and_step``); None when the glue is
        unavailable."""
        ts = nat.torchstep()
        if ts is None:
            return None
        import functools

        return functools.partial(ts.cvrp_step_td, self._lb_attr)

    def decode_and_step(self, td, logits, mode, temperature, tanh_clipping, action_in, seed,
                        offset, status, key="action"):
        """``DecodingStrategy.step`` + ``_step`` (``decoding.py:327-369``,
        ``cvrp/env.py:73-149``) in one ``co_cvrp_decode_step`` launch: the same selection,
        log-probability, RNG use and state (used / vehicle capacity, visited, current node,
        done, the recomputed action mask) as the two calls.  Returns ``(action, logp)``, or
        None when it does not apply (CPU tensors, non-f32 logits, long rows)."""
        mask, demand, used, vcap, visited = (td["action_mask"], td["demand"],
                                             td["used_capacity"], td["vehicle_capacity"],
                                             td["visited"])
        dev = logits.device
        if dev.type != "cuda" or any(x.device != dev for x in (mask, demand, used, vcap, visited)):
            return None
        if logits.dtype != torch.float32 or logits.dim() != 2 or logits.stride(-1) != 1:
            return None
        b, n = demand.shape
        if (logits.shape != (b, n + 1) or mask.shape != (b, n + 1) or n + 1 > 2048
                or visited.dtype != torch.uint8 or demand.dtype != torch.float32
                or used.dtype != torch.float32 or vcap.dtype != torch.float32
                or used.numel() != b or vcap.numel() != b):
            return None
        m, demand, used, vcap, visited = (x.contiguous() for x in (mask, demand, used, vcap, visited))
        ain = action_in.long().contiguous() if action_in is not None else None
        s = nat.stream_of(m)
        act = torch.empty(b, dtype=torch.int64, device=dev)  # kept by the strategy
        logp = torch.empty(b, dtype=torch.float32, device=dev)
        used_out = self._out(used.shape, used.dtype, dev, s)
        visited_out = self._out(visited.shape, visited.dtype, dev, s)
        cur = self._out((b, 1), torch.int64, dev, s)
        done = self._out((b,), torch.bool, dev, s)
        reward = self._out((b,), torch.bool, dev, s)
        mask_out = self._out((b, n + 1), torch.bool, dev, s)
        nat.call("co_cvrp_decode_step", b, n, nat.ptr(logits), logits.stride(0), nat.ptr(m),
                 float(tanh_clipping), float(temperature), mode, nat.ptr(ain), nat.ptr(act),
                 nat.ptr(logp), seed, offset, nat.ptr(demand), nat.ptr(used), nat.ptr(used_out),
                 nat.ptr(vcap), nat.ptr(visited), nat.ptr(visited_out), nat.ptr(cur),
                 nat.ptr(done), nat.ptr(reward), nat.ptr(mask_out), None, nat.ptr(status), s)
        sel = action_in if action_in is not None else act
        set_many(td, {key: sel})
        self._after_step(td, used_out, visited_out, cur, done, reward, mask_out)
        return sel, logp

    def poll_done(self, td):
        """``done = visited.sum(-1) == N+1`` (``cvrp/env.py:92``) and a step adds at most one
        to a row's sum: the largest row deficit d (``co_row_deficit_max``, one device read
        like ``done.all()``) means no instance set is all done for d - 1 more steps."""
        vis = td["visited"]
        if vis.device.type != "cuda" or vis.dim() != 2 or vis.stride(1) != 1 \
                or vis.dtype != torch.uint8:
            return super().poll_done(td)
        w = getattr(self, "_deficit_word", None)
        if w is None or w.device != vis.device:
            w = self._deficit_word = torch.zeros(1, dtype=torch.int32, device=vis.device)
        nat.call("co_row_deficit_max", nat.ptr(vis), vis.shape[0], vis.shape[1], vis.stride(0),
                 nat.ptr(w), nat.stream_of(vis))
        d = int(w.item())
        if d >= 1:
            return False, d
        return bool(td["done"].all()), 1

    def min_steps_to_done(self, td) -> int:
        """done = every node incl. the depot visited; a step visits one node."""
        return self._known_lb(td.get_raw("visited") if hasattr(td, "get_raw")
                              else td["visited"]) or 0

    @staticmethod
    def get_action_mask(td: TensorDict) -> torch.Tensor:
        """``cvrp/env.py:137-149``."""
        demand, used, vcap, visited, cur = (td["demand"], td["used_capacity"],
                                            td["vehicle_capacity"], td["visited"],
                                            td["current_node"])
        nat.require_device(demand, used, vcap, visited, cur)
        demand, used, vcap, visited, cur = (x.contiguous() for x in (demand, used, vcap, visited, cur))
        b, n = demand.shape
        mask = torch.empty((b, n + 1), dtype=torch.bool, device=demand.device)
        nat.call("co_cvrp_action_mask", b, n, nat.ptr(demand), nat.ptr(used), nat.ptr(vcap),
                 nat.ptr(visited), nat.ptr(cur), nat.ptr(mask), nat.stream_of(demand))
        return mask

    def _get_reward(self, td, actions, check: bool = False) -> torch.Tensor:
        """``cvrp/env.py:151-190``: -tour length through the depot, fused with the
        validity check and the sequential capacity scan."""
        locs, demand, vcap = td["locs"], td["demand"], td["vehicle_capacity"]
        nat.require_device(locs, actions, demand, vcap)
        locs, demand, vcap = locs.contiguous(), demand.contiguous(), vcap.contiguous()
        if actions.dtype != torch.int64:
            actions = actions.long()
        b, t = actions.shape
        n = demand.shape[-1]
        reward = torch.empty(b, dtype=torch.float32, device=locs.device)
        status = self.status_word(locs.device)
        nat.call("co_cvrp_reward", b, n, t, nat.ptr(locs), nat.ptr(actions), actions.stride(0),
                 actions.stride(1), nat.ptr(demand), nat.ptr(vcap), int(check), nat.ptr(reward),
                 nat.ptr(status), nat.stream_of(locs))
        msgs = [(nat.ST_INVALID_TOUR, AssertionError, "Invalid tour"),
                (nat.ST_OVER_CAPACITY, AssertionError, "Used more than capacity")] if check else []
        msgs.append((nat.ST_INDEX_RANGE, RuntimeError, "index out of range in gather (actions)"))
        self.raise_for_status(status, msgs)
        return reward

    def check_solution_validity(self, td, actions):
        """``cvrp/env.py:162-190``."""
        self._get_reward(td, actions, check=True)

    @staticmethod
    def load_data(fpath, batch_size=[]):
        """``cvrp/env.py:192-199``: normalise demand by capacity."""
        td = RL4COEnvBase.load_data(fpath, batch_size)
        td.set("demand", td["demand"] / td["capacity"][:, None])
        return td
