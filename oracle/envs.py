"""TSP / CVRP / SLAP environments restated on CPU (test infrastructure only).

Each method cites the reference lines it follows.  Dtypes, shapes, op order and
the fork's quirks are kept: the batch-wide ``i.all() == 0`` first-node test, the
bool ``reward`` written by ``_step``, the double TSP validity check, SLAP's
per-batch Python loop and its shrinking ``to_choose``.
"""
from __future__ import annotations

import numpy as np
import torch
from torch.distributions import Uniform

from .ops import gather_by_index, get_num_starts, get_tour_length, select_start_nodes
from .td import TD

# rl4co/envs/routing/cvrp/generator.py:15-30
CAPACITIES = {10: 20.0, 15: 25.0, 20: 30.0, 30: 33.0, 40: 37.0, 50: 40.0, 60: 43.0,
              75: 45.0, 100: 50.0, 125: 55.0, 150: 60.0, 200: 70.0, 500: 100.0,
              1000: 150.0}


class _EnvBase:
    """``RL4COEnvBase`` plumbing (``rl4co/envs/common/base.py:45-143,182-207``)."""

    name = "base"

    def __init__(self, check_solution=True, seed=None):
        self.check_solution = check_solution
        if seed is None:  # base.py:117-118
            seed = torch.empty((), dtype=torch.int64).random_().item()
        torch.manual_seed(seed)  # base.py:288-291 (global RNG)

    def reset(self, td=None, batch_size=None):
        # base.py:135-143 + TorchRL EnvBase.reset merge semantics (see td.py)
        if batch_size is None:
            batch_size = td.batch_size
        if td is None or td.is_empty():
            td = self.generate(batch_size)
        batch_size = [batch_size] if isinstance(batch_size, int) else list(batch_size)
        out = self._reset(td, batch_size)
        td.update(out)
        td["done"] = torch.zeros((*batch_size, 1), dtype=torch.bool)
        td["terminated"] = torch.zeros((*batch_size, 1), dtype=torch.bool)
        return td

    def step(self, td):  # base.py:121-130 (non-torchrl mode)
        return {"next": self._step(td)}

    def get_reward(self, td, actions):  # base.py:182-188
        if self.check_solution:
            self.check_solution_validity(td, actions)
        return self._get_reward(td, actions)

    def get_num_starts(self, td):  # base.py:203-204
        return get_num_starts(td, self.name)

    def select_start_nodes(self, td, num_starts):  # base.py:206-207
        num_loc = getattr(self, "num_loc", 0xFFFFFFFF)
        return select_start_nodes(td, self.name, num_loc, num_starts)

    def check_solution_validity(self, td, actions):
        raise NotImplementedError


class TSPOracle(_EnvBase):
    name = "tsp"

    def __init__(self, num_loc=20, min_loc=0.0, max_loc=1.0, **kw):
        super().__init__(**kw)
        self.num_loc, self.min_loc, self.max_loc = num_loc, min_loc, max_loc
        self.loc_sampler = Uniform(low=min_loc, high=max_loc)  # common/utils.py:152-153

    def generate(self, batch_size):  # tsp/generator.py:51-60
        batch_size = [batch_size] if isinstance(batch_size, int) else list(batch_size)
        locs = self.loc_sampler.sample((*batch_size, self.num_loc, 2))
        return TD({"locs": locs}, batch_size)

    def _reset(self, td, batch_size):  # tsp/env.py:95-120
        n = td["locs"].shape[-2]
        cur = torch.zeros(batch_size, dtype=torch.int64)
        return TD({
            "locs": td["locs"],
            "first_node": cur,
            "current_node": cur,
            "i": torch.zeros((*batch_size, 1), dtype=torch.int64),
            "action_mask": torch.ones((*batch_size, n), dtype=torch.bool),
            "reward": torch.zeros((*batch_size, 1), dtype=torch.float32),
        }, batch_size)

    @staticmethod
    def _step(td):  # tsp/env.py:67-93
        cur = td["action"]
        first = cur if td["i"].all() == 0 else td["first_node"]
        avail = td["action_mask"].scatter(-1, cur.unsqueeze(-1).expand_as(td["action_mask"]), 0)
        done = torch.sum(avail, dim=-1) == 0
        td.update({"first_node": first, "current_node": cur, "i": td["i"] + 1,
                   "action_mask": avail, "reward": torch.zeros_like(done), "done": done})
        return td

    def _get_reward(self, td, actions):  # tsp/env.py:157-163
        if self.check_solution:
            self.check_solution_validity(td, actions)
        return -get_tour_length(gather_by_index(td["locs"], actions))

    @staticmethod
    def check_solution_validity(td, actions):  # tsp/env.py:165-173
        ar = torch.arange(actions.size(1), dtype=actions.dtype).view(1, -1).expand_as(actions)
        assert (ar == actions.data.sort(1)[0]).all(), "Invalid tour"


class CVRPOracle(_EnvBase):
    name = "cvrp"

    def __init__(self, num_loc=20, min_loc=0.0, max_loc=1.0, min_demand=1, max_demand=10,
                 vehicle_capacity=1.0, capacity=None, **kw):
        super().__init__(**kw)
        self.num_loc, self.vehicle_capacity = num_loc, vehicle_capacity
        self.loc_sampler = Uniform(low=min_loc, high=max_loc)
        self.demand_sampler = Uniform(low=min_demand - 1, high=max_demand - 1)  # generator.py:96-98
        if capacity is None:  # generator.py:101-113
            capacity = CAPACITIES.get(num_loc)
            if capacity is None:
                capacity = CAPACITIES[min(CAPACITIES, key=lambda x: abs(x - num_loc))]
        self.capacity = capacity

    def generate(self, batch_size):  # cvrp/generator.py:116-143 (depot sampled with locs)
        batch_size = [batch_size] if isinstance(batch_size, int) else list(batch_size)
        locs = self.loc_sampler.sample((*batch_size, self.num_loc + 1, 2))
        depot, locs = locs[..., 0, :], locs[..., 1:, :]
        demand = self.demand_sampler.sample((*batch_size, self.num_loc))
        demand = (demand.int() + 1).float()
        return TD({"locs": locs, "depot": depot, "demand": demand / self.capacity,
                   "capacity": torch.full((*batch_size, 1), self.capacity)}, batch_size)

    def _reset(self, td, batch_size):  # cvrp/env.py:107-135
        out = TD({
            "locs": torch.cat((td["depot"][:, None, :], td["locs"]), -2),
            "demand": td["demand"],
            "current_node": torch.zeros(*batch_size, 1, dtype=torch.long),
            "used_capacity": torch.zeros((*batch_size, 1)),
            "vehicle_capacity": torch.full((*batch_size, 1), self.vehicle_capacity),
            "visited": torch.zeros((*batch_size, td["locs"].shape[-2] + 1), dtype=torch.uint8),
        }, batch_size)
        out["action_mask"] = self.get_action_mask(out)
        return out

    @staticmethod
    def get_action_mask(td):  # cvrp/env.py:137-149
        exceeds = td["demand"] + td["used_capacity"] > td["vehicle_capacity"]
        mask_loc = td["visited"][..., 1:].to(exceeds.dtype) | exceeds
        mask_depot = (td["current_node"] == 0) & ((mask_loc == 0).int().sum(-1) > 0)[:, None]
        return ~torch.cat((mask_depot, mask_loc), -1)

    def _step(self, td):  # cvrp/env.py:73-105
        cur = td["action"][:, None]
        n_loc = td["demand"].size(-1)
        d = gather_by_index(td["demand"], torch.clamp(cur - 1, 0, n_loc - 1), squeeze=False)
        used = (td["used_capacity"] + d) * (cur != 0).float()
        visited = td["visited"].scatter(-1, cur, 1)
        done = visited.sum(-1) == visited.size(-1)
        td.update({"current_node": cur, "used_capacity": used, "visited": visited,
                   "reward": torch.zeros_like(done), "done": done})
        td["action_mask"] = self.get_action_mask(td)
        return td

    def _get_reward(self, td, actions):  # cvrp/env.py:151-160
        ordered = torch.cat([td["locs"][..., 0:1, :], gather_by_index(td["locs"], actions)], dim=1)
        return -get_tour_length(ordered)

    @staticmethod
    def check_solution_validity(td, actions):  # cvrp/env.py:162-190
        b, n = td["demand"].size()
        sp = actions.data.sort(1)[0]
        ok = (torch.arange(1, n + 1, dtype=sp.dtype).view(1, -1).expand(b, n) == sp[:, -n:]).all()
        assert ok and (sp[:, :-n] == 0).all(), "Invalid tour"
        dwd = torch.cat((-td["vehicle_capacity"], td["demand"]), 1)
        d = dwd.gather(1, actions)
        used = torch.zeros_like(td["demand"][:, 0])
        for t in range(actions.size(1)):
            used += d[:, t]
            used[used < 0] = 0
            # [B] vs [B,1] broadcasts to [B,B] exactly as the reference does
            assert (used <= td["vehicle_capacity"] + 1e-5).all(), "Used more than capacity"


class SLAPOracle(_EnvBase):
    name = "slap"

    def __init__(self, n_products=20, n_aisles=10, n_locs=10, inter_loc_dist=1,
                 inter_aisle_dist=2.4, min_freq=1, max_freq=20, max_orders=20,
                 max_products_in_order=5, check_solution=False, **kw):
        super().__init__(check_solution=check_solution, **kw)
        self.n_products, self.n_aisles, self.n_locs = n_products, n_aisles, n_locs
        self.inter_loc_dist, self.inter_aisle_dist = inter_loc_dist, inter_aisle_dist
        self.max_orders, self.max_products_in_order = max_orders, max_products_in_order
        self.freq_sampler = Uniform(low=min_freq, high=max_freq)  # slap/generator.py:44-46

    # -- generator: slap/generator.py:51-155 ---------------------------------
    @staticmethod
    def distance_matrix(locs):  # generator.py:51-65 (Manhattan)
        diff = locs[..., :, None, :] - locs[..., None, :, :]
        return torch.sum(torch.abs(diff), dim=-1)

    def coordinates(self, batch_size):  # generator.py:67-81 (loop over B x L)
        total = self.n_aisles * self.n_locs
        out = torch.zeros((*batch_size, total, 2), dtype=torch.float32)
        for b in range(batch_size[0]):
            for i in range(total):
                y = (i % self.n_locs) * self.inter_loc_dist
                x = (i // self.n_locs) * self.inter_aisle_dist
                out[b, i] = torch.tensor([x, y], dtype=torch.float32)
        return out

    def picklist(self, batch_size):  # generator.py:91-112 (numpy global RNG)
        batches = []
        for _ in range(batch_size[0]):
            orders = [np.random.randint(0, self.n_products, size=self.max_products_in_order).tolist()
                      for _ in range(self.max_orders)]
            batches.append(orders)
        return torch.tensor(batches)

    def generate(self, batch_size):  # generator.py:137-155
        batch_size = [batch_size] if isinstance(batch_size, int) else list(batch_size)
        freq = self.freq_sampler.sample((*batch_size, self.n_products, 1))
        locs = self.coordinates(batch_size)
        dist = self.distance_matrix(locs)
        return TD({"freq": freq, "locs": locs, "dist_mat": dist,
                   "assignment": torch.full((*batch_size, self.n_products), -1, dtype=torch.int),
                   "picklist": self.picklist(batch_size),
                   "depot_loc_dist": dist[:, 0, :]}, batch_size)

    # -- env: slap/env.py ------------------------------------------------------
    def _reset(self, td, batch_size):  # slap/env.py:95-129
        p = td["freq"].shape[-2]
        avail = torch.ones((*batch_size, td["locs"].shape[1]), dtype=torch.bool)
        avail[..., 0] = False
        return TD({
            "assignment": td["assignment"],
            "to_choose": torch.arange(p, dtype=torch.float32).unsqueeze(0).repeat(*batch_size, 1),
            "i": torch.zeros((*batch_size, 1), dtype=torch.int64),
            "ratio": torch.zeros(td["depot_loc_dist"].shape),
            "action_mask": avail,
            "reward": torch.zeros((*batch_size, 1), dtype=torch.float32),
        }, batch_size)

    @staticmethod
    def _step(td):  # slap/env.py:38-93
        product = td["to_choose"][..., 0]
        to_choose = td["to_choose"][..., 1:]
        loc = td["action"]
        b = loc.shape[0]
        assignment = td["assignment"].clone()
        product = product.to(torch.int)
        loc = loc.to(torch.int)
        assignment[torch.arange(b), product] = loc
        done = td["i"] == td["freq"].shape[-2] - 1
        mask = td["action_mask"].clone()
        for k in range(b):  # the reference's per-batch Python loop (env.py:61-62)
            mask[k][loc[k]] = False
        td.update({"assignment": assignment, "to_choose": to_choose, "action_mask": mask,
                   "i": td["i"] + 1, "reward": torch.zeros_like(done), "done": done})
        return td

    @staticmethod
    def _get_reward(td, actions):  # slap/env.py:131-143
        assignment, orders = td["assignment"], td["picklist"]
        total = torch.full((orders.shape[0],), 0, dtype=torch.float32)
        rows = torch.arange(assignment.size(0)).unsqueeze(1)
        for o in range(orders.shape[1]):
            subset = assignment[rows, orders[:, o, :]].to(torch.int)
            total += -get_tour_length(td["locs"][rows, subset])
        return total


ORACLE_REGISTRY = {"tsp": TSPOracle, "cvrp": CVRPOracle, "slap": SLAPOracle}


# ---------------------------------------------------------------------------
# Cheap deterministic policies used by the env-throughput benchmark
# (SURVEY section 8d); these define the bench workloads, not reference code.
# ---------------------------------------------------------------------------
def _f32_sqrt(sq):
    """Correctly rounded f32 sqrt (via f64, where double rounding is exact for sqrt).
    ATen's vectorised CPU sqrt is not correctly rounded in rare cases (e.g. input bits
    0x3b9f879c: 0x3d8ee5db instead of 0x3d8ee5dc), which would make the bench policies'
    lowest-index tie rule depend on the CPU's SIMD path."""
    return torch.sqrt(sq.double()).float()


def tsp_nearest_action(td):
    """Step 0: node 0; afterwards the nearest unvisited node to ``current_node``
    (Euclidean, f32 ``dx*dx+dy*dy`` and its correctly rounded sqrt, ties -> lowest
    index)."""
    if bool((td["i"] == 0).all()):
        return torch.zeros(td.batch_size[0], dtype=torch.int64)
    locs = td["locs"]
    cur = gather_by_index(locs, td["current_node"])
    diff = locs - cur[:, None, :]
    dist = _f32_sqrt(diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1])
    dist = dist.masked_fill(~td["action_mask"], float("inf"))
    return dist.argmin(-1)


def cvrp_nearest_action(td):
    """Nearest feasible customer to ``current_node`` (ties -> lowest index); the depot
    when no customer is feasible (also for finished instances)."""
    locs = td["locs"]
    cur = gather_by_index(locs, td["current_node"].squeeze(-1))
    diff = locs - cur[:, None, :]
    dist = _f32_sqrt(diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1])
    feas = td["action_mask"].clone()
    feas[:, 0] = False
    dist = dist.masked_fill(~feas, float("inf"))
    act = dist.argmin(-1)
    return torch.where(feas.any(-1), act, torch.zeros_like(act))


def slap_closest_free_action(td):
    """Free location with the lowest ``depot_loc_dist`` (ties -> lowest index)."""
    d = td["depot_loc_dist"].masked_fill(~td["action_mask"], float("inf"))
    return d.argmin(-1)
