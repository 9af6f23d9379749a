"""Device-resident rollout engine: a whole env episode (reset -> every step ->
reward) as a fixed sequence of C-ABI launches on one stream, captured once into a
HIP graph and replayed.

This is the env-only rollout of ``rl4co/utils/decoding.py:88-109`` with the policy
in-kernel (teacher-forced actions = Evaluate mode, or a cheap deterministic policy;
SURVEY.md 8d) and no host synchronisation inside the episode: the reference's
``while not td["done"].all()`` poll (``constructive/base.py:230``) is replaced by
the known episode length (TSP: N steps, SLAP: P steps) and, for CVRP, by a chunked
graph with a device-side not-done count polled between chunks.

Stepwise mode keeps the reference's TensorDict contract in HBM between steps
(every step reads and writes the full per-instance state: SURVEY.md 8d's
250 / 733 / 234 bytes per env-step); state buffers ping-pong between two copies.
"""
from __future__ import annotations

import torch

from .. import _native as nat


class _GraphEpisode:
    def __init__(self, device):
        self.device = torch.device(device)
        self.graph = None
        self.stream = torch.cuda.Stream(self.device)

    def _launch(self, s):  # pragma: no cover - overridden
        raise NotImplementedError

    def capture(self):
        torch.cuda.synchronize(self.device)
        with torch.cuda.stream(self.stream):
            self._launch(self.stream.cuda_stream)  # warm (loads code objects)
        self.stream.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream):
            self._launch(torch.cuda.current_stream(self.device).cuda_stream)
        self.graph = g
        return self

    def run_eager(self):
        """One episode launched on the episode's stream, ordered after everything already
        queued on the caller's stream (inputs written there) and before whatever the caller
        queues next (reads of the outputs)."""
        cur = torch.cuda.current_stream(self.device)
        self.stream.wait_stream(cur)
        with torch.cuda.stream(self.stream):
            self._launch(self.stream.cuda_stream)
        cur.wait_stream(self.stream)

    def replay(self):
        if self.graph is None:
            self.capture()
        self.graph.replay()


class TSPStepwiseEpisode(_GraphEpisode):
    """Reset + N x co_tsp_step (+ optional in-kernel nearest policy) + co_tsp_reward.

    ``chunk`` > 1 (teacher actions): the steps go out as ceil(N / chunk) co_tsp_steps
    launches of `chunk` steps each -- the same per-step state writes into the same
    ping-pong buffers (bit-identical), fewer launch boundaries."""

    def __init__(self, locs: torch.Tensor, actions: torch.Tensor = None, policy: str = "teacher",
                 check: bool = True, chunk: int = 1):
        super().__init__(locs.device)
        b, n, _ = locs.shape
        self.b, self.n, self.policy, self.check = b, n, policy, check
        self.chunk = max(1, int(chunk)) if policy == "teacher" else 1
        d = locs.device
        self.locs = locs.contiguous()
        if policy == "teacher":
            assert actions is not None and actions.shape == (b, n)
            self.acts = actions.t().contiguous()  # step-major: each step's action is a [B] row
        else:
            self.acts = torch.empty((n, b), dtype=torch.int64, device=d)
        self.mask = [torch.empty((b, n), dtype=torch.bool, device=d) for _ in range(2)]
        self.i = [torch.empty((b, 1), dtype=torch.int64, device=d) for _ in range(2)]
        self.first = [torch.empty(b, dtype=torch.int64, device=d) for _ in range(2)]
        self.cur = torch.empty(b, dtype=torch.int64, device=d)
        self.done = torch.empty(b, dtype=torch.bool, device=d)
        self.step_reward = torch.empty(b, dtype=torch.bool, device=d)
        self.reset_reward = torch.empty((b, 1), dtype=torch.float32, device=d)
        self.reward = torch.empty(b, dtype=torch.float32, device=d)
        self.status = torch.zeros(1, dtype=torch.int32, device=d)

    def _launch(self, s):
        b, n = self.b, self.n
        nat.call("co_tsp_reset", b, n, nat.ptr(self.mask[0]), nat.ptr(self.first[0]),
                 nat.ptr(self.cur), nat.ptr(self.i[0]), nat.ptr(self.reset_reward), s)
        for t0 in range(0, n if self.chunk > 1 else 0, self.chunk):
            k = min(self.chunk, n - t0)
            a_, b_ = t0 & 1, (t0 + 1) & 1  # step t0 reads buffer a_ (the ping-pong parity)
            nat.call("co_tsp_steps", b, n, k, nat.ptr(self.acts[t0]), b, nat.ptr(self.mask[a_]),
                     nat.ptr(self.i[a_]), nat.ptr(self.first[a_]), nat.ptr(self.mask[b_]),
                     nat.ptr(self.i[b_]), nat.ptr(self.first[b_]), nat.ptr(self.cur),
                     nat.ptr(self.done), nat.ptr(self.step_reward), 1 if t0 == 0 else 0,
                     nat.ptr(self.status), s)
        for t in range(n if self.chunk == 1 else 0):
            src, dst = t & 1, (t + 1) & 1
            a = self.acts[t]
            if self.policy == "nearest":
                nat.call("co_tsp_nearest_action", b, n, nat.ptr(self.locs), nat.ptr(self.mask[src]),
                         nat.ptr(self.cur), int(t == 0), nat.ptr(a), s)
            nat.call("co_tsp_step", b, n, nat.ptr(a), nat.ptr(self.mask[src]),
                     nat.ptr(self.mask[dst]), nat.ptr(self.i[src]), nat.ptr(self.i[dst]),
                     nat.ptr(self.first[src]), nat.ptr(self.first[dst]), nat.ptr(self.cur),
                     nat.ptr(self.done), nat.ptr(self.step_reward), 1 if t == 0 else 0, None,
                     nat.ptr(self.status), s)
        nat.call("co_tsp_reward", b, n, n, nat.ptr(self.locs), b, nat.ptr(self.acts), 1, b,
                 int(self.check), nat.ptr(self.reward), nat.ptr(self.status), s)

    def final_state(self):
        k = self.n & 1
        return {"action_mask": self.mask[k], "i": self.i[k], "first_node": self.first[k],
                "current_node": self.cur, "done": self.done, "reward": self.reward,
                "actions": self.acts.t()}


class SLAPStepwiseEpisode(_GraphEpisode):
    """Reset + P x co_slap_step (in-place assignment) + co_slap_reward; with the
    closest-free bench policy each step is one co_slap_closest_step launch (policy +
    step), teacher-forced actions go through co_slap_step alone.

    ``chunk`` > 1 (closest policy): the steps go out as ceil(P / chunk)
    co_slap_closest_steps launches -- the same per-step state writes into the same
    ping-pong buffers (bit-identical), fewer launch boundaries."""

    def __init__(self, td, actions=None, policy: str = "teacher", chunk: int = 1):
        locs = td["locs"]
        super().__init__(locs.device)
        d = locs.device
        b, l = locs.shape[0], locs.shape[1]
        p = td["freq"].shape[-2]
        self.b, self.l, self.p, self.policy = b, l, p, policy
        self.chunk = max(1, int(chunk)) if policy == "closest" else 1
        self.locs = locs.contiguous()
        self.picklist = td["picklist"].contiguous()
        self.depot_dist = td["depot_loc_dist"].contiguous()
        self.assign0 = td["assignment"].contiguous()
        self.assign = torch.empty_like(self.assign0)
        if policy == "teacher":
            self.acts = actions.t().contiguous()
        else:
            self.acts = torch.empty((p, b), dtype=torch.int64, device=d)
        self.mask = [torch.empty((b, l), dtype=torch.bool, device=d) for _ in range(2)]
        self.i = [torch.empty((b, 1), dtype=torch.int64, device=d) for _ in range(2)]
        self.to_choose = torch.empty((b, p), dtype=torch.float32, device=d)
        self.ratio = torch.empty((b, l), dtype=torch.float32, device=d)
        self.done = torch.empty((b, 1), dtype=torch.bool, device=d)
        self.step_reward = torch.empty((b, 1), dtype=torch.bool, device=d)
        self.reset_reward = torch.empty((b, 1), dtype=torch.float32, device=d)
        self.reward = torch.empty(b, dtype=torch.float32, device=d)
        self.status = torch.zeros(1, dtype=torch.int32, device=d)

    def _launch(self, s):
        b, l, p = self.b, self.l, self.p
        nat.call("co_slap_reset", b, l, p, nat.ptr(self.mask[0]), nat.ptr(self.to_choose),
                 nat.ptr(self.i[0]), nat.ptr(self.reset_reward), nat.ptr(self.ratio), None, None,
                 s)
        for t0 in range(0, p if self.chunk > 1 else 0, self.chunk):
            k = min(self.chunk, p - t0)
            a_, b_ = t0 & 1, (t0 + 1) & 1  # step t0 reads buffer a_ (the ping-pong parity)
            nat.call("co_slap_closest_steps", b, l, p, k, nat.ptr(self.depot_dist),
                     nat.ptr(self.to_choose[:, t0:]), p,
                     nat.ptr(self.assign0 if t0 == 0 else self.assign), nat.ptr(self.assign),
                     nat.ptr(self.mask[a_]), nat.ptr(self.i[a_]), nat.ptr(self.mask[b_]),
                     nat.ptr(self.i[b_]), nat.ptr(self.acts[t0]), b, nat.ptr(self.done),
                     nat.ptr(self.step_reward), nat.ptr(self.status), s)
        for t in range(p if self.chunk == 1 else 0):
            src, dst = t & 1, (t + 1) & 1
            a = self.acts[t]
            tc = self.to_choose[:, t:]
            # the generator's -1 assignment is the episode's starting state: the first step
            # writes out of place from it (the reference clones, slap/env.py:50), later ones
            # in place
            a_in = self.assign0 if t == 0 else self.assign
            if self.policy == "closest":  # the bench policy fused with the step: one launch
                nat.call("co_slap_closest_step", b, l, p, nat.ptr(self.depot_dist), nat.ptr(tc), p,
                         nat.ptr(a_in), nat.ptr(self.assign), nat.ptr(self.mask[src]),
                         nat.ptr(self.mask[dst]),
                         nat.ptr(a), nat.ptr(self.i[src]), nat.ptr(self.i[dst]),
                         nat.ptr(self.done), nat.ptr(self.step_reward), nat.ptr(self.status), s)
                continue
            nat.call("co_slap_step", b, l, p, nat.ptr(a), nat.ptr(tc), p, nat.ptr(a_in),
                     nat.ptr(self.assign), nat.ptr(self.mask[src]), nat.ptr(self.mask[dst]),
                     nat.ptr(self.i[src]), nat.ptr(self.i[dst]), nat.ptr(self.done),
                     nat.ptr(self.step_reward), nat.ptr(self.status), s)
        nat.call("co_slap_reward", b, l, p, self.picklist.shape[1], self.picklist.shape[2],
                 nat.ptr(self.assign), nat.ptr(self.picklist), nat.ptr(self.locs),
                 nat.ptr(self.reward), nat.ptr(self.status), s)

    def final_state(self):
        k = self.p & 1
        return {"action_mask": self.mask[k], "i": self.i[k], "assignment": self.assign,
                "done": self.done, "reward": self.reward, "actions": self.acts.t()}


class TSPFusedEpisode(_GraphEpisode):
    """The whole TSP episode as ONE launch (``co_tsp_rollout_ex``): reset, N steps with the
    policy in-kernel (teacher-forced actions, or nearest-unvisited) and the reward, state
    in registers/LDS; writes the post-rollout TensorDict columns.

    Teacher actions stay in the caller's row-major ``[B, N]`` layout (the reference's
    ``[B, T]``: one lane group per instance reads contiguous rows) for N <= 1024;
    ``layout="steps"`` (or N > 1024) transposes them once to the step-major ``[N, B]`` the
    stepwise kernels read (the LDS-tile engine)."""

    def __init__(self, locs: torch.Tensor, actions: torch.Tensor = None, policy: str = "teacher",
                 check: bool = True, layout: str = "rows"):
        super().__init__(locs.device)
        b, n, _ = locs.shape
        d = locs.device
        self.b, self.n, self.policy, self.check = b, n, policy, check
        self.locs = locs.contiguous()
        self.rows = policy == "teacher" and layout == "rows" and n <= 1024
        if policy == "teacher":
            assert actions is not None and actions.shape == (b, n)
            # the episode owns its copy (the transposed layout always copied): a captured
            # graph replays on these, whatever the caller later does to its tensor
            self.acts = (actions.to(torch.long, memory_format=torch.contiguous_format, copy=True)
                         if self.rows else actions.t().contiguous())
        else:
            self.acts = torch.empty((n, b), dtype=torch.int64, device=d)
        self.mask = torch.empty((b, n), dtype=torch.bool, device=d)
        self.first = torch.empty(b, dtype=torch.int64, device=d)
        self.cur = torch.empty(b, dtype=torch.int64, device=d)
        self.i = torch.empty((b, 1), dtype=torch.int64, device=d)
        self.done = torch.empty(b, dtype=torch.bool, device=d)
        self.step_reward = torch.empty(b, dtype=torch.bool, device=d)
        self.reward = torch.empty(b, dtype=torch.float32, device=d)
        self.status = torch.zeros(1, dtype=torch.int32, device=d)

        teacher = self.policy == "teacher"
        sb, st = (n, 1) if self.rows else (1, b)
        self._bound = nat.bind(
            "co_tsp_rollout_ex", self.b, self.n, nat.ptr(self.locs),
            nat.ptr(self.acts) if teacher else None, sb, st,
            None if teacher else nat.ptr(self.acts),
            nat.ptr(self.mask), nat.ptr(self.first), nat.ptr(self.cur), nat.ptr(self.i),
            nat.ptr(self.done), nat.ptr(self.step_reward), nat.ptr(self.reward),
            int(self.check), nat.ptr(self.status))

    def _launch(self, s):
        self._bound(s)

    def final_state(self):
        return {"action_mask": self.mask, "i": self.i, "first_node": self.first,
                "current_node": self.cur, "done": self.done, "reward": self.reward,
                "actions": self.acts if self.rows else self.acts.t()}


class SLAPFusedEpisode(_GraphEpisode):
    """The whole SLAP episode as ONE launch (``co_slap_rollout``): reset, P steps with
    teacher-forced step-major actions or the closest-free policy, and the pick-tour
    reward; writes the post-rollout TensorDict columns."""

    def __init__(self, td, actions=None, policy: str = "teacher", write_ratio: bool = True):
        locs = td["locs"]
        super().__init__(locs.device)
        d = locs.device
        b, l = locs.shape[0], locs.shape[1]
        p = td["freq"].shape[-2]
        self.b, self.l, self.p, self.policy = b, l, p, policy
        # co_slap_rollout holds an instance's L locations in 8 registers of up to 32 lanes
        # (L <= 256); larger warehouses run the same episode as the stepwise launch sequence
        self._stepwise = SLAPStepwiseEpisode(td, actions, policy) if l > 256 else None
        if self._stepwise is not None:
            self.status = self._stepwise.status
            return
        self.locs = locs.contiguous()
        self.picklist = td["picklist"].contiguous()
        self.o, self.k = self.picklist.shape[1], self.picklist.shape[2]
        self.depot_dist = td["depot_loc_dist"].contiguous()
        self.assign0 = td["assignment"].contiguous()
        if policy == "teacher":
            self.acts = actions.t().contiguous()
        else:
            self.acts = torch.empty((p, b), dtype=torch.int64, device=d)
        self.mask = torch.empty((b, l), dtype=torch.bool, device=d)
        self.assign = torch.empty_like(self.assign0)
        self.i = torch.empty((b, 1), dtype=torch.int64, device=d)
        self.done = torch.empty((b, 1), dtype=torch.bool, device=d)
        self.step_reward = torch.empty((b, 1), dtype=torch.bool, device=d)
        self.reward = torch.empty(b, dtype=torch.float32, device=d)
        self.ratio = torch.empty((b, l), dtype=torch.float32, device=d) if write_ratio else None
        self.status = torch.zeros(1, dtype=torch.int32, device=d)

        teacher = self.policy == "teacher"
        self._bound = nat.bind(
            "co_slap_rollout", self.b, self.l, self.p, self.o, self.k, nat.ptr(self.locs),
            nat.ptr(self.picklist), nat.ptr(self.depot_dist), nat.ptr(self.assign0),
            nat.ptr(self.acts) if teacher else None, None if teacher else nat.ptr(self.acts),
            nat.ptr(self.mask), nat.ptr(self.assign), nat.ptr(self.i), nat.ptr(self.done),
            nat.ptr(self.step_reward), nat.ptr(self.reward), nat.ptr(self.ratio),
            nat.ptr(self.status))

    def _launch(self, s):
        if self._stepwise is not None:
            self._stepwise._launch(s)
            return
        self._bound(s)

    def final_state(self):
        if self._stepwise is not None:
            return self._stepwise.final_state()
        return {"action_mask": self.mask, "i": self.i, "assignment": self.assign,
                "done": self.done, "reward": self.reward, "actions": self.acts.t()}


class CVRPFusedEpisode(_GraphEpisode):
    """The whole CVRP episode as ONE C-ABI call (``co_cvrp_rollout``): reset from the
    generator columns, the nearest-feasible policy until every instance is done, the
    reference's trailing depot steps for early finishers, and the closed-tour reward.

    ``td`` holds the generator columns (``depot [B,2]``, ``locs [B,N,2]``, ``demand
    [B,N]`` already divided by the capacity); ``vehicle_capacity`` is the env's
    (``cvrp/env.py:126``, ``generator.vehicle_capacity``)."""

    # co_cvrp_rollout packs the step count into 15 bits; an episode ends within 2N + 1 <=
    # 2,047 steps (N <= 1023), so a larger caller limit is the same limit
    KERNEL_MAX_STEPS = 0x7fff

    def __init__(self, td, vehicle_capacity: float = 1.0, max_steps: int = None,
                 write_locs: bool = True):
        locs = td["locs"]
        super().__init__(locs.device)
        d = locs.device
        b, n = locs.shape[0], locs.shape[1]
        if n > 1023:
            # the register-resident group engine holds N + 1 <= 1024 nodes (64 lanes x 16);
            # the stepwise loop (CVRPStepwiseEpisode) has no such limit
            raise NotImplementedError(
                f"CVRPFusedEpisode: num_loc={n} > 1023; use CVRPStepwiseEpisode (co_cvrp_rollout "
                "keeps an instance's nodes in 64 lanes x 16 registers)")
        self.b, self.n, self.vcap = b, n, float(vehicle_capacity)
        self.max_steps = int(max_steps) if max_steps is not None else 2 * n + 1
        self.depot = td["depot"].contiguous()
        self.locs_in = locs.contiguous()
        self.demand = td["demand"].contiguous()
        self.acts = torch.empty((self.max_steps, b), dtype=torch.int64, device=d)
        self.locs = torch.empty((b, n + 1, 2), dtype=torch.float32, device=d) if write_locs else None
        self.cur = torch.empty((b, 1), dtype=torch.int64, device=d)
        self.used = torch.empty((b, 1), dtype=torch.float32, device=d)
        self.vcap_t = torch.empty((b, 1), dtype=torch.float32, device=d)
        self.visited = torch.empty((b, n + 1), dtype=torch.uint8, device=d)
        self.mask = torch.empty((b, n + 1), dtype=torch.bool, device=d)
        self.done = torch.empty(b, dtype=torch.bool, device=d)
        self.step_reward = torch.empty(b, dtype=torch.bool, device=d)
        self.reward = torch.empty(b, dtype=torch.float32, device=d)
        self.lens = torch.empty(b, dtype=torch.int32, device=d)
        self.steps = torch.zeros(1, dtype=torch.int32, device=d)
        self.status = torch.zeros(1, dtype=torch.int32, device=d)

        self._bound = nat.bind(
            "co_cvrp_rollout", self.b, self.n, nat.ptr(self.depot), nat.ptr(self.locs_in),
            nat.ptr(self.demand), self.vcap, min(self.max_steps, self.KERNEL_MAX_STEPS),
            nat.ptr(self.acts),
            nat.ptr(self.locs), nat.ptr(self.cur), nat.ptr(self.used), nat.ptr(self.vcap_t),
            nat.ptr(self.visited), nat.ptr(self.mask), nat.ptr(self.done),
            nat.ptr(self.step_reward), nat.ptr(self.reward), nat.ptr(self.lens),
            nat.ptr(self.steps), nat.ptr(self.status))

    def _launch(self, s):
        self._bound(s)

    def final_state(self):
        """Post-rollout columns; reads the episode length (one host sync)."""
        t = int(self.steps.item())
        if int(self.status.item()) & nat.ST_TRUNCATED:
            raise RuntimeError(f"CVRP rollout: an instance was not done after {self.max_steps} steps")
        return {"locs": self.locs, "current_node": self.cur, "used_capacity": self.used,
                "vehicle_capacity": self.vcap_t, "visited": self.visited,
                "action_mask": self.mask, "done": self.done, "reward": self.reward,
                "actions": self.acts[:t].t(), "steps": t}


class CVRPStepwiseEpisode:
    """Reference-shaped CVRP loop: one ``co_cvrp_nearest_action`` + ``co_cvrp_step``
    launch pair per env step with the TensorDict state in HBM, ``while not
    done.all()`` replaced by graph chunks and a device-side not-done count per step
    (accumulated by ``co_cvrp_step`` itself) read once per chunk.  No instance can be done
    before step N (N customers and one depot visit), so steps 0..N-1 are one graph that
    counts nothing; later chunks are ``chunk`` steps.  Per-step
    ``current_node``/``used_capacity`` rows are kept, so the state at the exact
    all-done step T is returned even when the last chunk runs past it (steps after T
    only repeat the depot action)."""

    def __init__(self, td, vehicle_capacity: float = 1.0, max_steps: int = None,
                 chunk: int = 8, fused_policy: bool = True):
        locs = td["locs"]
        # fused_policy: co_cvrp_nearest_step (policy + step, one launch); False: the
        # co_cvrp_nearest_action + co_cvrp_step pair (the env step alone, as a policy-agnostic
        # loop calls it)
        self.fused_policy = fused_policy
        d = locs.device
        self.device = d
        b, n = locs.shape[0], locs.shape[1]
        self.b, self.n, self.vcap, self.chunk = b, n, float(vehicle_capacity), chunk
        self.max_steps = int(max_steps) if max_steps is not None else 2 * n + 1
        T = self.max_steps
        self.depot = td["depot"].contiguous()
        self.locs_in = locs.contiguous()
        self.demand = td["demand"].contiguous()
        self.locs = torch.empty((b, n + 1, 2), dtype=torch.float32, device=d)
        self.acts = torch.empty((T, b), dtype=torch.int64, device=d)
        self.cur = torch.empty((T + 1, b), dtype=torch.int64, device=d)
        self.used = torch.empty((T + 1, b), dtype=torch.float32, device=d)
        self.vcap_t = torch.empty((b, 1), dtype=torch.float32, device=d)
        self.visited = [torch.empty((b, n + 1), dtype=torch.uint8, device=d) for _ in range(2)]
        self.mask = [torch.empty((b, n + 1), dtype=torch.bool, device=d) for _ in range(2)]
        self.done = torch.empty(b, dtype=torch.bool, device=d)
        self.step_reward = torch.empty(b, dtype=torch.bool, device=d)
        self.not_done = torch.empty(T, dtype=torch.int32, device=d)
        self.reward = torch.empty(b, dtype=torch.float32, device=d)
        self.status = torch.zeros(1, dtype=torch.int32, device=d)
        self.stream = torch.cuda.Stream(d)
        self.graphs = None
        self.T = None

    def _reset(self, s):
        self.not_done.zero_()  # per-step counters, incremented by co_cvrp_step
        nat.call("co_cvrp_reset", self.b, self.n, nat.ptr(self.depot), nat.ptr(self.locs_in),
                 nat.ptr(self.demand), self.vcap, nat.ptr(self.locs), nat.ptr(self.cur[0]),
                 nat.ptr(self.used[0]), nat.ptr(self.vcap_t), nat.ptr(self.visited[0]),
                 nat.ptr(self.mask[0]), s)

    def _step(self, t, s):
        k, k1 = t % 2, (t + 1) % 2
        nd = nat.ptr(self.not_done[t:]) if t >= self.n else None
        if self.fused_policy:  # the bench policy fused with the step: one launch
            nat.call("co_cvrp_nearest_step", self.b, self.n, nat.ptr(self.locs),
                     nat.ptr(self.demand), nat.ptr(self.used[t]), nat.ptr(self.used[t + 1]),
                     nat.ptr(self.vcap_t), nat.ptr(self.visited[k]), nat.ptr(self.visited[k1]),
                     nat.ptr(self.mask[k]), nat.ptr(self.cur[t]), nat.ptr(self.acts[t]),
                     nat.ptr(self.cur[t + 1]), nat.ptr(self.done), nat.ptr(self.step_reward),
                     nat.ptr(self.mask[k1]), nat.ptr(self.status), nd, s)
            return
        nat.call("co_cvrp_nearest_action", self.b, self.n, nat.ptr(self.locs),
                 nat.ptr(self.mask[k]), nat.ptr(self.cur[t]), nat.ptr(self.acts[t]), s)
        nat.call("co_cvrp_step", self.b, self.n, nat.ptr(self.acts[t]), nat.ptr(self.demand),
                 nat.ptr(self.used[t]), nat.ptr(self.used[t + 1]), nat.ptr(self.vcap_t),
                 nat.ptr(self.visited[k]), nat.ptr(self.visited[k1]), nat.ptr(self.cur[t + 1]),
                 nat.ptr(self.done), nat.ptr(self.step_reward), nat.ptr(self.mask[k1]),
                 nat.ptr(self.status), nd, s)

    def _ranges(self):
        first = min(self.n, self.max_steps)
        out = [(0, first)]
        t = first
        while t < self.max_steps:
            out.append((t, min(t + self.chunk, self.max_steps)))
            t += self.chunk
        return out

    def capture(self):
        torch.cuda.synchronize(self.device)
        with torch.cuda.stream(self.stream):  # warm-up: load code objects
            self._reset(self.stream.cuda_stream)
            self._step(0, self.stream.cuda_stream)
        self.stream.synchronize()
        self.graphs = []
        for j, (t0, t1) in enumerate(self._ranges()):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=self.stream):
                s = torch.cuda.current_stream(self.device).cuda_stream
                if j == 0:
                    self._reset(s)
                for t in range(t0, t1):
                    self._step(t, s)
            self.graphs.append((t0, t1, g))
        return self

    def replay(self):
        """One episode; returns the episode length T (host sync once per chunk)."""
        if self.graphs is None:
            self.capture()
        self.T = None
        for t0, t1, g in self.graphs:
            g.replay()
            if t1 > self.n and int(self.not_done[t1 - 1].item()) == 0:
                nd = self.not_done[t0:t1].cpu()
                self.T = t0 + int((nd == 0).nonzero()[0, 0]) + 1
                break
        if self.T is None:
            raise RuntimeError(f"CVRP rollout: not done after {self.max_steps} steps")
        acts = self.acts[:self.T]
        nat.call("co_cvrp_reward", self.b, self.n, self.T, nat.ptr(self.locs), nat.ptr(acts), 1,
                 self.b, nat.ptr(self.demand), nat.ptr(self.vcap_t), 1, nat.ptr(self.reward),
                 nat.ptr(self.status), torch.cuda.current_stream(self.device).cuda_stream)
        return self.T

    def final_state(self):
        T = self.T
        return {"locs": self.locs, "current_node": self.cur[T].view(self.b, 1),
                "used_capacity": self.used[T].view(self.b, 1),
                "vehicle_capacity": self.vcap_t, "visited": self.visited[T % 2],
                "action_mask": self.mask[T % 2], "done": self.done, "reward": self.reward,
                "actions": self.acts[:T].t(), "steps": T}
