"""World-size-2 gloo test of the multi-GPU path's host logic: instance sharding and the
all-gather of per-instance POMO shared-baseline results (RCCL on the GPU pool, gloo here
on CPU tensors).  The per-instance values come from the CPU oracle."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rl4co_slap_amd.rollout.pomo import global_metrics, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _per_instance(reward_bs, ll_bs):
    bl = reward_bs.mean(1)
    mx = reward_bs.max(1).values
    lterm = ((reward_bs - bl[:, None]) * ll_bs).sum(1)
    return bl, mx, lterm


def _worker(rank, world, port, total, starts, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(0)
    reward = -torch.rand(total, starts, generator=g) * 10
    ll = -torch.rand(total, starts, generator=g) * 50
    lo, hi = shard_range(total, world, rank)
    bl, mx, lt = _per_instance(reward[lo:hi], ll[lo:hi])
    # the bench's path: shard sizes from shard_range, one padded all-gather, no host read
    m = global_metrics(bl, mx, lt, starts, total_instances=total)
    # sizes exchanged (callers that do not know the total)
    m2 = global_metrics(bl, mx, lt, starts)
    assert torch.equal(m["per_instance"], m2["per_instance"])
    if rank == 0:
        q.put({k: (v.item() if torch.is_tensor(v) and v.dim() == 0 else v) for k, v in m.items()
               if k != "per_instance"})
    dist.barrier()
    dist.destroy_process_group()


def test_shard_range_covers_everything():
    for total in (0, 1, 7, 8192, 8193):
        for world in (1, 2, 3, 8):
            spans = [shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_global_metrics_world2_matches_single_process():
    total, starts = 37, 20  # odd total: uneven shards exercise the padded all-gather
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    mp.spawn(_worker, args=(2, port, total, starts, q), nprocs=2, join=True)
    got = q.get(timeout=60)
    g = torch.Generator().manual_seed(0)
    reward = -torch.rand(total, starts, generator=g) * 10
    ll = -torch.rand(total, starts, generator=g) * 50
    adv = reward - reward.mean(1, keepdim=True)  # SharedBaseline (baselines.py:60-61)
    ref_loss = -(adv * ll).mean()                # reinforce.py:103-105
    assert got["instances"] == total
    assert abs(got["loss"] - ref_loss.item()) < 1e-4
    assert abs(got["reward_mean"] - reward.mean().item()) < 1e-5
    assert abs(got["max_reward_mean"] - reward.max(1).values.mean().item()) < 1e-5


def _oracle_pomo_terms(lo, hi, n):
    """Per-instance POMO terms of instances [lo, hi) from the oracle's multistart greedy
    episode (the env results a rank's shard produces; logits = a fixed seeded stand-in
    for the policy network, indexed by global instance so shards agree with the whole)."""
    from oracle.envs import TSPOracle
    from oracle.rollout import constructive_forward
    from oracle.ops import unbatchify
    from oracle.td import TD

    torch.manual_seed(1234)
    locs_all = torch.rand(12, n, 2)
    g = torch.Generator().manual_seed(99)
    logits_all = torch.randn(n - 1, n, 12, n, generator=g)  # [step, start, instance, node]
    b = hi - lo
    env = TSPOracle(num_loc=n, seed=n)
    td = env.reset(TD({"locs": locs_all[lo:hi].clone()}, [b]))
    step = {"t": 0}

    def logits_fn(_):
        lg = logits_all[step["t"], :, lo:hi].reshape(n * b, n)  # env e = s*b + i
        step["t"] += 1
        return lg.clone()

    out = constructive_forward(td, env, logits_fn, decode_type="multistart_greedy",
                               tanh_clipping=10.0)
    return _per_instance(unbatchify(out["reward"], n), unbatchify(out["log_likelihood"], n))


def _pomo_worker(rank, world, port, n, q):
    from rl4co_slap_amd.rollout.pomo import global_metrics, shard_range

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_range(12, world, rank)  # the bench's contiguous balanced shards
    bl, mx, lt = _oracle_pomo_terms(lo, hi, n)
    m = global_metrics(bl, mx, lt, n, total_instances=12)
    if rank == 0:
        q.put({k: (v.item() if torch.is_tensor(v) and v.dim() == 0 else v) for k, v in m.items()
               if k != "per_instance"})
    dist.barrier()
    dist.destroy_process_group()


def test_pomo_shards_world2_match_whole_batch():
    """Each rank runs the oracle POMO episode on its shard_range of 12 TSP-10 instances
    and all-gathers the per-instance terms; the global loss / rewards equal the
    single-process episode over all 12 (pomo/model.py:105-114)."""
    n = 10
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.spawn(_pomo_worker, args=(2, _free_port(), n, q), nprocs=2, join=True)
    got = q.get(timeout=60)
    bl, mx, lt = _oracle_pomo_terms(0, 12, n)
    assert got["instances"] == 12
    assert abs(got["loss"] - (-lt.sum() / (12 * n)).item()) < 1e-5
    assert abs(got["reward_mean"] - bl.mean().item()) < 1e-5
    assert abs(got["max_reward_mean"] - mx.mean().item()) < 1e-5
