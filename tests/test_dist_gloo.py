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
    m = global_metrics(bl, mx, lt, starts)
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
