"""Child process of tests/test_gpu_rccl.py (test helper, not product code): an ``nccl``
(RCCL) process group of world size 1 on cuda:0, initialised over a tcp://127.0.0.1 store
before any other GPU work in this process; ``global_metrics`` (the counterpart of
``rl4co/models/rl/common/base.py:238``'s cross-rank reduction) runs its
all-gather through RCCL and is compared bit for bit with the local computation of the same
per-instance values.  The values come from a POMO TSP-20 episode on the device
(``rollout/pomo.py``), so the exchange carries real shared-baseline results.
Prints ``RCCL_OK <backend> <instances>`` and exits 0 on success."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main(port: int):
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0,
                            world_size=1, device_id=dev)
    backend = dist.get_backend()
    assert backend == "nccl", backend
    from rl4co_slap_amd import _native
    from rl4co_slap_amd.rollout.pomo import POMOEpisode, global_metrics

    _native.load()
    b, n = 64, 20
    g = torch.Generator().manual_seed(11)
    locs = torch.rand(b, n, 2, generator=g).to(dev)
    logits = torch.randn(n - 1, n * b, n, generator=g).to(dev)
    ep = POMOEpisode(locs, logits)
    ep.replay()
    torch.cuda.synchronize(dev)
    assert int(ep.status.item()) == 0
    bl, mx, lt = ep.bl.clone(), ep.max_reward.clone(), ep.loss_terms.clone()
    local = torch.stack([bl, mx, lt])
    # through RCCL: shard sizes from shard_range (one all-gather), then exchanged (two)
    m1 = global_metrics(bl, mx, lt, n, total_instances=b)
    m2 = global_metrics(bl, mx, lt, n)
    torch.cuda.synchronize(dev)
    for m in (m1, m2):
        assert m["instances"] == b
        assert m["per_instance"].device == dev
        assert torch.equal(m["per_instance"], local), "RCCL all-gather changed the values"
        assert torch.equal(m["loss"], -local[2].sum() / (b * n))
        assert torch.equal(m["reward_mean"], local[0].mean())
        assert torch.equal(m["max_reward_mean"], local[1].mean())
    # a plain all-reduce on the same communicator (the bench's max-over-ranks timing path)
    t = torch.tensor([3.25], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert float(t.item()) == 3.25
    dist.barrier()
    dist.destroy_process_group()
    print(f"RCCL_OK {backend} {b}", flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]))
