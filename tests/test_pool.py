"""utils/pool.py on CPU tensors (the pool's reuse rule is device-independent; the envs
enable it for HIP tensors only): a pooled tensor is handed out again only when nothing
else refers to it -- no Python reference, no view of its storage, no C++ owner."""
import torch

from rl4co_slap_amd.utils.pool import OutputPool

D = torch.device("cpu")


def _pool():
    return OutputPool(per_key=3, device_types=("cpu",))


def test_reuse_only_when_unreferenced():
    p = _pool()
    a = p.empty((4,), torch.int64, D)
    ida = id(a)
    b = p.empty((4,), torch.int64, D)
    assert a is not b
    del a
    c = p.empty((4,), torch.int64, D)
    assert id(c) == ida  # released: the same buffer again
    assert c is not b


def test_views_and_aliases_block_reuse():
    p = _pool()
    a = p.empty((6,), torch.float32, D)
    ida = id(a)
    v = a[2:]  # a view keeps the storage
    del a
    assert id(p.empty((6,), torch.float32, D)) != ida
    del v
    a = p.empty((6,), torch.float32, D)
    assert id(a) == ida
    h = a.detach()  # a second tensor object on the same storage
    del a
    assert id(p.empty((6,), torch.float32, D)) != ida
    del h
    a = p.empty((6,), torch.float32, D)
    assert id(a) == ida
    lst = [a]  # any Python reference
    del a
    assert id(p.empty((6,), torch.float32, D)) != ida
    del lst


def test_keys_and_capacity():
    p = _pool()
    x = p.empty((2, 3), torch.bool, D)
    assert p.empty((3, 2), torch.bool, D) is not x  # another shape: another slot list
    held = [p.empty((5,), torch.int32, D) for _ in range(5)]  # beyond per_key: plain allocs
    assert len(p._slots[((5,), torch.int32, D, 0)]) == 3
    assert len({id(t) for t in held}) == 5


def test_disabled_device_types_allocate_fresh():
    p = OutputPool()  # HIP only
    a = p.empty((4,), torch.int64, D)
    ida = id(a)
    del a
    assert not p._slots
    assert p.empty((4,), torch.int64, D) is not None and ida is not None
