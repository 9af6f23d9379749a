"""Device instance generation checker -- TEST INFRASTRUCTURE ONLY.

``co_uniform_fill`` (ops.hip) draws the reference's Uniform instance samplers
(``rl4co/envs/routing/tsp/generator.py:51-60``, ``cvrp/generator.py:116-143``: loc
``Uniform(min_loc, max_loc)``, demand ``(Uniform(min-1, max-1).int() + 1) / capacity``)
from a Philox-4x32-10 counter stream.  The stream is not torch's CPU generator, so this
file restates it in numpy: the Philox block function (Salmon et al., "Parallel random
numbers: as easy as 1, 2, 3", SC'11; pinned by its published known-answer vectors in
tests/test_oracle_kat.py), torch's f32 uniform grid ``u = (x >> 8) * 2^-24`` and the
samplers' transforms in float32 with one rounding per operation.
"""
import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(ctr, key):
    """Philox-4x32 with 10 rounds.  ``ctr``: uint64 array ``[n, 4]`` of 32-bit words,
    ``key``: ``[n, 2]`` (or broadcastable).  Returns ``[n, 4]`` uint64 words."""
    c = [np.asarray(ctr[..., i], dtype=np.uint64) for i in range(4)]
    k0 = np.asarray(key[..., 0], dtype=np.uint64).copy()
    k1 = np.asarray(key[..., 1], dtype=np.uint64).copy()
    for _ in range(10):
        p0 = np.uint64(M0) * c[0]
        p1 = np.uint64(M1) * c[2]
        c = [((p1 >> np.uint64(32)) ^ c[1] ^ k0) & np.uint64(MASK), p1 & np.uint64(MASK),
             ((p0 >> np.uint64(32)) ^ c[3] ^ k1) & np.uint64(MASK), p0 & np.uint64(MASK)]
        k0 = (k0 + np.uint64(W0)) & np.uint64(MASK)
        k1 = (k1 + np.uint64(W1)) & np.uint64(MASK)
    return np.stack(c, axis=-1)


def _words(n, seed, offset):
    nb = (n + 3) // 4
    blk = np.arange(nb, dtype=np.uint64) + np.uint64(offset)
    ctr = np.zeros((nb, 4), dtype=np.uint64)
    ctr[:, 0] = blk & np.uint64(MASK)
    ctr[:, 1] = blk >> np.uint64(32)
    key = np.array([seed & MASK, seed >> 32], dtype=np.uint64)[None, :]
    return philox4x32_10(ctr, key).reshape(-1)[:n]


def randint_fill(n, low, high, seed, offset=0):
    """``co_randint_fill``: ``low + (x * (high - low)) >> 32`` on the same stream layout."""
    x = _words(n, seed, offset)
    return np.int64(low) + ((x * np.uint64(high - low)) >> np.uint64(32)).astype(np.int64)


def uniform_fill(n, low, high, seed, offset=0, capacity=None):
    """Element ``i`` of ``co_uniform_fill``: word ``i % 4`` of the block at counter
    ``offset + i // 4`` (counter words 0/1 = its low/high halves, 2/3 = 0), key = seed."""
    x = _words(n, seed, offset)
    u = (x >> np.uint64(8)).astype(np.float32) * np.float32(2.0 ** -24)
    v = np.float32(low) + u * (np.float32(high) - np.float32(low))
    if capacity is None:
        return v
    return (v.astype(np.int32) + 1).astype(np.float32) / np.float32(capacity)
