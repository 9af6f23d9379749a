"""Pins the oracle's C restatement of ATen's CPU log_softmax math (``oracle/c/aten_math.c``)
against torch itself: F.log_softmax bit for bit over every width class, and SLEEF
expf/logf (the functions ATen's vectorised kernels call, reached through the symbols
libtorch_cpu exports) over the inputs log_softmax feeds them.  The gfx950 decode step
restates the same math (``csrc/co_math.hpp``); its GPU tests compare with F.log_softmax
directly (``tests/test_gpu_decode_exact.py``)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import aten_math

WIDTH = {"AVX512": 16, "AVX2": 8}.get(torch.backends.cpu.get_cpu_capability(), None)


def test_cpu_capability_is_the_one_the_kernel_restates():
    # csrc/co_math.hpp sums in the 16-lane order of ATen's AVX512 build; the GPU box's
    # EPYC 9575F reports AVX512 too (profiles/r02_host.txt)
    assert WIDTH == 16, torch.backends.cpu.get_cpu_capability()


def _rows(b, n, g, scale=3.0, p_mask=0.3):
    x = torch.randn(b, n, generator=g) * scale
    m = torch.rand(b, n, generator=g) > p_mask
    m[torch.arange(b), torch.randint(0, n, (b,), generator=g)] = True
    x[~m] = float("-inf")
    return x


@pytest.mark.parametrize("n", [1, 2, 5, 15, 16, 17, 20, 31, 32, 33, 50, 64, 100, 101, 128, 129,
                               255, 256, 500, 1000, 2048])
def test_log_softmax_bit_exact(n):
    g = torch.Generator().manual_seed(n)
    b = max(64, 20000 // n)
    for scale, p in ((3.0, 0.3), (0.01, 0.0), (40.0, 0.9)):
        x = _rows(b, n, g, scale, p)
        ref = F.log_softmax(x, dim=-1).numpy()
        got = aten_math.log_softmax(x.numpy(), WIDTH)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (n, scale)


def test_log_softmax_clip_and_temperature_bit_exact():
    # process_logits' pre-steps (decoding.py:172-180) are elementwise f32 ops; the
    # restatement applies log_softmax to what they produce
    g = torch.Generator().manual_seed(5)
    x = torch.randn(3000, 100, generator=g) * 4
    for clip, temp in ((10.0, 1.0), (0.0, 0.7), (10.0, 1.3)):
        y = torch.tanh(x) * clip if clip else x.clone()
        y = y / temp
        ref = F.log_softmax(y, dim=-1).numpy()
        assert np.array_equal(aten_math.log_softmax(y.numpy(), WIDTH).view(np.uint32),
                              ref.view(np.uint32))


def test_log_softmax_degenerate_rows():
    x = torch.tensor([[float("-inf")] * 20, [0.0] * 20, [float("inf")] + [0.0] * 19,
                      [float("nan")] + [1.0] * 19])
    ref = F.log_softmax(x, dim=-1).numpy()
    got = aten_math.log_softmax(x.numpy(), WIDTH)
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    assert np.array_equal(got[fin], ref[fin])


def _need_probe():
    # resolved inside the tests (not at collection): a `-m gpu` run collects this module
    # and must not map the oracle's probe library
    if aten_math.probe() is None:
        pytest.skip("torch's SLEEF probe needs an AVX512F host")


def test_expf_matches_torch_sleef():
    _need_probe()
    rng = np.random.default_rng(0)
    # log_softmax feeds exp with x - max <= 0: a dense sweep of the bit patterns of
    # [-104, 0] plus the saturation edges
    bits = rng.integers(0x80000000, 0xC2D00000, size=1 << 22, dtype=np.uint64).astype(np.uint32)
    x = np.concatenate([bits.view(np.float32), np.float32([0.0, -0.0, -103.97, -104.0, -104.01,
                                                           -87.3, -88.8, -1e-30, -np.inf] + [0] * 7)])
    x = x[: x.size - x.size % 16]
    got, ref = aten_math.expf(x), aten_math.sleef_expf(x)
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_logf_matches_torch_sleef():
    _need_probe()
    # every f32 in [1, 2) (the mantissa range), then a dense sample of the exp-sum range
    lo = np.arange(0x3F800000, 0x40000000, dtype=np.uint32).view(np.float32)
    rng = np.random.default_rng(1)
    hi = rng.integers(0x3F800000, 0x45800000, size=1 << 22, dtype=np.uint64).astype(np.uint32)
    for x in (lo, hi.view(np.float32)):
        got, ref = aten_math.logf(x), aten_math.sleef_logf(x)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))


def test_tanh_cr_is_correctly_rounded_and_close_to_torch():
    rng = np.random.default_rng(2)
    x = np.concatenate([rng.uniform(-12, 12, 1 << 20), rng.uniform(-1e-3, 1e-3, 1 << 16)])
    x = x.astype(np.float32)
    got = aten_math.tanh_cr(x)
    cr = np.tanh(x.astype(np.float64)).astype(np.float32)
    assert np.array_equal(got, cr)
    # torch.tanh (MKL VML) is within one ulp of it and equal on > 98 % of inputs
    t = torch.tanh(torch.from_numpy(x)).numpy()
    d = np.abs(got.view(np.int32).astype(np.int64) - t.view(np.int32).astype(np.int64))
    assert d.max() <= 1 and (d == 0).mean() > 0.98
