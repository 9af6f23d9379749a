"""``Generator`` base and ``get_sampler`` (``rl4co/envs/common/utils.py:11-92``)."""
from __future__ import annotations

import abc
from typing import Callable, Union

import torch
from torch.distributions import Exponential, Normal, Poisson, Uniform

from .. import _native as nat


class Generator(metaclass=abc.ABCMeta):
    """Instances are produced on the CPU from torch's (or numpy's) global RNG exactly
    like the reference, then moved to the env device by ``reset``."""

    def __init__(self, **kwargs):
        self.kwargs = kwargs

    def __call__(self, batch_size):
        batch_size = [batch_size] if isinstance(batch_size, int) else list(batch_size)
        return self._generate(batch_size)

    @abc.abstractmethod
    def _generate(self, batch_size, **kwargs):
        raise NotImplementedError


def device_uniform(sampler, shape, device, capacity: float = None):
    """Device instance generation for throughput runs (``co_uniform_fill``, SURVEY.md 8f
    rank 1): ``sampler.sample(shape)`` for a scalar ``Uniform`` drawn on ``device`` from a
    Philox stream.  Values follow torch's f32 uniform grid and ``low + u * (high - low)``;
    the stream is not torch's CPU Mersenne Twister, so parity instances keep the host
    samplers.  The Philox key is drawn from torch's global CPU generator, so
    ``env.set_seed`` still makes the instances reproducible.  With ``capacity`` the
    CVRP demand transform ``((int)v + 1) / capacity`` (``cvrp/generator.py:137-143``) is
    applied in the same pass.  Returns ``None`` when ``sampler`` is not a scalar Uniform
    (the caller then samples on the host)."""
    if torch.device(device).type != "cuda" or not isinstance(sampler, Uniform) \
            or sampler.low.numel() != 1 or sampler.high.numel() != 1:
        return None
    out = torch.empty(tuple(shape), dtype=torch.float32, device=device)
    nat.require_device(out)
    seed = int(torch.randint(0, 2 ** 62, (), dtype=torch.int64))
    nat.call("co_uniform_fill", nat.ptr(out), out.numel(), float(sampler.low), float(sampler.high),
             float(capacity) if capacity is not None else 1.0, int(capacity is not None), seed, 0,
             nat.stream_of(out))
    return out


def get_sampler(val_name: str, distribution: Union[int, float, str, type, Callable], low: float = 0,
                high: float = 1.0, **kwargs):
    """``common/utils.py:26-92`` for the distributions the hot-path configs use;
    cluster / mixture samplers (``distribution_utils.py``) are out of scope."""
    if isinstance(distribution, (int, float)):
        return Uniform(low=distribution, high=distribution)
    if distribution == Uniform or distribution == "uniform":
        return Uniform(low=low, high=high)
    if distribution in (Normal, "normal", "gaussian"):
        return Normal(loc=kwargs[val_name + "_loc"], scale=kwargs[val_name + "_scale"])
    if distribution in (Exponential, "exponential"):
        return Exponential(rate=kwargs[val_name + "_rate"])
    if distribution in (Poisson, "poisson"):
        return Poisson(rate=kwargs[val_name + "_rate"])
    if distribution == "center":
        return Uniform(low=(high - low) / 2, high=(high - low) / 2)
    if distribution == "corner":
        return Uniform(low=low, high=low)
    if isinstance(distribution, Callable):
        return distribution(**kwargs)
    raise ValueError(f"Invalid distribution type of {distribution}")
