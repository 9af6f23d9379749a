"""``Generator`` base and ``get_sampler`` (``rl4co/envs/common/utils.py:11-92``)."""
from __future__ import annotations

import abc
from typing import Callable, Union

from torch.distributions import Exponential, Normal, Poisson, Uniform


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
