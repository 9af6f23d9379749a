"""Env registry (``rl4co/envs/__init__.py:38-83``) for the three hot-path envs.

Only ``tsp``, ``cvrp`` and ``slap`` are built MI355X-native; asking for any other
reference env raises the reference's ``ValueError``.
"""
from .base import RL4COEnvBase
from .common import Generator, get_sampler
from .cvrp import CVRPEnv, CVRPGenerator
from .slap import SLAPEnv, SLAPGenerator
from .tsp import TSPEnv, TSPGenerator

ENV_REGISTRY = {"cvrp": CVRPEnv, "tsp": TSPEnv, "slap": SLAPEnv}


def get_env(env_name: str, *args, **kwargs) -> RL4COEnvBase:
    env_cls = ENV_REGISTRY.get(env_name, None)
    if env_cls is None:
        raise ValueError(
            f"Unknown environment {env_name}. Available environments: {ENV_REGISTRY.keys()}")
    return env_cls(*args, **kwargs)


__all__ = ["RL4COEnvBase", "Generator", "get_sampler", "TSPEnv", "TSPGenerator", "CVRPEnv",
           "CVRPGenerator", "SLAPEnv", "SLAPGenerator", "ENV_REGISTRY", "get_env"]
