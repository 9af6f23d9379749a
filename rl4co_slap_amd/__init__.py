"""rl4co_slap_amd -- MI355X-native (gfx950) batched CO-environment + rollout engine.

Drop-in for the hot path of j4n1k/rl4co-slap: the TSP / CVRP / SLAP env step,
mask and reward functions, the autoregressive decode step and
``utils.ops.gather_by_index``, as hand-written HIP kernels behind a C ABI
(``include/co_env.h``).  The Python layer keeps the reference's TensorDict env API
and ``rl4co.envs`` registry names.
"""
from . import _native
from .envs import ENV_REGISTRY, CVRPEnv, SLAPEnv, TSPEnv, get_env
from .td import TensorDict

__all__ = ["ENV_REGISTRY", "CVRPEnv", "SLAPEnv", "TSPEnv", "get_env", "TensorDict", "_native"]
