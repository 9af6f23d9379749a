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


def check_errors(device="cuda") -> None:
    """Raise any error a device kernel without a caller-held status word recorded since
    the last read (an out-of-range ``gather_by_index`` index, the analogue of torch.gather's
    device-side assert).  The env's reward and ``post_decoder_hook`` read it with their own
    status read; code that calls ``gather_by_index`` outside a decode loop / reward calls
    this (one host sync) or runs with ``CO_SYNC_CHECKS=1`` (a read after every gather)."""
    import torch

    device = torch.device(device)
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    _native.check_deferred(device)


__all__ = ["ENV_REGISTRY", "CVRPEnv", "SLAPEnv", "TSPEnv", "get_env", "TensorDict", "_native",
           "check_errors"]
