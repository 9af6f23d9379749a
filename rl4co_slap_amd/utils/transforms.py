"""``rl4co/data/transforms.py`` (POMO / SymNCO state augmentation) on the gfx950 kernels.

``dihedral_8_augmentation`` is one launch (``co_dihedral8_augment``) writing the eight
reflections/rotations in the reference's order and batchify layout; the SR-group
``symmetric_augmentation`` draws its angles exactly as the reference does
(``torch.rand`` on the data's device, first ``B/num_augment`` rows = identity unless
``first_augment``) and transforms in one launch (``co_symmetric_augment``).
"""
from __future__ import annotations

import math
from typing import Union

import torch
from torch import Tensor

from .. import _native as nat
from .ops import batchify


def dihedral_8_augmentation(xy: Tensor) -> Tensor:
    """``transforms.py:15-37``: ``[B, N, 2] -> [8B, N, 2]``."""
    nat.require_device(xy)
    b, n, _ = xy.shape
    xy = xy.contiguous().float()
    out = torch.empty((8 * b, n, 2), dtype=torch.float32, device=xy.device)
    nat.call("co_dihedral8_augment", b, n, nat.ptr(xy), nat.ptr(out), nat.stream_of(xy))
    return out


def dihedral_8_augmentation_wrapper(xy: Tensor, reduce: bool = True, *args, **kw) -> Tensor:
    """``transforms.py:40-46``."""
    xy = xy[: xy.shape[0] // 8, ...] if reduce else xy
    return dihedral_8_augmentation(xy)


def symmetric_transform(x: Tensor, y: Tensor, phi: Tensor, offset: float = 0.5):
    """``transforms.py:49-71`` (``x``, ``y``: ``[B, N, 1]``; ``phi``: ``[B, 1, 1]``)."""
    xy = torch.cat((x, y), dim=-1).contiguous().float()
    nat.require_device(xy, phi)
    b, n, _ = xy.shape
    ph = phi.reshape(b).contiguous().float()
    out = torch.empty_like(xy)
    nat.call("co_symmetric_augment", b, n, nat.ptr(xy), nat.ptr(ph), float(offset),
             nat.ptr(out), nat.stream_of(xy))
    return out


def symmetric_augmentation(xy: Tensor, num_augment: int = 8, first_augment: bool = False):
    """``transforms.py:74-93``."""
    phi = torch.rand(xy.shape[0], device=xy.device) * 4 * math.pi
    if not first_augment:
        phi[: xy.shape[0] // num_augment] = 0.0
    x, y = xy[..., [0]], xy[..., [1]]
    return symmetric_transform(x, y, phi[:, None, None])


def min_max_normalize(x):
    """``transforms.py:96-97``."""
    return (x - x.min()) / (x.max() - x.min())


def get_augment_function(augment_fn: Union[str, callable]):
    """``transforms.py:100-107``."""
    if callable(augment_fn):
        return augment_fn
    if augment_fn == "dihedral8":
        return dihedral_8_augmentation_wrapper
    if augment_fn == "symmetric":
        return symmetric_augmentation
    raise ValueError(f"Unknown augment_fn: {augment_fn}. Available options: 'symmetric', "
                     "'dihedral8' or a custom callable")


class StateAugmentation:
    """``transforms.py:110-160``: augment ``feats`` of a TensorDict ``num_augment`` times
    (batchify layout, row ``r*B + b``)."""

    def __init__(self, num_augment: int = 8, augment_fn: Union[str, callable] = "symmetric",
                 first_aug_identity: bool = True, normalize: bool = False, feats: list = None):
        self.augmentation = get_augment_function(augment_fn)
        assert not (self.augmentation == dihedral_8_augmentation_wrapper and num_augment != 8), \
            "When using the `dihedral8` augmentation function, then num_augment must be 8"
        self.feats = ["locs"] if feats is None else feats
        self.num_augment = num_augment
        self.normalize = normalize
        self.first_aug_identity = first_aug_identity

    def __call__(self, td):
        td_aug = batchify(td, self.num_augment)
        for feat in self.feats:
            if not self.first_aug_identity:
                init_aug_feat = td_aug[feat][list(td.size()), 0].clone()
            aug_feat = self.augmentation(td_aug[feat], self.num_augment)
            if self.normalize:
                aug_feat = min_max_normalize(aug_feat)
            if not self.first_aug_identity:
                aug_feat[list(td.size()), 0] = init_aug_feat
            td_aug[feat] = aug_feat
        return td_aug
