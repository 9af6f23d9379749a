"""TensorDict: the real ``tensordict.TensorDict`` when installed, else a minimal
dict-backed stand-in with the surface the env API and the decode loop use.

The stand-in models: key access/set/update/get, ``batch_size``/``shape``,
``device``/``to``, ``clone``, ``is_empty``, ``exclude``, batch indexing, and the
``expand``/``contiguous``/``view``/``permute`` used by ``batchify``/``unbatchify``
(``rl4co/utils/ops.py:11-62``).  Leading dims of every entry are the batch dims.
"""
from __future__ import annotations

import torch

class RepeatedRows:
    """A batchified ``[S*B, ...]`` entry kept as its ``[B, ...]`` rows (multistart layout
    ``e = s*B + b`` reads row ``e % B``): ``batchify`` (``rl4co/utils/ops.py:16``,
    ``x.expand(S, ...).contiguous()``) stores entries this way, and the copy is made only
    when something reads the entry through the TensorDict.  The env kernels that accept
    the row-index scheme (the TSP reward's ``locs_batch``) read ``base`` directly
    (``TensorDict.get_raw``), so an unread ``locs`` is never replicated (655 MB at POMO
    config 5 on one GPU)."""

    __slots__ = ("base", "repeats", "_version")

    def __init__(self, base: torch.Tensor, repeats: int):
        self.base, self.repeats = base, repeats
        # the reference copies at batchify time; the lazy copy is only the same values
        # while the source is unchanged (an in-place write bumps its version)
        self._version = base._version

    def source(self) -> torch.Tensor:
        """``base`` after checking it was not written in place since ``batchify`` (the
        values the reference's copy holds would be lost: raise instead of reading them)."""
        if self.base._version != self._version:
            raise RuntimeError(
                "batchify: the source tensor was modified in place after batchify; the "
                "lazy (zero-copy) multistart entry can no longer reproduce the copy the "
                "reference makes at batchify time. Set CO_EAGER_BATCHIFY=1 to copy eagerly.")
        return self.base

    @property
    def shape(self):
        return torch.Size((self.repeats * self.base.shape[0], *self.base.shape[1:]))

    @property
    def device(self):
        return self.base.device

    def materialize(self) -> torch.Tensor:
        self.source()
        s = self.base.shape
        return self.base.expand(self.repeats, *s).contiguous().view(s[0] * self.repeats, *s[1:])


try:  # pragma: no cover - exercised only where tensordict is installed
    from tensordict import TensorDict  # type: ignore

    HAVE_TENSORDICT = True
except ImportError:  # the stand-in
    HAVE_TENSORDICT = False

    class TensorDict(dict):
        def __init__(self, source=None, batch_size=None, device=None):
            super().__init__()
            if batch_size is None:
                batch_size = ()
            if isinstance(batch_size, int):
                batch_size = (batch_size,)
            self.batch_size = torch.Size(batch_size)
            self._device = torch.device(device) if device is not None else None
            for k, v in (source or {}).items():
                self[k] = v

        def __setitem__(self, key, value):
            if self._device is not None and isinstance(value, torch.Tensor) and value.device != self._device:
                value = value.to(self._device)
            super().__setitem__(key, value)

        def __getitem__(self, key):
            if isinstance(key, str):
                v = super().__getitem__(key)
                if isinstance(v, RepeatedRows):  # first read: make the batchify copy
                    v = v.materialize()
                    super().__setitem__(key, v)
                return v
            out = {k: v[key] for k, v in self.items()}
            ref = torch.empty(self.batch_size, device="meta")[key]
            return TensorDict(out, ref.shape, self._device)

        def __iter__(self):  # keys; also keeps dict(td) off the raw-value fast path
            return iter(list(super().keys()))

        def items(self):
            return [(k, self[k]) for k in list(super().keys())]

        def values(self):
            return [self[k] for k in list(super().keys())]

        def get_raw(self, key, default=None):
            """The stored entry without materialising a lazy batchify (``RepeatedRows``)."""
            return super().get(key, default)

        def is_lazy(self, key) -> bool:
            return isinstance(super().get(key), RepeatedRows)

        # -- tensordict-like API -------------------------------------------------
        def set(self, key, value):
            self[key] = value
            return self

        def get(self, key, default=None):
            return self[key] if key in self else default

        def update(self, other, **kw):  # noqa: D401
            for k in list(other.keys()):
                self[k] = other[k]
            for k, v in kw.items():
                self[k] = v
            return self

        @property
        def shape(self):
            return self.batch_size

        @property
        def device(self):
            if self._device is not None:
                return self._device
            for v in dict.values(self):
                if isinstance(v, (torch.Tensor, RepeatedRows)):
                    return v.device
            return None

        def to(self, device):
            device = torch.device(device)
            return TensorDict({k: v.to(device) for k, v in self.items()}, self.batch_size, device)

        def cuda(self):
            return self.to("cuda")

        def cpu(self):
            return self.to("cpu")

        def clone(self):
            return TensorDict({k: v.clone() for k, v in self.items()}, self.batch_size, self._device)

        def is_empty(self):
            return len(self) == 0

        def exclude(self, *keys):
            return TensorDict({k: v for k, v in self.items() if k not in keys}, self.batch_size,
                              self._device)

        def select(self, *keys):
            return TensorDict({k: self[k] for k in keys}, self.batch_size, self._device)

        def detach(self):
            return TensorDict({k: v.detach() for k, v in self.items()}, self.batch_size, self._device)

        def numel(self):
            n = 1
            for s in self.batch_size:
                n *= s
            return n

        # -- batch-dim reshaping used by batchify / unbatchify ------------------
        def _map(self, fn, new_batch):
            return TensorDict({k: fn(v) for k, v in self.items()}, new_batch, self._device)

        def expand(self, *shape):
            shape = tuple(shape[0]) if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)) else shape
            nb = len(self.batch_size)
            extra = len(shape) - nb
            return self._map(lambda v: v.expand(*shape, *v.shape[nb:]) if extra >= 0 else v,
                             torch.Size(shape))

        def contiguous(self):
            return self._map(lambda v: v.contiguous(), self.batch_size)

        def view(self, *shape):
            shape = tuple(shape[0]) if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)) else shape
            nb = len(self.batch_size)
            new = torch.empty(self.batch_size, device="meta").view(*shape).shape
            return self._map(lambda v: v.view(*new, *v.shape[nb:]), new)

        def permute(self, *dims):
            dims = tuple(dims[0]) if len(dims) == 1 and isinstance(dims[0], (tuple, list)) else dims
            nb = len(self.batch_size)
            new = torch.Size([self.batch_size[d] for d in dims])
            return self._map(lambda v: v.permute(*dims, *range(nb, v.dim())), new)

        def __repr__(self):
            fields = ", ".join(f"{k}: {tuple(v.shape)}" for k, v in dict.items(self))
            return f"TensorDict({{{fields}}}, batch_size={tuple(self.batch_size)}, device={self.device})"


def set_many(td, entries: dict):
    """``td.update(entries)`` for values already on the device of ``td``'s own tensors (a
    step's outputs): the stand-in stores them without re-checking each value's device."""
    if not HAVE_TENSORDICT and type(td) is TensorDict:
        dict.update(td, entries)
    else:
        td.update(entries)
    return td
