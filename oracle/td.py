"""Dict-backed TensorDict stand-in for the oracle (test infrastructure only).

Only the behaviour the hot path relies on is modelled:
* ``td[key]`` / ``td.set`` / ``td.update`` / ``td.get``;
* ``batch_size`` and ``clone``;
* TorchRL's ``EnvBase.reset`` merge: the keys returned by ``_reset`` are merged
  into the input td and ``done``/``terminated`` default to ``zeros([*B, 1], bool)``
  (evidence: the td dump of ``examples/test_slap.ipynb`` cell 13 output, where
  generator keys ``dist_mat``/``picklist`` survive reset next to ``done`` and
  ``terminated`` of shape ``[3, 1]``).
"""
from __future__ import annotations

import torch


class TD(dict):
    def __init__(self, data=None, batch_size=()):
        super().__init__(data or {})
        if isinstance(batch_size, int):
            batch_size = (batch_size,)
        self.batch_size = torch.Size(batch_size)

    def set(self, key, value):
        self[key] = value
        return self

    def update(self, other):  # noqa: D401 - dict.update returning self like TensorDict
        for k, v in other.items():
            self[k] = v
        return self

    def clone(self):
        return TD({k: v.clone() for k, v in self.items()}, self.batch_size)

    @property
    def device(self):
        for v in self.values():
            return v.device
        return None

    def is_empty(self):
        return len(self) == 0


def batchify_td(td: TD, repeats: int) -> TD:
    """``_batchify_single`` on every entry (``rl4co/utils/ops.py:11-16``)."""
    out = {}
    for k, v in td.items():
        s = v.shape
        out[k] = v.expand(repeats, *s).contiguous().view(s[0] * repeats, *s[1:])
    return TD(out, (td.batch_size[0] * repeats,))


def unbatchify_td(td: TD, repeats: int) -> TD:
    out = {}
    for k, v in td.items():
        s = v.shape
        out[k] = v.view(repeats, s[0] // repeats, *s[1:]).permute(1, 0, *range(2, len(s) + 1))
    return TD(out, (td.batch_size[0] // repeats, repeats))
