"""Per-env output pool for the step functions' fresh state tensors.

The reference's ``_step`` returns new tensors every step (out-of-place ``scatter``,
``clone``; SURVEY.md section 7 hard part 7), and a caller may keep any of them.  A
torch.empty on the HIP device costs ~1.2-1.7 us of host time and the drop-in decode loop
makes several per step, so the step functions take their outputs from here instead: a
pooled tensor is handed out again only when nothing but the pool refers to it -- no
Python reference (``sys.getrefcount``), no other C++ owner (``_use_count``: autograd,
DLPack, TensorDict internals) and no view of its storage (storage use count) -- which is
exactly when a fresh allocation would be indistinguishable from it.  Entries are keyed by
(shape, dtype, device, stream): a reused buffer is written by a kernel queued on the same
stream as every earlier reader, as the caching allocator's own reuse is.  At most
``max_keys`` keys are kept (least recently used dropped first), so shape changes (a last
partial batch, a validation batch size) do not accumulate device memory.
"""
import collections
import sys

import torch

_storage_use_count = getattr(torch._C, "_storage_Use_Count", None)


class OutputPool:
    def __init__(self, per_key: int = 4, device_types=("cuda",), max_keys: int = 16):
        self.per_key = per_key
        self.device_types = device_types
        self.max_keys = max_keys
        self._slots = collections.OrderedDict()

    def empty(self, shape, dtype, device, stream=0):
        """A tensor of this shape/dtype on ``device`` that no one else can observe."""
        if _storage_use_count is None or device.type not in self.device_types:
            return torch.empty(shape, dtype=dtype, device=device)
        key = (tuple(shape), dtype, device, stream)
        slots = self._slots.get(key)
        if slots is None:
            if len(self._slots) >= self.max_keys:
                self._slots.popitem(last=False)  # the least recently used key
            slots = self._slots[key] = []
        else:
            self._slots.move_to_end(key)
        getrc, suc = sys.getrefcount, _storage_use_count
        for t in slots:
            # references while checking: the slot list, the loop variable, getrefcount's
            # argument; the storage: the tensor and the temporary storage object
            if getrc(t) == 3 and t._use_count() == 1 and suc(t.untyped_storage()._cdata) == 2:
                return t
        t = torch.empty(shape, dtype=dtype, device=device)
        if len(slots) < self.per_key:
            slots.append(t)
        return t

    def clear(self):
        self._slots.clear()
