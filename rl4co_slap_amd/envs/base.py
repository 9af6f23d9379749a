"""``RL4COEnvBase`` surface for the HIP env engine.

Mirrors ``rl4co/envs/common/base.py:19-333`` (constructor kwargs, ``step``/``reset``
dispatch, ``get_reward`` wrapper, multistart helpers, dataset plumbing) without
TorchRL: ``reset`` reproduces TorchRL's merge of the ``_reset`` keys into the input
td plus ``done``/``terminated`` zeros ``[*B, 1]`` (the td dump of
``examples/test_slap.ipynb`` cell 13 shows both).

Differences from the reference, all deliberate:
* ``device`` defaults to ``"cuda"`` when a HIP device is present (the reference
  defaults to ``"cpu"``); the step/reward functions run only on the device.
* every tensor the reference allocates on the CPU by accident
  (``slap/env.py:107,114,135``, ``tsp/env.py:117``) lives on the td's device.
* data-dependent errors raised synchronously by the reference inside ``_step``
  (out-of-range scatter index) are recorded in a device status word and raised at
  the next ``get_reward``/``check_status`` (no per-step host sync).
"""
from __future__ import annotations

import abc
import os
from typing import Iterable, Optional

import torch

from .. import _native as nat
from ..td import TensorDict
from ..utils.ops import get_num_starts, select_start_nodes
from ..utils.pool import OutputPool


def _default_device():
    return "cuda" if torch.cuda.is_available() else "cpu"


class RL4COEnvBase(metaclass=abc.ABCMeta):
    batch_locked = False
    name = "base"

    def __init__(self, *, data_dir: str = "data/", train_file: str = None, val_file: str = None,
                 test_file: str = None, val_dataloader_names: list = None,
                 test_dataloader_names: list = None, check_solution: bool = True,
                 dataset_cls: callable = None, seed: int = None, device: str = None,
                 batch_size: torch.Size = None, run_type_checks: bool = False,
                 allow_done_after_reset: bool = False, _torchrl_mode: bool = False, **kwargs):
        kwargs.pop("name", None)
        if kwargs:
            raise TypeError(f"Unused keyword arguments: {', '.join(kwargs)}")
        self.device = torch.device(device if device is not None else _default_device())
        self.batch_size = torch.Size([] if batch_size is None else batch_size)
        self.data_dir = data_dir
        self.train_file = os.path.join(data_dir, train_file) if train_file is not None else None
        self._torchrl_mode = _torchrl_mode
        self.dataset_cls = dataset_cls

        def files(f):
            if f is None:
                return None
            if isinstance(f, Iterable) and not isinstance(f, str):
                return [os.path.join(data_dir, x) for x in f]
            return os.path.join(data_dir, f)

        self.val_file, self.test_file = files(val_file), files(test_file)
        self.val_dataloader_names = val_dataloader_names
        self.test_dataloader_names = test_dataloader_names
        self.check_solution = check_solution
        if seed is None:
            seed = torch.empty((), dtype=torch.int64).random_().item()
        self.set_seed(seed)
        # host-side knowledge about state tensors the env produced is kept ON those tensors
        # as (version, value) attributes, valid while the tensor's version counter is
        # unchanged: "_co_i" = the value every entry of a td["i"] holds, and the lower bound
        # on the steps before `done` can be all true under this env's own attribute name
        self._lb_attr = "_co_lb_" + self.name
        # the step functions' fresh outputs (utils/pool.py); CO_NO_POOL=1: torch.empty
        self._pool = None if os.environ.get("CO_NO_POOL") else OutputPool()

    # -- seeding (base.py:288-291) ---------------------------------------------
    def set_seed(self, seed: Optional[int]):
        self._set_seed(seed)
        return seed

    def _set_seed(self, seed: Optional[int]):
        self.rng = torch.manual_seed(seed)

    # -- step / reset (base.py:121-143) ----------------------------------------
    def step(self, td: TensorDict):
        if self._torchrl_mode:
            nxt = self._step(td.clone())
            td.set("next", nxt)
            return td
        td = self._step(td)
        return {"next": td}

    def reset(self, td: Optional[TensorDict] = None, batch_size=None) -> TensorDict:
        if batch_size is None:
            batch_size = self.batch_size if td is None else td.batch_size
        if td is None or td.is_empty():
            td = self.generator(batch_size=batch_size)
        batch_size = [batch_size] if isinstance(batch_size, int) else list(batch_size)
        if td.device is None or td.device != self.device:
            td = td.to(self.device)
        out = self._reset(td, batch_size=batch_size)
        if out is td:  # the env stored its reset state, done / terminated included, in td
            return td
        td.update(out)
        if "done" not in out:  # else the env's reset kernel wrote the zeros
            z = torch.zeros((2, *batch_size, 1), dtype=torch.bool, device=self.device)
            td.set("done", z[0])
            td.set("terminated", z[1])
        return td

    @abc.abstractmethod
    def _step(self, td):
        raise NotImplementedError

    @abc.abstractmethod
    def _reset(self, td=None, batch_size=None):
        raise NotImplementedError

    # -- reward / mask / validity (base.py:182-213) ----------------------------
    def get_reward(self, td, actions) -> torch.Tensor:
        """``base.py:182-188``: validity (if ``check_solution``) + reward, fused in one
        kernel pass; the reference's second validity pass inside ``_get_reward`` is
        the same predicate and is not repeated."""
        return self._get_reward(td, actions, check=self.check_solution)

    @abc.abstractmethod
    def _get_reward(self, td, actions, check: bool = False):
        raise NotImplementedError

    def get_action_mask(self, td):
        raise NotImplementedError

    def check_solution_validity(self, td, actions):
        raise NotImplementedError

    def get_num_starts(self, td):
        return get_num_starts(td, self.name)

    def select_start_nodes(self, td, num_starts):
        return select_start_nodes(td, self, num_starts)

    def replace_selected_actions(self, cur_actions, new_actions, selection_mask):
        raise NotImplementedError

    def local_search(self, td, actions, **kwargs):
        raise NotImplementedError(f"Local is not implemented yet for {self.name} environment")

    # -- datasets (base.py:236-286) --------------------------------------------
    def dataset(self, batch_size=[], phase="train", filename=None):
        """``base.py:236-270``: the phase's file(s) if set (a list gives a dict of named
        datasets), else generated instances; a missing file falls back to generation."""
        from ..data import TensorDictDataset

        cls = self.dataset_cls if self.dataset_cls is not None else TensorDictDataset
        f = getattr(self, f"{phase}_file") if filename is None else filename
        if f is None:
            td = self.generator(batch_size)
        else:
            try:
                if isinstance(f, Iterable) and not isinstance(f, str):
                    names = getattr(self, f"{phase}_dataloader_names")
                    return {name: cls(self.load_data(_f, batch_size)) for name, _f in zip(names, f)}
                td = self.load_data(f, batch_size)
            except FileNotFoundError:
                td = self.generator(batch_size)
        return cls(td)

    @staticmethod
    def load_data(fpath, batch_size=[]):
        import numpy as np

        with np.load(fpath, allow_pickle=False) as z:
            data = {k: torch.as_tensor(z[k]) for k in z.files}
        bs = next(iter(data.values())).shape[:1]
        return TensorDict(data, batch_size=bs)

    def transform(self):
        return self

    def render(self, *args, **kwargs):
        raise NotImplementedError

    def to(self, device):
        if device is None:
            return self
        self.device = torch.device(device)
        return self

    # -- status word -------------------------------------------------------------
    # While a decode loop collects its checks (``DecodingStrategy.defer_checks``), the
    # reward's status word is a word of the strategy's status tensor and its read is
    # deferred to the loop's single host read (``_checks``: the collector).
    _checks = None

    def status_word(self, device) -> torch.Tensor:
        """A zeroed status word for one of this env's kernels."""
        if self._checks is not None:
            return self._checks.env_word()
        return nat.scratch_status(device)

    def raise_for_status(self, status: torch.Tensor, messages):
        """Read a device status word (one host sync, which also carries the device's
        deferred word: an earlier out-of-range ``gather_by_index``) and raise the
        reference's error -- or, inside a decode loop's collection, register the messages
        for its single read."""
        if self._checks is not None and self._checks.owns(status):
            self._checks.add(messages)
            return
        d = nat.pending_deferred(status.device) if status.device.type != "cpu" else None
        if d is not None:
            bits, dbits = (int(v) for v in torch.cat([status.reshape(1), d]).tolist())
            nat.raise_deferred(dbits, status.device)
        else:
            bits = int(status.item())
        nat.release_status(status, (bits,))
        for bit, exc, msg in messages:
            if bits & bit:
                raise exc(msg)

    # -- i-tracking for the batch-wide `i.all() == 0` test ------------------------
    # (the record lives on the tensor: it dies with it, and an in-place change bumps the
    # version; one int (version << 32) | value, which csrc/pycall/co_torchstep.cpp reads
    # and writes in the tensor's instance dict)
    @staticmethod
    def _remember_i(t: torch.Tensor, value: int):
        t._co_i = (t._version << 32) | int(value)

    @staticmethod
    def _known_i(t: torch.Tensor):
        rec = getattr(t, "_co_i", None)
        if rec is None or (rec >> 32) != t._version:
            return None
        return rec & 0xFFFFFFFF

    # -- step outputs -------------------------------------------------------------
    def _out(self, shape, dtype, device, stream):
        """A fresh output tensor for a step function: from the env's pool when nothing
        else refers to a pooled one (indistinguishable from a new allocation), else
        torch.empty.  Host-side knowledge about a reused tensor's old contents is dropped."""
        if self._pool is None:
            return torch.empty(shape, dtype=dtype, device=device)
        t = self._pool.empty(shape, dtype, device, stream)
        d = t.__dict__
        d.pop("_co_i", None)
        d.pop(self._lb_attr, None)
        return t

    # -- done-poll lower bounds ---------------------------------------------------
    def _remember_lb(self, t: torch.Tensor, steps: int):
        setattr(t, self._lb_attr, (t._version << 32) | max(int(steps), 0))

    def _known_lb(self, t) -> Optional[int]:
        if not isinstance(t, torch.Tensor):
            return None
        rec = getattr(t, self._lb_attr, None)
        if rec is None or (rec >> 32) != t._version:
            return None
        return rec & 0xFFFFFFFF

    def poll_done(self, td):
        """The decode loop's ``td["done"].all()`` (``constructive/base.py:245``), read on
        the host: ``(all_done, k)``; when not all done, the next ``k - 1`` steps cannot
        make every instance done either, so the loop polls again after ``k`` steps (the
        same stopping step; fewer host syncs).  Default: ``k = 1``."""
        return bool(td["done"].all()), 1

    def min_steps_to_done(self, td) -> int:
        """A host-side lower bound on the env steps still needed before every instance
        of ``td`` can be done (0 = unknown: poll).  The decode loop skips the
        ``td["done"].all()`` host sync while fewer steps than this have been taken,
        which cannot change when it stops (``constructive/base.py:245``).  The bound
        comes from state tensors this env produced itself and nobody modified since
        (TSP: unvisited nodes, CVRP: unvisited nodes incl. the depot, SLAP: products
        left); anything else gives 0."""
        return 0

