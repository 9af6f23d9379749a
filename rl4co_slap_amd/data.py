"""Datasets and npz I/O of ``rl4co/data/{utils,dataset,generate_data}.py`` (SURVEY.md 8f
rank 4): feeding fixed validation / test sets to the envs.

The reference's dataset classes are mirrored for API parity; ``DeviceTdDataset`` is the
MI355X path: the whole set stays resident in HBM and a batch is assembled by one device
gather per column (``co_gather_by_index`` along the instance dim) instead of per-item
Python dicts re-stacked on the host.  npz files are read with the safe loader only.
"""
from __future__ import annotations

import os
from typing import Union

import numpy as np
import torch
from torch.utils.data import Dataset

from .td import TensorDict
from .utils.ops import gather_by_index


def load_npz_to_tensordict(filename):
    """``data/utils.py:11-19`` (``allow_pickle=False``: no code runs from the file)."""
    with np.load(filename, allow_pickle=False) as x:
        x_dict = {k: torch.as_tensor(x[k]) for k in x.files}
    batch_size = x_dict[list(x_dict.keys())[0]].shape[0]
    return TensorDict(x_dict, batch_size=[batch_size])


def save_tensordict_to_npz(tensordict, filename, compress: bool = False):
    """``data/utils.py:22-31``."""
    x_dict = {k: v.detach().cpu().numpy() for k, v in tensordict.items()}
    (np.savez_compressed if compress else np.savez)(filename, **x_dict)


def check_extension(filename, extension=".npz"):
    """``data/utils.py:34-38``."""
    if os.path.splitext(filename)[1] != extension:
        return filename + extension
    return filename


# -- generate_data.py (numpy global RNG, same draw order) ------------------------------
CAPACITIES = {10: 20.0, 15: 25.0, 20: 30.0, 30: 33.0, 40: 37.0, 50: 40.0, 60: 43.0, 75: 45.0,
              100: 50.0, 125: 55.0, 150: 60.0, 200: 70.0, 500: 100.0, 1000: 150.0}


def generate_tsp_data(dataset_size, tsp_size):
    """``generate_data.py:40-43``."""
    return {"locs": np.random.uniform(size=(dataset_size, tsp_size, 2)).astype(np.float32)}


def generate_vrp_data(dataset_size, vrp_size, capacities=None):
    """``generate_data.py:46-83``."""
    caps = dict(CAPACITIES)
    if capacities is not None:
        for k, v in capacities.items():
            if k in caps:
                caps[k] = v
    return {
        "depot": np.random.uniform(size=(dataset_size, 2)).astype(np.float32),
        "locs": np.random.uniform(size=(dataset_size, vrp_size, 2)).astype(np.float32),
        "demand": np.random.randint(1, 10, size=(dataset_size, vrp_size)).astype(np.float32),
        "capacity": np.full(dataset_size, caps[vrp_size]).astype(np.float32),
    }


# -- dataset.py ------------------------------------------------------------------------
class FastTdDataset(Dataset):
    """``dataset.py:8-31``: batched ``__getitems__`` on the TensorDict."""

    def __init__(self, td: TensorDict):
        self.data_len = td.batch_size[0]
        self.data = td

    def __len__(self):
        return self.data_len

    def __getitems__(self, idx):
        return TensorDict({k: v[idx] for k, v in self.data.items()}, batch_size=[len(idx)])

    def add_key(self, key, value):
        return ExtraKeyDataset(TensorDictDataset(self.data), value, key_name=key)

    @staticmethod
    def collate_fn(batch: Union[dict, TensorDict]):
        return batch


class TensorDictDataset(Dataset):
    """``dataset.py:34-66``: per-item dicts, stacked by ``collate_fn``."""

    def __init__(self, td: TensorDict):
        self.data_len = td.batch_size[0]
        self.data = [{key: value[i] for key, value in td.items()} for i in range(self.data_len)]

    def __len__(self):
        return self.data_len

    def __getitem__(self, idx):
        return self.data[idx]

    def add_key(self, key, value):
        return ExtraKeyDataset(self, value, key_name=key)

    @staticmethod
    def collate_fn(batch: Union[dict, TensorDict]):
        return TensorDict({key: torch.stack([b[key] for b in batch]) for key in batch[0].keys()},
                          batch_size=[len(batch)])


class ExtraKeyDataset(TensorDictDataset):
    """``dataset.py:69-86``: adds e.g. a REINFORCE baseline reward per item."""

    def __init__(self, dataset: TensorDictDataset, extra: torch.Tensor, key_name="extra"):
        self.data_len = len(dataset)
        assert self.data_len == len(extra), "Data and extra must be same length"
        self.data = dataset.data
        self.extra = extra
        self.key_name = key_name

    def __getitem__(self, idx):
        data = dict(self.data[idx])
        data[self.key_name] = self.extra[idx]
        return data


class TensorDictDatasetFastGeneration(Dataset):
    """``dataset.py:89-127``."""

    def __init__(self, td: TensorDict):
        self.data = td

    def __len__(self):
        return self.data.batch_size[0]

    def __getitems__(self, index):
        return TensorDict({key: item[index] for key, item in self.data.items()},
                          batch_size=[len(index)])

    def add_key(self, key, value):
        self.data.update({key: value})
        return self

    @staticmethod
    def collate_fn(batch: Union[dict, TensorDict]):
        return batch


class DeviceTdDataset(Dataset):
    """The whole set resident on the device; ``__getitems__(idx)`` gathers the batch rows
    of every column with the gfx950 gather kernel (one launch per column, indices on the
    device, no host round trip).  Use with ``torch.utils.data.DataLoader(ds,
    batch_size=..., collate_fn=ds.collate_fn)`` (batched fetching) or call
    ``__getitems__`` with a device index tensor directly."""

    def __init__(self, td: TensorDict, device=None):
        device = torch.device(device) if device is not None else td.device
        self.data = {k: v.to(device).contiguous() for k, v in td.items()}
        self.data_len = td.batch_size[0]
        self.device = device

    def __len__(self):
        return self.data_len

    def __getitems__(self, idx):
        idx = torch.as_tensor(idx, dtype=torch.int64).to(self.device)
        out = {}
        for k, v in self.data.items():
            if v.dim() == 1:  # [B] columns: view as [B, 1]
                out[k] = gather_by_index(v[:, None], idx, dim=0).squeeze(-1)
            else:
                out[k] = gather_by_index(v, idx, dim=0, squeeze=False)
        return TensorDict(out, batch_size=[idx.numel()])

    def add_key(self, key, value):
        self.data[key] = torch.as_tensor(value).to(self.device).contiguous()
        return self

    @staticmethod
    def collate_fn(batch: Union[dict, TensorDict]):
        return batch
