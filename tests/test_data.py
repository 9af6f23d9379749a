"""Dataset / npz I/O mirror of rl4co/data: numpy generator streams,
safe npz round trip, dataset classes and env.dataset's file / fallback logic."""
import numpy as np
import pytest
import torch

from rl4co_slap_amd import TensorDict
from rl4co_slap_amd import data as D


def test_generate_data_streams():
    np.random.seed(3)
    t = D.generate_tsp_data(5, 7)
    v = D.generate_vrp_data(4, 20)
    np.random.seed(3)
    assert np.array_equal(t["locs"], np.random.uniform(size=(5, 7, 2)).astype(np.float32))
    assert np.array_equal(v["depot"], np.random.uniform(size=(4, 2)).astype(np.float32))
    assert np.array_equal(v["locs"], np.random.uniform(size=(4, 20, 2)).astype(np.float32))
    assert np.array_equal(v["demand"], np.random.randint(1, 10, size=(4, 20)).astype(np.float32))
    assert (v["capacity"] == 30.0).all()
    assert D.generate_vrp_data(2, 20, capacities={20: 7.0})["capacity"][0] == 7.0


def test_npz_round_trip_and_datasets(tmp_path):
    td = TensorDict({"locs": torch.rand(6, 4, 2), "demand": torch.rand(6, 4),
                     "capacity": torch.full((6,), 3.0)}, [6])
    fn = D.check_extension(str(tmp_path / "x"))
    assert fn.endswith(".npz")
    D.save_tensordict_to_npz(td, fn, compress=True)
    back = D.load_npz_to_tensordict(fn)
    assert back.batch_size[0] == 6 and all(torch.equal(back[k], td[k]) for k in td.keys())
    ds = D.TensorDictDataset(td)
    batch = ds.collate_fn([ds[i] for i in (4, 1)])
    assert torch.equal(batch["locs"], td["locs"][[4, 1]])
    ex = ds.add_key("bl", torch.arange(6.0))
    assert ex[5]["bl"] == 5.0 and "bl" not in ds[5]
    fast = D.FastTdDataset(td).__getitems__([0, 5])
    assert torch.equal(fast["demand"], td["demand"][[0, 5]])
    fg = D.TensorDictDatasetFastGeneration(td).add_key("z", torch.zeros(6))
    assert fg.__getitems__([2])["z"].shape == (1,)


def test_env_dataset_files_and_fallback(tmp_path):
    from rl4co_slap_amd.envs import CVRPEnv

    np.random.seed(0)
    arrays = D.generate_vrp_data(5, 20)
    np.savez(tmp_path / "val.npz", **arrays)
    env = CVRPEnv(generator_params=dict(num_loc=20), data_dir=str(tmp_path),
                  val_file="val.npz", test_file=["val.npz", "val.npz"],
                  test_dataloader_names=["a", "b"], device="cpu")
    val = env.dataset(phase="val")
    assert len(val) == 5
    # cvrp/env.py:192-199: demand normalised by the capacity on load
    assert torch.allclose(val[0]["demand"], torch.as_tensor(arrays["demand"][0] / 30.0))
    tests = env.dataset(phase="test")
    assert sorted(tests) == ["a", "b"] and len(tests["a"]) == 5
    gen = env.dataset(batch_size=[3], phase="val", filename=str(tmp_path / "missing.npz"))
    assert len(gen) == 3  # missing file -> generated instances
