"""DeviceTdDataset: batches gathered on the device equal host-side indexing for every
column dtype / rank, directly and through a DataLoader with batched fetching."""
import pytest
import torch

from rl4co_slap_amd import TensorDict
from rl4co_slap_amd.data import DeviceTdDataset

pytestmark = pytest.mark.gpu


def test_device_dataset_gather(dev):
    b = 1000
    td = TensorDict({"locs": torch.rand(b, 37, 2), "mask": torch.rand(b, 37) > 0.5,
                     "idx": torch.arange(b), "capacity": torch.rand(b),
                     "picklist": torch.randint(0, 20, (b, 20, 5))}, [b])
    ds = DeviceTdDataset(td, device=dev)
    assert len(ds) == b
    idx = torch.randint(0, b, (333,))
    got = ds.__getitems__(idx.to(dev))
    for k in td.keys():
        assert got[k].device.type == "cuda"
        assert torch.equal(got[k].cpu(), td[k][idx]), k
    ds.add_key("bl", torch.arange(b, dtype=torch.float32) * 2)
    dl = torch.utils.data.DataLoader(ds, batch_size=64, shuffle=False, collate_fn=ds.collate_fn)
    first = next(iter(dl))
    assert torch.equal(first["bl"].cpu(), torch.arange(64, dtype=torch.float32) * 2)
    assert torch.equal(first["locs"].cpu(), td["locs"][:64])
