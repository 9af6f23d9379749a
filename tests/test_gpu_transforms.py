"""GPU parity for the state augmentations of rl4co/data/transforms.py: dihedral-8
bit-exact, the SR-group transform within 2e-6 (cos/sin may differ from ATen's by 1 ulp)."""
import math

import pytest
import torch

from oracle import transforms as ot
from rl4co_slap_amd import TensorDict
from rl4co_slap_amd.utils import transforms as tr

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("b,n", [(1, 1), (5, 20), (64, 100), (33, 7)])
def test_dihedral8_exact(dev, b, n):
    xy = torch.rand(b, n, 2)
    got = tr.dihedral_8_augmentation(xy.to(dev)).cpu()
    assert torch.equal(got, ot.dihedral_8_augmentation(xy))


def test_symmetric_transform(dev):
    b, n = 96, 50
    xy = torch.rand(b, n, 2)
    phi = torch.rand(b) * 4 * math.pi
    phi[:12] = 0.0
    phi[12] = 2 * math.pi  # boundary of the reflection test
    want = ot.symmetric_transform(xy[..., [0]], xy[..., [1]], phi[:, None, None])
    x, y = xy.to(dev)[..., [0]], xy.to(dev)[..., [1]]
    got = tr.symmetric_transform(x, y, phi.to(dev)[:, None, None]).cpu()
    assert torch.allclose(got, want, rtol=0, atol=2e-6)
    assert torch.equal(got[:12], xy[:12])  # phi = 0 is the identity


def test_state_augmentation_dihedral(dev):
    b, n = 16, 20
    locs = torch.rand(b, n, 2)
    td = TensorDict({"locs": locs.to(dev), "x": torch.arange(b, device=dev)}, [b])
    aug = tr.StateAugmentation(num_augment=8, augment_fn="dihedral8")(td)
    assert aug["locs"].shape == (8 * b, n, 2)
    assert torch.equal(aug["locs"].cpu(), ot.dihedral_8_augmentation(locs))
    assert torch.equal(aug["x"].cpu(), torch.arange(b).repeat(8))  # batchify layout
