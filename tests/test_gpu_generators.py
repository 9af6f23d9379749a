"""On-device SLAP instance generation (co_slap_generate) equals the
host generator -- itself checked against the oracle's reference-loop restatement in
test_host_cpu.py -- bit-exact on every column, with the same RNG streams consumed."""
import numpy as np
import pytest
import torch

from rl4co_slap_amd.envs.slap import SLAPGenerator

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("params", [{}, {"n_aisles": 7, "n_locs": 9, "inter_aisle_dist": 2.4,
                                         "inter_loc_dist": 1.3, "n_products": 13}])
@pytest.mark.parametrize("dist", [True, False])
def test_slap_device_generator_matches_host(dev, params, dist):
    b = 37
    torch.manual_seed(5)
    np.random.seed(5)
    host = SLAPGenerator(materialize_dist_mat=dist, **params)(b)
    after_host = (torch.rand(1).item(), np.random.rand())
    torch.manual_seed(5)
    np.random.seed(5)
    devg = SLAPGenerator(materialize_dist_mat=dist, device=dev, **params)(b)
    after_dev = (torch.rand(1).item(), np.random.rand())
    assert after_host == after_dev  # the same RNG draws were consumed
    assert sorted(host.keys()) == sorted(devg.keys())
    for k in host.keys():
        assert devg[k].device.type == "cuda", k
        assert devg[k].dtype == host[k].dtype, k
        assert torch.equal(devg[k].cpu(), host[k]), k
