import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and the built gfx950 library")


def pytest_collection_modifyitems(config, items):
    import torch

    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def dev():
    import torch

    from rl4co_slap_amd import _native

    if os.environ.get("CO_TEST_LIB"):  # a tuning variant (tools/build_variants.sh)
        _native.LIB_PATH = os.environ["CO_TEST_LIB"]
    else:  # test infrastructure builds a missing / stale in-tree library; the product
        # itself never builds and fails loudly without it
        from rl4co_slap_amd.csrc.build import build

        build(force=False)
    _native.load()
    return torch.device("cuda:0")
