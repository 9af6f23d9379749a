"""Build provenance (VERDICT r1 "build provenance is not visible"): the device library
carries the sha256 of the sources it was compiled from (co_build_provenance, written by
csrc/build.py), and the library this GPU run loaded must have been built from the
sources of this tree."""
import pytest

from rl4co_slap_amd import _native as nat

pytestmark = pytest.mark.gpu


def test_loaded_library_was_built_from_this_tree(dev):
    info = nat.provenance()
    print("co_build_provenance:", info)
    assert info["arch"] == "gfx950"
    assert info["matches_tree"] is True, info
