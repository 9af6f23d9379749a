"""The committed golden fixtures (tests/golden/*.npz) load with the safe
loader and are reproduced by the oracle: exact for indices / masks / bool state, 1e-6
for floats (CPU float kernels may differ in the last bit across hosts).  This pins the
oracle against drift; tests/test_gpu_golden.py runs the same vectors through the HIP
path."""
import importlib.util
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = sorted(f[:-4] for f in os.listdir(HERE) if f.endswith(".npz"))


def _maker():
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(HERE, "make_golden.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_fixture_set_complete():
    assert NAMES == sorted(["tsp20_b128_teacher", "tsp20_b128_nearest", "tsp100_b64_teacher",
                            "tsp100_b64_nearest", "cvrp20_b64_nearest", "cvrp100_b64_nearest",
                            "slap_b32_closest", "slap_b32_random", "decode_b256_n100_noclip",
                            "decode_b256_n100_clip10", "pomo_tsp20_b8"])


@pytest.fixture(scope="module")
def regenerated():
    return _maker().build_all()


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_fixture(regenerated, name):
    saved = np.load(os.path.join(HERE, name + ".npz"), allow_pickle=False)
    new = regenerated[name]
    assert sorted(saved.files) == sorted(new.keys())
    for k in saved.files:
        a, b = saved[k], np.asarray(new[k])
        assert a.shape == b.shape and a.dtype == b.dtype, (name, k)
        if np.issubdtype(a.dtype, np.floating):
            np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6, err_msg=f"{name}:{k}")
        else:
            np.testing.assert_array_equal(a, b, err_msg=f"{name}:{k}")


def test_fixture_invariants():
    """Size-independent properties the fixtures must satisfy on their own."""
    for n in ("tsp20_b128_teacher", "tsp20_b128_nearest", "tsp100_b64_teacher", "tsp100_b64_nearest"):
        f = np.load(os.path.join(HERE, n + ".npz"))
        acts = f["actions"]
        assert (np.sort(acts, 1) == np.arange(acts.shape[1])).all()  # permutations
        assert f["done"][-1].all() and not f["done"][:-1].any()
        assert (f["reward"] < 0).all()
    f = np.load(os.path.join(HERE, "cvrp100_b64_nearest.npz"))
    assert f["visited"].all() and f["done"][-1].all()
    assert (f["used_capacity"] <= f["vehicle_capacity"] + 1e-5).all()
    f = np.load(os.path.join(HERE, "slap_b32_closest.npz"))
    assert (f["assignment"] == f["actions"]).all()  # product t <- step t's location
