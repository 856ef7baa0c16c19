"""CPU: the oracle reproduces the committed golden fixtures (tests/golden/golden_v1.npz, made by
tests/golden/make_golden.py). Guards the checker itself against drift; the GPU path is held to the
same fixtures in tests/test_gpu_golden.py. Reference parity is pinned separately, at the
reference's MKL boundary (tests/test_mkl_fixtures.py)."""
import os

import numpy as np
import pytest

from tests.golden import make_golden as MG

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))


def test_philox_and_normals_golden(oracle_mod):
    for c, k, o in zip(G["philox/ctr"], G["philox/key"], G["philox/out"]):
        assert np.array_equal(oracle_mod.philox(c, k), o)
    for (s, e, k), r in zip(G["normals/ids"], G["normals/out"]):
        np.testing.assert_allclose(oracle_mod.normals(int(s), int(e), int(k)), r, rtol=0, atol=1e-15)


@pytest.mark.parametrize("name", list(MG.CASES))
def test_oracle_reproduces_golden(name):
    got = MG.make_case(name, MG.CASES[name])
    for key, ref in got.items():
        np.testing.assert_allclose(ref, G[key], rtol=0, atol=1e-13, equal_nan=True, err_msg=key)
