"""The C-ABI library loads and exports every symbol include/qcart.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "deepreinforcementlearningcontrolofquantumcartpoles_amd", "libqcart.so")


def declared_symbols():
    txt = open(os.path.join(ROOT, "include", "qcart.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*|uint64_t)\s+\*?(qc_\w+)\s*\(", txt, re.M)))


def test_header_declares_expected_surface():
    syms = declared_symbols()
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib
    assert set(syms) == set(_lib.EXPORTS)


@pytest.mark.skipif(not os.path.exists(LIB), reason="libqcart.so not built")
def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(LIB)
    for s in declared_symbols():
        assert hasattr(L, s), s
    L.qc_abi_version.restype = ctypes.c_int
    assert L.qc_abi_version() == 1


@pytest.mark.skipif(not os.path.exists(LIB), reason="libqcart.so not built")
def test_create_without_gpu_fails_loudly():
    """No CPU fallback: without a HIP device qc_create must return an error, not compute."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib
    p = _lib.QcParams()
    p.family, p.n_max, p.omega, p.gamma, p.dt, p.f_max, p.n_actions, p.batch = 1, 63, 3.14159, 6.28, 1 / 1440, 8.0, 21, 4
    h = ctypes.c_void_p()
    rc = _lib.lib().qc_create(ctypes.byref(p), 0, ctypes.byref(h))
    assert rc < 0 and not h.value
    assert b"HIP" in _lib.lib().qc_last_error(None) or rc == -3
