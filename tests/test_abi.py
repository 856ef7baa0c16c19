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


def test_params_struct_matches_header(tmp_path):
    """_lib.QcParams mirrors qc_params exactly: same field order, and (compiled against the header)
    the same offsets and total size, including the precision field."""
    import shutil
    import subprocess
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib
    txt = open(os.path.join(ROOT, "include", "qcart.h")).read()
    body = re.search(r"typedef struct qc_params \{(.*?)\} qc_params;", txt, re.S).group(1)
    names = re.findall(r"^\s*(?:u?int(?:32|64)_t|double)\s+(\w+);", body, re.M)
    assert names == [f[0] for f in _lib.QcParams._fields_]
    assert "QC_FP32 = 1" in txt
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    src = tmp_path / "off.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "qcart.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof(qc_params, {n}));\n' for n in names)
                   + 'printf("%zu\\n", sizeof(qc_params));return 0;}\n')
    exe = tmp_path / "off"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [getattr(_lib.QcParams, n).offset for n in names] + [ctypes.sizeof(_lib.QcParams)]
    assert got == want


@pytest.mark.skipif(not os.path.exists(LIB), reason="libqcart.so not built")
def test_moment_order_range_is_validated_before_the_device():
    """get_moments orders 1..16 (at most 3 observables per lane of the env's wave); 17 is refused with the reason,
    before any device is touched (QO/setupC.py compiles any MOMENT >= 1)."""
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib
    p = _lib.QcParams()
    p.family, p.x_max, p.grid_size, p.lambda_, p.mass = 2, 8.5, 0.1, 0.04 * 3.14159, 1 / 3.14159
    p.gamma, p.dt, p.f_max, p.n_actions, p.batch, p.moment_order = 0.0314, 1 / 1440, 5.0, 21, 2, 17
    h = ctypes.c_void_p()
    rc = _lib.lib().qc_create(ctypes.byref(p), 0, ctypes.byref(h))
    assert rc == -1 and not h.value
    assert b"1..16" in _lib.lib().qc_last_error(None)


CLIENT = os.path.join(ROOT, "deepreinforcementlearningcontrolofquantumcartpoles_amd", "libqcart_client.so")


@pytest.mark.skipif(not os.path.exists(CLIENT), reason="libqcart_client.so not built")
def test_client_library_exports_every_declared_symbol():
    """libqcart_client.so (the step server's actor side, include/qcart_client.h): plain C, every declared
    symbol exported, and no HIP runtime linked (an actor process never creates a GPU context)."""
    import subprocess
    txt = open(os.path.join(ROOT, "include", "qcart_client.h")).read()
    syms = sorted(set(re.findall(r"^\s*(?:int|void|const char\*)\s+\*?(qcc_\w+)\s*\(", txt, re.M)))
    assert len(syms) >= 10
    L = ctypes.CDLL(CLIENT)
    for s in syms:
        assert hasattr(L, s), s
    deps = subprocess.run(["ldd", CLIENT], capture_output=True, text=True).stdout
    assert "amdhip" not in deps and "hsa" not in deps


def test_env_tail_args_struct_matches_header(tmp_path):
    """_lib.QcEnvTailArgs mirrors qc_env_tail_args (field order, offsets, size) compiled against the header."""
    import shutil
    import subprocess
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib
    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    names = [f[0] for f in _lib.QcEnvTailArgs._fields_]
    src = tmp_path / "tail.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "qcart.h"\nint main(void){\n'
                   + "".join(f'printf("%zu\\n", offsetof(qc_env_tail_args, {n}));\n' for n in names)
                   + 'printf("%zu\\n", sizeof(qc_env_tail_args));return 0;}\n')
    exe = tmp_path / "tail"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    want = [getattr(_lib.QcEnvTailArgs, n).offset for n in names] + [ctypes.sizeof(_lib.QcEnvTailArgs)]
    assert got == want
