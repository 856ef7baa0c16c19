"""GPU: the HIP path (in-kernel Philox noise, through the C ABI) against the committed golden
fixtures (tests/golden/golden_v1.npz). Tolerances: psi 1e-9 (2-norm, BASELINE north_star),
observables 1e-9; the in-kernel Box-Muller differs from the oracle's libm by <1e-15 per normal."""
import os
from math import sqrt

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402
from tests.golden import make_golden as MG  # noqa: E402

G = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_v1.npz"))


@pytest.mark.parametrize("name", list(MG.CASES))
def test_hip_path_matches_golden(name):
    ph = MG.CASES[name]
    st = Stepper(ph, MG.B, 0, seed=MG.SEED)
    psi = torch.from_numpy(G[f"{name}/psi0"].copy()).cuda()
    acts = G[f"{name}/actions"]
    qs, xs = [], []
    for c in range(MG.N_CHUNK):
        out = st.step(psi, torch.from_numpy(acts[c].copy()).cuda(), MG.CHUNK, want_q=True, want_fail=True)
        assert int(out["fail_step"].max()) == 0
        qs.append(out["q"].cpu().numpy())
        xs.append(out["x_mean"].cpu().numpy())
    w = 1.0 if ph.fock else sqrt(ph.grid_size)
    err = np.linalg.norm(psi.cpu().numpy() - G[f"{name}/psi"], axis=1) * w
    assert err.max() < 1e-9, err
    np.testing.assert_allclose(np.concatenate(xs), G[f"{name}/x_mean"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(np.concatenate(qs), G[f"{name}/q"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(st.moments(psi).cpu().numpy(), G[f"{name}/obs"], rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(st.x_expectation(psi).cpu().numpy(), G[f"{name}/x_expectation"], atol=1e-10)
    if ph.fock:
        np.testing.assert_allclose(st.phonon_number(psi).cpu().numpy(), G[f"{name}/phonon"], rtol=1e-10)
    else:
        np.testing.assert_allclose(st.energy(psi).cpu().numpy(), G[f"{name}/energy"], rtol=1e-9)
