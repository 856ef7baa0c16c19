"""GPU parity of the measurement-record input mode (qc_record) against the
pure-Python restatement of the reference's lists (oracle/measure.py, IHO/main_parallel.py:270-309).

Bar: bit-exact float32 (network input, forces_to_store, experience rows) from the same fp64 q stream.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.env import BatchedEnv  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.measurements import MeasurementRecord  # noqa: E402
from oracle.measure import MeasureLists  # noqa: E402


@pytest.mark.parametrize("family,time_steps,n_con,scaling", [
    (cfg.IHO, 1440, 18, 0.7),     # IHO defaults: L = 5760, coarse_grain 1, m = 80 (float4 path)
    (cfg.HO, 2880, 18, 1.0),      # coarse_grain 2: interval 160, m = 80, L = 4320
    (cfg.IHO, 1440, 16, 1.3),     # interval 90: m = 90 (scalar path), L = 5760 = 64 * 90
])
def test_record_matches_reference_lists(family, time_steps, n_con, scaling):
    ph = cfg.DEFAULTS[family].with_(n_max=63, time_steps=time_steps, n_con=n_con)
    B = 6
    st = Stepper(ph, B, 0, seed=11)
    psi = st.new_state()
    st.reset(psi, 1, arg0=8)
    rec = MeasurementRecord(st, input_scaling=scaling)
    L, m, K, ci = rec.read_length, rec.m, rec.K, ph.control_interval
    orc = [MeasureLists(L, ci, rec.coarse_grain, scaling) for _ in range(B)]
    rows = torch.zeros((B, rec.row_len), dtype=torch.float32, device=st.device)
    rng = np.random.default_rng(3)
    for k in range(8):
        acts = np.full(B, 10, dtype=np.int32) if k == 0 else rng.integers(0, 21, B).astype(np.int32)
        mode = np.full(B, 2 if k == 0 else 1, dtype=np.uint8)
        if k == 5:
            mode[1] = 0            # frozen: untouched, no row
            mode[2] = 2            # a new episode for env 2
            orc[2].reset()
        out = st.step(psi, torch.from_numpy(acts).cuda(), ci, want_q=True,
                      env_steps=torch.from_numpy((mode > 0).astype(np.int32) * ci).cuda())
        q = out["q"].cpu().numpy()
        reward = rng.normal(size=B).astype(np.float32)
        before = (rec.hist.clone(), rows.clone())
        rec.record(out["q"], torch.from_numpy(acts).cuda(), mode=torch.from_numpy(mode).cuda(),
                   reward=torch.from_numpy(reward).cuda(), rows=rows)
        hist, frc, rw = rec.hist.cpu().numpy(), rec.forces.cpu().numpy(), rows.cpu().numpy()
        for e in range(B):
            if mode[e] == 0:
                assert torch.equal(rec.hist[e], before[0][e]) and torch.equal(rows[e], before[1][e])
                continue
            f = ph.force(int(acts[e]))
            for s in range(ci):
                orc[e].physics_step(float(q[s, e]), f)
            row_ref, net_ref = orc[e].control_step(f, int(acts[e]), float(reward[e]))
            assert row_ref.shape == (rec.row_len,)
            np.testing.assert_array_equal(rw[e], row_ref)
            np.testing.assert_array_equal(hist[e], net_ref)
            np.testing.assert_array_equal(frc[e], row_ref[L + m:L + m + K + 1])


def test_env_measurement_mode_loop():
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    B = 16
    env = BatchedEnv(ph, B, 0, seed=5, input="measurements", input_scaling=0.5)
    obs = env.reset()
    L, m, K = env.rec.read_length, env.rec.m, env.rec.K
    assert obs.shape == (B, 2, L) and L == 5760
    # after the zero-force first interval: m measurements, zero forces, the rest of the record empty
    assert bool((obs[:, 1] == 0).all()) and bool((obs[:, 0, m:] == 0).all())
    for k in range(4):
        a = torch.randint(0, 21, (B,), dtype=torch.int32, device=env.dev)
        prev = env.rec.hist[:, 0].clone()
        obs, r, done, info = env.step(a)
        rows = info["rows"]
        live = ~done
        assert torch.equal(rows[live, :L], obs[live, 0])
        assert torch.equal(rows[:, L:L + m], prev[:, L - m:])
        fs = (a.double().sub(10) * 0.8 * 0.5).float()
        assert torch.equal(rows[:, L + m], fs)
        assert torch.equal(rows[:, -2], a.float()) and torch.equal(rows[:, -1], r)
        assert torch.equal(obs[live, 1, :m], fs[live, None].expand(-1, m))


def test_record_out_of_range_action_is_reported():
    """qc_record clamps an out-of-range action on the device and raises the handle's error word, so the
    next check() reports it like a bad qc_step action (no silent clamping)."""
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    B = 4
    st = Stepper(ph, B, 0, seed=2)
    psi = st.new_state()
    st.reset(psi, 1, arg0=8)
    rec = MeasurementRecord(st)
    ok = torch.full((B,), 10, dtype=torch.int32, device="cuda")
    out = st.step(psi, ok, ph.control_interval, want_q=True)
    rec.record(out["q"], ok)
    st.check()
    bad = torch.tensor([10, 25, 3, 10], dtype=torch.int32, device="cuda")
    rec.record(out["q"], bad)
    with pytest.raises(ValueError, match="actions must lie"):
        st.check()
    st.check()      # cleared
    assert torch.isfinite(rec.hist).all()
