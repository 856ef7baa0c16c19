"""GPU parity: the HIP path (through the C ABI) against the CPU restatement (oracle/) on identical
inputs and identical Wiener noise.

Tolerance (BASELINE.json north_star): ||psi_GPU - psi_ref||_2 < 1e-9 after 1000 steps, fp64.
The oracle is the checker only; it is pinned at the reference's MKL boundary (tests/test_mkl_fixtures.py,
oracle/qcart_oracle.h).
"""
from math import pi, sqrt

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402

TOL_1000 = 1e-9


def oracle_sys(oracle_mod, ph):
    return oracle_mod.OracleSystem(ph.family, n_max=ph.n_max, omega=ph.omega, x_max=ph.x_max,
                                   grid_size=ph.grid_size, lambda_=ph.lambda_, mass=ph.mass,
                                   moment_order=ph.moment_order, a_mode=ph.a_mode)


def init_states(osys, ph, B, seed=1234):
    if ph.fock:
        return np.stack([osys.fock_random_state(seed, e, 16) for e in range(B)])
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(B):
        psi = osys.gaussian_packet(rng.uniform(-0.3, 0.3), rng.uniform(-1, 1), rng.uniform(0.7, 1.3))
        psi /= np.linalg.norm(psi) * sqrt(ph.grid_size)
        out.append(psi)
    return np.stack(out)


def wnorm(ph, v):
    return np.linalg.norm(v, axis=-1) * (sqrt(ph.grid_size) if not ph.fock else 1.0)


CASES = {
    "iho64": cfg.DEFAULTS[cfg.IHO].with_(n_max=63),
    "iho181": cfg.DEFAULTS[cfg.IHO],
    # omega != pi: the step kernel's X rel+- through X^2 = -H/omega + diag(d) at another omega
    "iho181_w2": cfg.DEFAULTS[cfg.IHO].with_(omega=2.0),
    "iho512": cfg.DEFAULTS[cfg.IHO].with_(n_max=511),
    # gamma = 2 pi at N = 512 needs dt = 1/2880 for 1000 physical steps: at 1/1440 rounding in the top
    # Fock levels grows until the run blows up after ~700 steps (oracle and MKL-ordered stepper alike;
    # tests/golden/make_mkl_fixtures.py), 5 of 8 PD-controlled envs Fail
    "iho512_dt2": cfg.DEFAULTS[cfg.IHO].with_(n_max=511, time_steps=2880),
    "iho512_exact": cfg.DEFAULTS[cfg.IHO].with_(n_max=511, a_mode=1),
    "iho64_g05": cfg.DEFAULTS[cfg.IHO].with_(n_max=63, gamma=0.5 * pi),
    "iho512_g05": cfg.DEFAULTS[cfg.IHO].with_(n_max=511, gamma=0.5 * pi),
    "iho512_exact_g05": cfg.DEFAULTS[cfg.IHO].with_(n_max=511, gamma=0.5 * pi, a_mode=1),
    # N = 1024: the largest fp64 instantiation (R = 16 rows per lane, one wave per SIMD; the opt-in
    # two-waves-per-env pair kernel was measured slower and removed)
    "iho1024_g05": cfg.DEFAULTS[cfg.IHO].with_(n_max=1023, gamma=0.5 * pi),
    "ho256": cfg.DEFAULTS[cfg.HO].with_(n_max=255),
    "ho71": cfg.DEFAULTS[cfg.HO],
    "qo171": cfg.DEFAULTS[cfg.QO],
    "iqo513": cfg.DEFAULTS[cfg.IQO].with_(x_max=12.8),
    # C3 grid: x_n = 1025 (R = 17). On this fine grid (h = 8.5/512) the scheme is only stable for dt <=
    # 1/11520 (the oracle Fails every env within 1000 steps at 1/1440, 1/2880 and 1/5760): parity runs use
    # that dt (throughput is dt-independent)
    "qo1025": cfg.BENCH_CONFIGS["C3"]["physics"].with_(time_steps=11520),
}


def pd_actions(osys, ph, states):
    """Saturated PD feedback F = -(2<x> + 2<p>) on the 21 force levels (classically critically damped
    for H = w/2 (p^2 - x^2) - w F x). With gamma = pi/2 it keeps the cartpole physical for the
    1000-step parity runs (the reference's own LQG, IHO/main_parallel.py:194-206, does not at
    gamma = 2 pi from these states)."""
    half = ph.n_actions // 2
    acts = []
    for psi in states:
        x, p = osys.moments(psi)[:2]
        f = min(max(-(2 * x + 2 * p), -ph.f_max), ph.f_max)
        acts.append(round(f / (ph.f_max / half)) + half)
    return np.array(acts, dtype=np.int32)


def run_pair(oracle_mod, ph, steps, B, act_lo, act_hi, chunk=80, seed=7, policy="random"):
    """GPU vs oracle in control-interval chunks with per-chunk actions (random or LQG) and injected
    noise. Returns (max error over envs that never Failed, alive mask, per-env first Fail step)."""
    osys = oracle_sys(oracle_mod, ph)
    psi0 = init_states(osys, ph, B)
    if policy == "pd":                       # the reference's reset: |0> (IHO/main_parallel.py:231-232)
        psi0 = np.zeros_like(psi0)
        psi0[:, 0] = 1.0
    rng = np.random.default_rng(seed)
    st = Stepper(ph, B, 0)
    ref = psi0.copy()
    psi = torch.from_numpy(psi0.copy()).cuda()
    alive = np.ones(B, bool)
    first_fail = np.zeros(B, np.int64)
    worst = 0.0
    done = 0
    while done < steps:
        n = min(chunk, steps - done)
        acts = rng.integers(act_lo, act_hi + 1, size=B).astype(np.int32)
        if policy == "pd":
            acts = pd_actions(osys, ph, ref)
        noise = rng.standard_normal((n, B, 2))
        f_ref, q_ref, xm_ref = osys.run_batch(ref, acts, ph.f_max, n, ph.dt, ph.gamma, noise=noise, want_q=True,
                                              n_threads=8)
        out = st.step(psi, torch.from_numpy(acts).cuda(), n, noise=torch.from_numpy(noise).cuda(), want_q=True)
        f_got = out["fail_step"].cpu().numpy()
        # the Fail flag (check_boundary_error) must agree while the trajectories are physical
        assert np.array_equal(f_got[alive], f_ref[alive]), (f_got, f_ref)
        xm, qq = out["x_mean"].cpu().numpy(), out["q"].cpu().numpy()
        # an env is compared up to the step at which it Failed (the reference ends the episode at
        # the next control step, IHO/main_parallel.py:243-267); past that psi is truncation noise
        for e in np.nonzero(alive)[0]:
            upto = n if f_ref[e] == 0 else f_ref[e] - 1
            np.testing.assert_allclose(xm[:upto, e], xm_ref[:upto, e], atol=1e-9)
            np.testing.assert_allclose(qq[:upto, e], q_ref[:upto, e], atol=1e-7)
        err = wnorm(ph, psi.cpu().numpy() - ref)
        newly = alive & (f_ref > 0)
        first_fail[newly] = done + f_ref[newly]
        alive &= f_ref == 0
        if alive.any():
            worst = max(worst, float(err[alive].max()))
        done += n
    return worst, alive, first_fail


@pytest.mark.parametrize("name,steps,B,policy", [
    ("iho64", 1000, 8, "pd"), ("iho181", 1000, 8, "random"), ("iho181_w2", 1000, 8, "random"),
    ("iho512_g05", 1000, 8, "pd"),
    # the metric's own physics (N = 512, gamma = 2 pi, dt = 1/1440) as far as it stays physical: 8 control intervals,
    # 7 of 8 PD-controlled envs physical, ~1e-14 (tools/probe_metric_parity_len.py: 5.6e-13 at 720 steps with 4 left;
    # past ~700 steps the top Fock levels' rounding blows the trajectories up in the oracle too)
    ("iho512", 640, 8, "pd"),
    ("iho512_dt2", 1000, 8, "pd"), ("iho512_exact_g05", 1000, 4, "pd"),
    ("ho256", 1000, 6, "random"), ("ho71", 1000, 8, "random"), ("qo171", 1000, 6, "random"),
    ("iqo513", 1000, 4, "random"), ("qo1025", 1000, 3, "random"), ("iho1024_g05", 1000, 4, "pd"),
])
def test_psi_parity_injected_noise(oracle_mod, name, steps, B, policy):
    """||psi_GPU - psi_ref||_2 < 1e-9 after 1000 steps (640 at the metric's own physics) (fp64) for every env whose trajectory stays
    physical (no boundary Fail); Fail steps themselves must agree. Every case must keep at least half of
    its envs physical to step 1000, so the 1000-step bound is never vacuous (random forces are drawn
    from the middle 7 levels for the inverted oscillator, whose pole falls under full pushes; the PD
    policy keeps it up from |0>)."""
    ph = CASES[name]
    lo, hi = (7, 13) if ph.family == cfg.IHO else (0, 20)
    worst, alive, _ = run_pair(oracle_mod, ph, steps, B, lo, hi, policy=policy)
    print(f"{name}: {int(alive.sum())}/{B} envs physical at step {steps}, max |dpsi| {worst:.2e}")
    assert alive.sum() >= B // 2, f"only {int(alive.sum())}/{B} envs stayed physical to step {steps}"
    assert worst < TOL_1000, worst


# every rows-per-lane instantiation, at sizes whose row count is not a multiple of the lane count (ragged
# padding: the grid's flushed padding rows at every N mod R, Lᵀ reads reaching 2-4 lanes ahead at R < kl),
# with a ragged batch of 3 envs
EDGE_SIZES = [
    ("iho31_R1", cfg.DEFAULTS[cfg.IHO].with_(n_max=30)), ("iho101_R2", cfg.DEFAULTS[cfg.IHO].with_(n_max=100)),
    ("iho151_R3", cfg.DEFAULTS[cfg.IHO].with_(n_max=150)), ("iho201_R4", cfg.DEFAULTS[cfg.IHO].with_(n_max=200)),
    ("iho401_R8", cfg.DEFAULTS[cfg.IHO].with_(n_max=400)), ("iho701_R16", cfg.DEFAULTS[cfg.IHO].with_(n_max=700)),
    ("ho41_R1", cfg.DEFAULTS[cfg.HO].with_(n_max=40)), ("ho101_R2", cfg.DEFAULTS[cfg.HO].with_(n_max=100)),
    ("ho201_R4", cfg.DEFAULTS[cfg.HO].with_(n_max=200)), ("ho401_R8", cfg.DEFAULTS[cfg.HO].with_(n_max=400)),
    ("qo35_R1", cfg.DEFAULTS[cfg.QO].with_(grid_size=0.5)), ("qo85_R2", cfg.DEFAULTS[cfg.QO].with_(grid_size=0.2)),
    ("qo285_R5", cfg.DEFAULTS[cfg.QO].with_(grid_size=0.06)),
    ("qo567_R9", cfg.DEFAULTS[cfg.QO].with_(grid_size=0.03, time_steps=5760)),
    ("qo1063_R17", cfg.DEFAULTS[cfg.QO].with_(grid_size=0.016, time_steps=11520)),
    ("iqo301_R5", cfg.DEFAULTS[cfg.IQO].with_(x_max=7.5)),
]


@pytest.mark.parametrize("name,ph", EDGE_SIZES, ids=[n for n, _ in EDGE_SIZES])
def test_psi_parity_every_rows_per_lane(oracle_mod, name, ph):
    """20 steps of every rows-per-lane instantiation at a ragged size and batch: psi, Fail, <x> and q equal
    the oracle's (fp64, injected noise, random force slots)."""
    lo, hi = (7, 13) if ph.family == cfg.IHO else (0, 20)
    worst, alive, _ = run_pair(oracle_mod, ph, 20, 3, lo, hi, chunk=20)
    assert alive.sum() >= 2, f"{name}: only {int(alive.sum())}/3 envs physical"
    assert worst < 1e-11, (name, worst)


def test_psi_parity_inkernel_philox(oracle_mod):
    """In-kernel Philox4x32-10 noise keyed by (seed, global env id, step) reproduces the oracle's."""
    ph = CASES["iho181"]
    B, steps, seed, off = 5, 200, 99, 1000
    osys = oracle_sys(oracle_mod, ph)
    psi0 = init_states(osys, ph, B)
    acts = np.arange(B, dtype=np.int32) * 4
    ref = psi0.copy()
    osys.run_batch(ref, acts, ph.f_max, steps, ph.dt, ph.gamma, seed=seed, env_offset=off, step0=0, n_threads=4)
    st = Stepper(ph, B, 0, seed=seed, env_offset=off)
    psi = torch.from_numpy(psi0).cuda()
    st.step(psi, torch.from_numpy(acts).cuda(), 120)
    st.step(psi, torch.from_numpy(acts).cuda(), 80)   # counter continues across calls
    assert st.step_counter == 200
    assert wnorm(ph, psi.cpu().numpy() - ref).max() < 1e-10


def test_split_calls_equal_and_deterministic():
    ph = CASES["iho512"]
    B = 8
    st1 = Stepper(ph, B, 0, seed=5)
    st2 = Stepper(ph, B, 0, seed=5)
    a = st1.new_state()
    st1.reset(a, 1, arg0=16)
    b = a.clone()
    acts = torch.randint(0, 21, (B,), dtype=torch.int32, device="cuda")
    st1.step(a, acts, 80)
    st2.step(b, acts, 30)
    st2.step(b, acts, 50)
    # <x> of the first step of a call is recomputed from the normalised psi, inside a call it is
    # carried from the normalisation reduction: equal to rounding, not bitwise
    assert float((a - b).abs().max()) < 1e-13
    # identical call sequences are bitwise reproducible
    c = st1.new_state()
    st1.reset(c, 1, arg0=16)
    st1.step_counter = 0
    st1.step(c, acts, 80)
    assert torch.equal(a, c)


def test_shard_invariance_bitwise():
    """1 handle x 8 envs == 2 handles x 4 envs with env_offset (multi-GPU sharding contract)."""
    ph = CASES["iho181"]
    full = Stepper(ph, 8, 0, seed=3)
    s0 = Stepper(ph, 4, 0, seed=3, env_offset=0)
    s1 = Stepper(ph, 4, 0, seed=3, env_offset=4)
    a = full.new_state()
    full.reset(a, 1, arg0=16)
    acts = torch.randint(0, 21, (8,), dtype=torch.int32, device="cuda")
    b0, b1 = a[:4].clone(), a[4:].clone()
    full.step(a, acts, 100)
    s0.step(b0, acts[:4].contiguous(), 100)
    s1.step(b1, acts[4:].contiguous(), 100)
    assert torch.equal(a, torch.cat([b0, b1]))


@pytest.mark.parametrize("name", ["iho181", "iho512", "ho71", "qo171", "iqo513"])
def test_moments_parity(oracle_mod, name):
    ph = CASES[name]
    B = 4
    osys = oracle_sys(oracle_mod, ph)
    psi0 = init_states(osys, ph, B, seed=11)
    # evolve a little so the states are generic
    osys.run_batch(psi0, np.full(B, 3, np.int32), ph.f_max, 40, ph.dt, ph.gamma, seed=1, n_threads=4)
    st = Stepper(ph, B, 0)
    psi = torch.from_numpy(psi0).cuda()
    got = st.moments(psi).cpu().numpy()
    ref = np.stack([osys.moments(p) for p in psi0])
    np.testing.assert_allclose(got, ref, rtol=1e-10, atol=1e-11)
    xe = st.x_expectation(psi).cpu().numpy()
    np.testing.assert_allclose(xe, [osys.x_expectation(p) for p in psi0], atol=1e-12)
    bf = st.boundary_fail(psi).cpu().numpy()
    assert list(bf) == [osys.boundary_fail(p) for p in psi0]
    # fused observation at the end of a step call equals the standalone kernel (the same arithmetic; the
    # two inlining contexts may contract one FMA differently: <= 2 ulp)
    out = st.step(psi, None, 0, want_obs=True)
    np.testing.assert_allclose(out["obs"].cpu().numpy(), got, rtol=5e-16, atol=1e-15)


@pytest.mark.parametrize("case,order", [("qo171", 1), ("qo171", 7), ("qo171", 9), ("qo171", 10), ("qo171", 13),
                                        ("qo171", 16), ("iqo513", 12), ("qo1025", 10)])
def test_high_moment_orders_match_oracle(oracle_mod, case, order):
    """get_moments beyond the drivers' default order (QO/setupC.py compiles any MOMENT >= 1;
    QO/simulation_quart.cpp:326-388): orders above the step kernel's fused epilogue (6) run the observation
    kernel after the step; up to 9 ((2+9+1)*9/2 = 54 observables) one per lane, up to 16 (152) with several per lane
    (its second instantiation; at C3's R = 17 it spills, a path no driver takes); 17 is refused. Tolerance: the
    order-m observables reach |x - <x>|^a |p|^b with a + b = m, so they are compared to 1e-10 of the vector's largest
    entry beside the relative 1e-10 (the oracle sums each moment in another order)."""
    ph = CASES[case].with_(moment_order=order)
    B = 3
    osys = oracle_sys(oracle_mod, ph)
    psi0 = init_states(osys, ph, B, seed=5)
    osys.run_batch(psi0, np.full(B, 14, np.int32), ph.f_max, 30, ph.dt, ph.gamma, seed=2, n_threads=4)
    st = Stepper(ph, B, 0)
    assert st.n_obs == (2 + order + 1) * order // 2
    psi = torch.from_numpy(psi0.copy()).cuda()
    got = st.moments(psi).cpu().numpy()
    ref = np.stack([osys.moments(p) for p in psi0])
    assert ref.shape == got.shape
    assert np.isfinite(ref).all() and np.isfinite(got).all()
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=1e-10, atol=1e-11 + (1e-10 * np.abs(r).max() if order > 9 else 0.0))
    out = st.step(psi, None, 0, want_obs=True)   # the step call's observation (fused or after the step)
    np.testing.assert_allclose(out["obs"].cpu().numpy(), got, rtol=5e-16, atol=1e-15)
    with pytest.raises(Exception):
        Stepper(ph.with_(moment_order=17), B, 0)


def test_outside_probability_and_term_step(oracle_mod):
    ph = CASES["iqo513"]
    B = 3
    osys = oracle_sys(oracle_mod, ph)
    psi0 = np.stack([osys.gaussian_packet(0.0, mu, 1.0) for mu in (0.0, 3.5, 4.8)])
    st = Stepper(ph, B, 0)
    psi = torch.from_numpy(psi0.copy()).cuda()
    got = st.outside_prob(psi, ph.xth).cpu().numpy()
    np.testing.assert_allclose(got, [osys.outside_prob(p, ph.xth) for p in psi0], atol=1e-13)
    # per-step termination index against the oracle
    steps = 160
    noise = np.random.default_rng(3).standard_normal((steps, B, 2))
    acts = np.array([20, 20, 20], np.int32)
    ref = psi0.copy()
    term_ref = np.full(B, -1)
    for e in range(B):
        if osys.outside_prob(ref[e], ph.xth) > 0.5:
            term_ref[e] = 0
    for k in range(steps):
        osys.run_batch(ref, acts, ph.f_max, 1, ph.dt, ph.gamma, noise=noise[k:k + 1])
        for e in range(B):
            if term_ref[e] < 0 and osys.outside_prob(ref[e], ph.xth) > 0.5:
                term_ref[e] = k + 1
    out = st.step(psi, torch.from_numpy(acts).cuda(), steps, noise=torch.from_numpy(noise).cuda(), want_term=True)
    assert list(out["term_step"].cpu().numpy()) == list(term_ref)


def test_reset_kernels_match_oracle(oracle_mod):
    ph = CASES["iho181"]
    st = Stepper(ph, 6, 0, seed=1234, env_offset=10)
    osys = oracle_sys(oracle_mod, ph)
    psi = st.new_state()
    st.reset(psi, 1, arg0=16)
    ref = np.stack([osys.fock_random_state(1234, 10 + e, 16) for e in range(6)])
    np.testing.assert_allclose(psi.cpu().numpy(), ref, atol=1e-15)
    mask = torch.tensor([1, 0, 1, 0, 0, 1], dtype=torch.uint8, device="cuda")
    st.reset(psi, 0, mask=mask)
    got = psi.cpu().numpy()
    assert got[0, 0] == 1 and np.count_nonzero(got[0]) == 1 and np.allclose(got[1], ref[1])
    g = CASES["iqo513"]
    sg = Stepper(g, 2, 0)
    og = oracle_sys(oracle_mod, g)
    pg = sg.new_state()
    sg.reset(pg, 2, arg0=0.0, arg1=0.0, arg2=1.0)
    np.testing.assert_allclose(pg.cpu().numpy()[0], og.gaussian_packet(0.0, 0.0, 1.0), atol=1e-15)


def test_scan_truncation_levels_reported():
    st = Stepper(CASES["iho512"], 1, 0)
    kf, kb = st.scan_levels(20)
    assert 1 <= kf <= 6 and 1 <= kb <= 6


def test_custom_force_slot_matches_oracle(oracle_mod):
    ph = CASES["iho181"]
    osys = oracle_sys(oracle_mod, ph)
    st = Stepper(ph, 2, 0)
    slot = st.add_force(1.2345)
    assert slot >= 21
    psi0 = init_states(osys, ph, 2)
    noise = np.random.default_rng(0).standard_normal((100, 2, 2))
    ref = psi0.copy()
    for e in range(2):
        t = ref[e].copy()
        for k in range(100):
            osys.step(t, ph.dt, 1.2345, ph.gamma, noise[k, e])
        ref[e] = t
    psi = torch.from_numpy(psi0).cuda()
    st.step(psi, None, 100, default_action=slot, noise=torch.from_numpy(noise).cuda())
    assert wnorm(ph, psi.cpu().numpy() - ref).max() < 1e-11


@pytest.mark.parametrize("name", ["ho71", "iho181", "qo171"])
def test_energy_and_phonon(oracle_mod, name):
    ph = CASES[name]
    osys = oracle_sys(oracle_mod, ph)
    psi0 = init_states(osys, ph, 3, seed=5)
    st = Stepper(ph, 3, 0)
    psi = torch.from_numpy(psi0).cuda()
    np.testing.assert_allclose(st.energy(psi).cpu().numpy(), [osys.energy(p) for p in psi0], rtol=1e-12, atol=1e-12)
    if ph.fock:
        np.testing.assert_allclose(st.phonon_number(psi).cpu().numpy(), [osys.phonon(p) for p in psi0], rtol=1e-13)


def test_env_steps_budget_freezes_envs():
    ph = CASES["iho181"]
    st = Stepper(ph, 4, 0, seed=9)
    a = st.new_state()
    st.reset(a, 1, arg0=16)
    b = a.clone()
    budget = torch.tensor([80, 0, 30, 80], dtype=torch.int32, device="cuda")
    st.step(a, None, 80, env_steps=budget)
    assert torch.equal(a[1], b[1])                 # frozen env untouched
    st.step_counter = 0
    ref = b.clone()
    st.step(ref, None, 80)
    assert torch.equal(a[0], ref[0]) and torch.equal(a[3], ref[3])
    assert not torch.equal(a[2], ref[2])


@pytest.mark.parametrize("name", ["iho181", "ho256", "qo171", "iqo513"])
def test_empty_inputs_and_single_env(oracle_mod, name):
    """Edge cases of the step boundary: an empty batch (B = 0: every call is a no-op returning QC_OK, like the
    reference's loop over no actors), zero physics steps (psi bitwise unchanged, no Fail), and a batch of one
    env (a single partially-filled workgroup) equal to the oracle over one control interval."""
    ph = CASES[name]
    st0 = Stepper(ph, 0, 0, seed=3)
    empty = st0.new_state()
    assert empty.shape == (0, st0.N)
    out = st0.step(empty, torch.zeros(0, dtype=torch.int32, device="cuda"), 10, want_q=True, want_obs=True)
    assert out["fail_step"].numel() == 0 and out["q"].shape == (10, 0)
    assert st0.moments(empty).shape[0] == 0 and st0.x_expectation(empty).numel() == 0
    osys = oracle_sys(oracle_mod, ph)
    psi0 = init_states(osys, ph, 1)
    st = Stepper(ph, 1, 0, seed=3)
    psi = torch.from_numpy(psi0.copy()).cuda()
    acts = torch.tensor([ph.n_actions // 2 + 3], dtype=torch.int32, device="cuda")
    out = st.step(psi, acts, 0, want_q=True)
    torch.cuda.synchronize()
    assert torch.equal(psi.cpu(), torch.from_numpy(psi0)) and int(out["fail_step"][0]) == 0
    n = ph.control_interval
    noise = np.random.default_rng(11).standard_normal((n, 1, 2))
    ref = psi0.copy()
    f_ref, _, xm_ref = osys.run_batch(ref, acts.cpu().numpy(), ph.f_max, n, ph.dt, ph.gamma, noise=noise,
                                      want_q=True, n_threads=1)
    out = st.step(psi, acts, n, noise=torch.from_numpy(noise).cuda(), want_q=True)
    assert int(out["fail_step"][0]) == int(f_ref[0])
    np.testing.assert_allclose(out["x_mean"].cpu().numpy(), xm_ref, atol=1e-10)
    assert float(wnorm(ph, psi.cpu().numpy() - ref)[0]) < 1e-10


@pytest.mark.parametrize("case", ["iho512", "ho256", "iqo513", "qo1025"])
def test_table_placements_bitwise_equal(monkeypatch, case):
    """The step kernel's factor-table placements (0: global buffer loads, 1: workgroup LDS image of
    lc/uc/di/m2, 2: + scan composites; qo1025 (C3): 4 — the forward composites only — in place of 2) agree
    (1 and 2 / 4 bit-identical; 0 may contract differently, <1e-12), with envs of mixed force slots grouped per
    workgroup; the grouping must not change any env's trajectory (bitwise)."""
    ph = CASES[case]
    B = 37
    st = Stepper(ph, B, 0, seed=11)
    a = st.new_state()
    if ph.fock:
        st.reset(a, 1, arg0=16)
    else:
        st.reset(a, 2, arg0=0.0, arg1=0.0, arg2=1.0)
    init = a.clone()
    acts = torch.randint(0, 21, (B,), dtype=torch.int32, device="cuda")
    outs = []
    for mode in ("2", "1", "0"):
        monkeypatch.setenv("QCART_TAB_MODE", mode)
        st.step_counter = 0
        x = init.clone()
        st.step(x, acts, 40)
        outs.append(x)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    assert float((outs[0] - outs[2]).abs().max()) < 1e-12
    # per-env trajectories do not depend on which other envs share the call
    monkeypatch.setenv("QCART_TAB_MODE", "2")
    st1 = Stepper(ph, 1, 0, seed=11, env_offset=5)
    y = init[5:6].clone()
    st1.step(y, acts[5:6], 40)
    torch.cuda.synchronize()
    assert torch.equal(y[0], outs[0][5])


@pytest.mark.parametrize("case", ["iho512", "ho256", "iqo513", "qo1025"])
def test_short_call_layouts_bitwise_equal(case):
    """Short calls (n <= 10 steps, tables from L2): a small batch runs one env per workgroup ("spread", batch <=
    1024), a larger one eight envs per workgroup, and the state rows, budget and action are read together up front
    (R <= 8). The same 37 envs stepped ten one-step calls in a 37-env handle and inside an 1100-env handle (the
    other envs without a step budget) give bit-identical states, q and x_mean."""
    ph = CASES[case]
    B1, B2, K = 37, 1100, 10
    rng = np.random.default_rng(3)
    acts = torch.from_numpy(rng.integers(0, 21, B1).astype(np.int32)).cuda()
    noise = torch.from_numpy(rng.standard_normal((K, 1, B1, 2))).cuda()
    res = []
    for B in (B1, B2):
        st = Stepper(ph, B, 0, seed=11)
        a = st.new_state()
        if ph.fock:
            st.reset(a, 1, arg0=16)
        else:
            st.reset(a, 2, arg0=0.0, arg1=0.0, arg2=1.0)
        x = a[:B1].clone() if B == B1 else a
        if B == B2:
            x[:B1] = res[0][2]                                   # the same initial states
        act = acts if B == B1 else torch.cat([acts, torch.full((B2 - B1,), 10, dtype=torch.int32, device="cuda")])
        bud = torch.zeros(B, dtype=torch.int32, device="cuda")
        bud[:B1] = 1
        qs = []
        for k in range(K):
            nz = noise[k] if B == B1 else torch.cat([noise[k], torch.zeros((1, B2 - B1, 2), dtype=torch.float64,
                                                                              device="cuda")], 1)
            out = st.step(x, act, 1, noise=nz, env_steps=bud, want_q=True)
            qs.append((out["q"][0, :B1].clone(), out["x_mean"][0, :B1].clone()))
        torch.cuda.synchronize()
        if B == B1:
            res.append((x.clone(), qs, a[:B1].clone()))
        else:
            res.append((x[:B1].clone(), qs))
    assert torch.equal(res[0][0], res[1][0])
    for (q1, m1), (q2, m2) in zip(res[0][1], res[1][1]):
        assert torch.equal(q1, q2) and torch.equal(m1, m2)


@pytest.mark.parametrize("case", ["iho512", "ho256", "iqo513", "qo171"])
@pytest.mark.parametrize("mode", ["2", "1"])
def test_two_slot_workgroups_bitwise_equal(monkeypatch, case, mode):
    """k_group's packed layout (slots with >= 8 envs back to back, the workgroups that straddle two slots run
    the MODE 3 body with both slots' tables in LDS, k_step DUAL) against per-slot padded workgroups
    (QCART_DUAL=0): every env's trajectory, q, x_mean and Fail step are bit-identical — with small slots
    (< 8 envs: padded on their own), slots of exactly 8, big slots, out-of-order slot ids, envs without a
    step budget, and the MODE 1 pure body too."""
    ph = CASES[case]
    B = 203
    rng = np.random.default_rng(5)
    # skewed action histogram: slots of 1..7 envs, exactly 8, and big ones
    counts = {0: 3, 2: 8, 3: 1, 5: 40, 7: 9, 10: 61, 11: 7, 13: 17, 17: 33, 20: 24}
    acts_np = rng.permutation(np.concatenate([np.full(c, s, np.int32) for s, c in counts.items()]))
    assert len(acts_np) == B
    budget = np.full(B, 30, np.int32)
    budget[rng.choice(B, 12, replace=False)] = 0
    budget[rng.choice(B, 5, replace=False)] = 17
    monkeypatch.setenv("QCART_TAB_MODE", mode)
    outs = []
    for dual in ("1", "0"):
        monkeypatch.setenv("QCART_DUAL", dual)
        st = Stepper(ph, B, 0, seed=21)
        psi = st.new_state()
        if ph.fock:
            st.reset(psi, 1, arg0=16)
        else:
            st.reset(psi, 2, arg0=0.0, arg1=0.0, arg2=1.0)
        out = st.step(psi, torch.from_numpy(acts_np).cuda(), 30,
                      env_steps=torch.from_numpy(budget).cuda(), want_q=True, want_fail=True)
        torch.cuda.synchronize()
        outs.append((psi.clone(), out["q"].clone(), out["x_mean"].clone(), out["fail_step"].clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    # q / x_mean rows past an env's budget and the Fail step of an env without one are never written
    steps = torch.arange(30, device="cuda")[:, None] < torch.from_numpy(budget).cuda()[None, :]
    for i in (1, 2):
        assert torch.equal(outs[0][i][steps], outs[1][i][steps])
    ran = torch.from_numpy(budget).cuda() > 0
    assert torch.equal(outs[0][3][ran], outs[1][3][ran])


@pytest.mark.parametrize("B", [4096, 203])
def test_group_layout_packs_slots(B):
    """k_group's layout (qc_group_layout): every env with a step budget in exactly one workgroup; each
    single-slot workgroup holds one slot; each two-slot workgroup exactly two; slots of >= 8 envs fill
    ceil(their total / 8) workgroups; smaller slots and the no-budget envs are padded on their own."""
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=511)
    rng = np.random.default_rng(B)
    acts = rng.integers(0, 21, B).astype(np.int32)
    if B < 1000:   # one slot of exactly 9 envs, one of 2
        acts[acts == 3] = 4
        acts[:9] = 3
        acts[acts == 6] = 5
        acts[9:11] = 6
    budget = np.full(B, 80, np.int32)
    budget[rng.choice(B, B // 20, replace=False)] = 0
    st = Stepper(ph, B, 0, seed=1)
    psi = st.new_state()
    st.reset(psi, 1, arg0=4)
    # (12 steps: calls of <= 10 steps on small batches read their tables from L2 without grouping, qc_step)
    st.step(psi, torch.from_numpy(acts).cuda(), 12, env_steps=torch.from_numpy(budget).cuda())
    order, mixed = st.group_layout()
    g = order.shape[1]
    mixed = np.array([wg for wg in mixed if (wg >= 0).any()]).reshape(-1, g)
    assert len(mixed) > 0
    seen = np.concatenate([order.ravel(), mixed.ravel()])
    seen = seen[seen >= 0]
    assert sorted(seen.tolist()) == list(range(B))
    ran = budget > 0
    slot = np.where(ran, acts, 99)
    for wg in order:
        e = wg[wg >= 0]
        assert len(set(slot[e].tolist())) <= 1
    for wg in mixed:
        e = wg[wg >= 0]
        assert len(set(slot[e].tolist())) == 2 and ran[e].all()
    cnt = np.bincount(acts[ran], minlength=21)
    big, small = cnt[cnt >= g].sum(), cnt[(cnt > 0) & (cnt < g)]
    busy = [wg for wg in order if (wg >= 0).any()]
    n_nobudget = (B - ran.sum() + g - 1) // g
    assert len(busy) + len(mixed) == (big + g - 1) // g + len(small) + n_nobudget
    print(f"B={B}: {len(busy)} single-slot + {len(mixed)} two-slot workgroups "
          f"(padded per slot: {int(sum((c + g - 1) // g for c in cnt if c)) + n_nobudget})")


@pytest.mark.parametrize("config", ["C2", "C3", "C4", "metric"])
def test_config_size_batch_properties(oracle_mod, config):
    """At a BASELINE config's full per-GPU batch (C2: IHO N=512 B=4096; C3: QO x_n=1025, B=16384; C4: IQO
    x_n=513, B=8192 per GPU of its 8-GPU run; the metric: IHO N=512, B=65536 per GPU, the bench workload): every env stays
    normalised, the call is deterministic, and sampled envs of the big batch match the oracle run alone
    with the same in-kernel Philox stream (1e-10 over 80 steps)."""
    conf = cfg.BENCH_CONFIGS[config]
    ph = conf["physics"] if config != "C3" else CASES["qo1025"]   # C3 at its stable dt
    B = conf["batch"] // 8 if config == "C4" else conf["batch"]
    st = Stepper(ph, B, 0, seed=99)
    psi = st.new_state()
    if ph.fock:
        st.reset(psi, 1, arg0=16)
    else:
        st.reset(psi, 2, arg0=0.0, arg1=0.0, arg2=1.0)
    psi0 = psi.clone()
    acts = torch.randint(0, 21, (B,), generator=torch.Generator(device="cuda").manual_seed(5),
                         device="cuda", dtype=torch.int32)
    st.step(psi, acts, 80)
    st.step_counter = 0
    again = psi0.clone()
    st.step(again, acts, 80)
    torch.cuda.synchronize()
    assert torch.equal(psi, again)
    w = 1.0 if ph.fock else ph.grid_size
    norms = (psi.abs() ** 2).sum(1) * w
    assert float((norms - 1).abs().max()) < 1e-12
    osys = oracle_sys(oracle_mod, ph)
    for e in (0, 1, B // 2, B - 1):
        ref = psi0[e:e + 1].cpu().numpy().copy()
        osys.run_batch(ref, acts[e:e + 1].cpu().numpy(), ph.f_max, 80, ph.dt, ph.gamma, seed=99, env_offset=e,
                       n_threads=1)
        err = wnorm(ph, psi[e].cpu().numpy() - ref[0])
        assert err < 1e-10, (e, err)


@pytest.mark.parametrize("n_max", [511, 1023, 2047])
def test_fp32_path_tracks_fp64_oracle(oracle_mod, n_max):
    """fp32 working precision (config C5: IHO N = 2048 in fp32): the complex64 state stays within
    fp32 accumulation error of the fp64 oracle on identical injected noise (measured ~8e-7 at 200
    steps; bound 2e-5), and the Fail flag agrees."""
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=n_max, precision=1, gamma=0.5 * pi)
    B = 4
    osys = oracle_sys(oracle_mod, ph)
    ref = np.zeros((B, ph.dim), np.complex128)
    ref[:, 0] = 1.0
    st = Stepper(ph, B, 0, seed=1)
    psi = torch.from_numpy(ref.astype(np.complex64)).cuda()
    rng = np.random.default_rng(0)
    for _ in range(5):
        acts = rng.integers(8, 13, B).astype(np.int32)
        nz = rng.standard_normal((40, B, 2))
        f_ref, _, _ = osys.run_batch(ref, acts, ph.f_max, 40, ph.dt, ph.gamma, noise=nz, n_threads=4)
        out = st.step(psi, torch.from_numpy(acts).cuda(), 40, noise=torch.from_numpy(nz).cuda(), want_fail=True)
        assert np.array_equal(out["fail_step"].cpu().numpy(), f_ref)
    err = np.linalg.norm(psi.cpu().numpy().astype(np.complex128) - ref, axis=1)
    assert err.max() < 2e-5, err


def test_fp32_c5_batch_properties(oracle_mod):
    """C5's per-GPU batch (262144 / 8 envs at N = 2048, fp32): normalised, deterministic, and a sampled
    env matches the fp64 oracle run alone with the same Philox stream to fp32 accuracy."""
    conf = cfg.BENCH_CONFIGS["C5"]
    ph = conf["physics"]
    B = conf["batch"] // 8
    st = Stepper(ph, B, 0, seed=7)
    psi = st.new_state()
    assert psi.dtype == torch.complex64
    st.reset(psi, 1, arg0=16)
    psi0 = psi.clone()
    acts = torch.randint(0, 21, (B,), generator=torch.Generator(device="cuda").manual_seed(2), device="cuda",
                         dtype=torch.int32)
    st.step(psi, acts, 80)
    st.step_counter = 0
    again = psi0.clone()
    st.step(again, acts, 80)
    torch.cuda.synchronize()
    assert torch.equal(psi, again)
    norms = (psi.abs().double() ** 2).sum(1)
    assert float((norms - 1).abs().max()) < 1e-5
    osys = oracle_sys(oracle_mod, ph)
    for e in (0, B - 1):
        ref = psi0[e:e + 1].cpu().numpy().astype(np.complex128)
        osys.run_batch(ref, acts[e:e + 1].cpu().numpy(), ph.f_max, 80, ph.dt, ph.gamma, seed=7, env_offset=e,
                       n_threads=1)
        err = np.linalg.norm(psi[e].cpu().numpy().astype(np.complex128) - ref[0])
        assert err < 1e-5, (e, err)


def test_fp32_rejects_grid_and_wrong_dtype():
    with pytest.raises(Exception):
        Stepper(cfg.DEFAULTS[cfg.IQO].with_(x_max=12.8, precision=1), 2, 0)
    st = Stepper(cfg.DEFAULTS[cfg.IHO].with_(n_max=511, precision=1), 2, 0)
    with pytest.raises(ValueError, match="Complex64"):
        st.step(torch.zeros((2, 512), dtype=torch.complex128, device="cuda"), None, 1)


@pytest.mark.parametrize("case", ["iho512", "ho256", "iqo513"])
def test_env_steps_grouping_bitwise(case):
    """Step budgets with per-env actions (the grouped path: no-budget envs in a workgroup group of their
    own, k_group): frozen envs stay bitwise untouched, full-budget envs equal an unbudgeted call and
    partial-budget envs equal a call of that many steps, bitwise."""
    ph = CASES[case]
    B = 100
    st = Stepper(ph, B, 0, seed=21)
    psi0 = st.new_state()
    if ph.fock:
        st.reset(psi0, 1, arg0=16)
    else:
        st.reset(psi0, 2, arg0=0.0, arg1=0.0, arg2=1.0)
    g = torch.Generator(device="cuda").manual_seed(4)
    acts = torch.randint(0, 21, (B,), generator=g, device="cuda", dtype=torch.int32)
    budget = torch.tensor([[0, 40, 80][i % 3] for i in range(B)], dtype=torch.int32, device="cuda")
    a = psi0.clone()
    out = st.step(a, acts, 80, env_steps=budget, want_fail=True)
    st.step_counter = 0
    full = psi0.clone()
    st.step(full, acts, 80)
    st.step_counter = 0
    part = psi0.clone()
    st.step(part, acts, 40)
    bz = budget.cpu().numpy()
    for e in range(B):
        want = {0: psi0, 40: part, 80: full}[int(bz[e])]
        assert torch.equal(a[e], want[e]), e
    assert int(out["fail_step"][budget == 0].abs().sum()) == 0


@pytest.mark.parametrize("case,steps", [("iho512", 4000), ("iqo513", 6000)])
def test_diverging_envs_stay_finite_in_long_calls(case, steps):
    """Lazy normalisation carries psi unnormalised through a call; an env past its Fail diverges (IHO N = 512
    at gamma 2 pi, dt 1/1440 blows up after ~700 steps; the inverted quartic's packet falls off its grid under full pushes),
    and its carried scale would overflow within a long call. The kernel folds the scale back into psi once it
    leaves [2^-100, 2^100] (lazy_rescale): psi stays finite and normalised, and the observation finite."""
    ph = CASES[case]
    B = 4
    st = Stepper(ph, B, 0, seed=5)
    psi = st.new_state()
    if ph.fock:
        st.reset(psi, 1, arg0=16)
        acts = torch.tensor([0, 20, 10, 3], dtype=torch.int32, device="cuda")
    else:
        st.reset(psi, 2, arg0=0.0, arg1=0.0, arg2=1.0)
        acts = torch.tensor([0, 20, 0, 20], dtype=torch.int32, device="cuda")
    out = st.step(psi, acts, steps, want_fail=True, want_obs=True)
    torch.cuda.synchronize()
    p = psi.cpu().numpy()
    assert np.all(np.isfinite(p))
    assert np.all(np.isfinite(out["obs"].cpu().numpy()))
    norms = wnorm(ph, p)
    np.testing.assert_allclose(norms, 1.0, atol=1e-9)
    if ph.fock:
        assert int((out["fail_step"] > 0).sum()) >= 1
    print(f"{case}: fail steps {out['fail_step'].tolist()}, norms {norms}")
