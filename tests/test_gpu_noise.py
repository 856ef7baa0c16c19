"""GPU tests of the noise streams: the reference's MT19937 + Box-Muller stream on the device
(qc_set_seed_mt19937), the drop-in reproducing the MKL-ordered reference trajectory from set_seed(seed)
alone, and per-env Philox counters (an env's stream depends only on its own steps)."""
from math import pi
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd import simulation as S  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.core import Stepper  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.env import BatchedEnv  # noqa: E402

FIX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mkl_v1.npz")


def test_mt19937_states_and_trajectories_match_oracle(oracle_mod):
    """Per-env MT19937 on the device: after a call with step budgets every env's state words equal the
    oracle's stream advanced by exactly 4 words per step taken (bitwise), and the trajectories equal the
    oracle fed the oracle's MT19937 normals (1e-12)."""
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    seeds = [0, 1, 42, 99998, 4294967295]
    B = len(seeds)
    st = Stepper(ph, B, 0)
    st.set_seed_mt19937(seeds)
    assert st.noise_mode == "mt19937"
    psi = st.new_state()
    psi[:, 0] = 1.0
    psi0 = psi.cpu().numpy()
    budget = [170, 0, 100, 170, 5]      # 170 steps = 680 words: crosses a twist
    acts = np.array([10, 12, 7, 9, 10], np.int32)
    out = st.step(psi, torch.from_numpy(acts).cuda(), 170, env_steps=torch.tensor(budget, dtype=torch.int32,
                                                                                   device="cuda"), want_q=True)
    torch.cuda.synchronize()
    W = 626
    dev_state = st.mt19937_state().cpu().numpy().view(np.uint32).reshape(B, W)
    osys = oracle_mod.OracleSystem(1, n_max=63)
    for e, s in enumerate(seeds):
        mt = oracle_mod.MT19937(s)
        r = mt.normals(2 * budget[e]).reshape(budget[e], 1, 2)
        assert np.array_equal(dev_state[e, :624], mt.st[:624]), e
        assert dev_state[e, 624] == mt.st[624], e
        ref = psi0[e:e + 1].copy()
        if budget[e]:
            osys.run_batch(ref, acts[e:e + 1], ph.f_max, budget[e], ph.dt, ph.gamma, noise=r, n_threads=1)
        err = np.linalg.norm(psi[e].cpu().numpy() - ref[0])
        assert err < 1e-12, (e, err)
    # the next call continues each stream where it stopped
    st.step(psi, torch.from_numpy(acts).cuda(), 3)
    dev2 = st.mt19937_state().cpu().numpy().view(np.uint32).reshape(B, W)
    for e, s in enumerate(seeds):
        mt = oracle_mod.MT19937(s)
        mt.words(4 * (budget[e] + 3))
        assert np.array_equal(dev2[e, :625], mt.st), e


def test_mt19937_prefetched_pairs_continue_the_stream(oracle_mod):
    """qc_mt19937_normals (the step server's prefetch): a one-step draw into `pre`, then a ten-step draw that takes
    the drawn pair as step 0 (has_pre) — each env's normals and its state words are exactly the plain stream's:
    pair k of the stream at step k, 4 words per step."""
    import ctypes
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import _lib as L
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    seeds = [7, 1234, 99]
    B = len(seeds)
    st = Stepper(ph, B, 0)
    st.set_seed_mt19937(seeds)
    lib = L.lib()
    pre = torch.zeros((B, 2), dtype=torch.float64, device="cuda")
    out = torch.full((10, B, 2), -7.0, dtype=torch.float64, device="cuda")
    one = torch.tensor([1, 1, 0], dtype=torch.int32, device="cuda")
    st._bind_stream()
    L.check(lib.qc_mt19937_normals(st._h, 1, one.data_ptr(), None, None, pre.data_ptr()), st._h)
    has = torch.tensor([1, 1, 0], dtype=torch.uint8, device="cuda")
    bud = torch.tensor([10, 3, 10], dtype=torch.int32, device="cuda")
    L.check(lib.qc_mt19937_normals(st._h, 10, bud.data_ptr(), pre.data_ptr(), has.data_ptr(), out.data_ptr()), st._h)
    torch.cuda.synchronize()
    got, p0 = out.cpu().numpy(), pre.cpu().numpy()
    words = st.mt19937_state().cpu().numpy().view(np.uint32).reshape(B, -1)
    for e, s in enumerate(seeds):
        n = int(bud[e])
        want = oracle_mod.MT19937(s).normals(2 * n).reshape(n, 2)
        np.testing.assert_allclose(got[:n, e], want, rtol=1e-14, atol=1e-15)
        assert np.all(got[n:, e] == -7.0)                            # steps past the budget untouched
        if e < 2:
            assert np.array_equal(p0[e], got[0, e])                   # the prefetched pair is step 0
        mt = oracle_mod.MT19937(s)
        mt.words(4 * n)
        assert np.array_equal(words[e, :625], mt.st), e


@pytest.mark.parametrize("name", ["iho181", "iho512"])
def test_dropin_set_seed_reproduces_mkl_reference_trajectory(name):
    """The drop-in with the reference's call sequence — set_seed(seed), then step(state, dt, force,
    gamma) 1000 times — equals the MKL-call-ordered stepper (tests/golden/mklref.py) on MKL's
    CBWR=COMPATIBLE stream for that seed: psi to 1e-9 after 1000 steps, every step's q and x_mean to
    1e-9, Fail never raised. Against MKL's default (AVX-512, reduced-accuracy normals) stream the
    difference is bounded (< 1e-5) and reported, not a parity claim."""
    with np.load(FIX) as z:
        n_max = int(z[f"traj/{name}/n_max"])
        dt, gamma, f_max = z[f"traj/{name}/phys"]
        seed = int(z[f"traj/{name}/seed"])
        acts = z[f"traj/{name}/actions"]
        ref_q, ref_x = z[f"traj/{name}/cnr/q"], z[f"traj/{name}/cnr/x_mean"]
        ref_psi, dflt_psi = z[f"traj/{name}/cnr/psi"], z[f"traj/{name}/default/psi"]
    sim = S.load(cfg.IHO, n_max=n_max, time_steps=int(round(1 / dt)))
    sim.set_seed(seed)
    state = np.zeros(n_max + 1, np.complex128)
    state[0] = 1.0
    qs, xs, snaps = [], [], []
    for k in range(len(ref_q)):
        F = (int(acts[k // 80]) - 10) * (f_max / 10.)
        q, xm, fail = sim.step(state, dt, F, gamma)
        assert fail == 0
        qs.append(q)
        xs.append(xm)
        if k + 1 in (100, 500, 1000):
            snaps.append(state.copy())
    assert np.abs(np.array(qs) - ref_q).max() < 1e-9
    assert np.abs(np.array(xs) - ref_x).max() < 1e-9
    errs = [np.linalg.norm(a - b) for a, b in zip(snaps, ref_psi)]
    assert max(errs) < 1e-9, errs
    d = np.linalg.norm(snaps[-1] - dflt_psi[-1])
    print(f"{name}: |psi - psi_mkl_cnr| = {errs[-1]:.2e}, |psi - psi_mkl_default| = {d:.2e} after 1000 steps")
    assert d < 1e-5


def test_dropin_simulate_10_steps_matches_oracle(oracle_mod):
    """simulate_10_steps (IHO/simulation_i.cpp:391-421): ten go_one_step calls, the LAST step's (q,
    x_mean) and Fail of the final state only — against the oracle on the same MT19937 stream, up to and
    including the call where the pushed pole first reaches the basis boundary (Fail = 1)."""
    sim = S.load(cfg.IHO, n_max=31)
    sim.set_seed(5)
    o = oracle_mod.OracleSystem(1, n_max=31)
    mt = oracle_mod.MT19937(5)
    state = np.zeros(32, dtype=np.complex128)
    state[0] = 1.0
    ref = state.copy()
    dt, gamma = 1 / 1440, 2 * pi
    first_fail = None
    for call in range(100):
        force = 8.0 if call >= 5 else 0.8
        q, xm, fail = sim.simulate_10_steps(state, dt, force, gamma)
        for k in range(10):
            q2, xm2, f2 = o.step(ref, dt, force, gamma, mt.normals(2))
        assert abs(q - q2) < 1e-9 and abs(xm - xm2) < 1e-9, call
        assert fail == f2, call                     # Fail of the final state, not "any step"
        assert np.linalg.norm(state - ref) < 1e-9, call
        if fail:
            first_fail = call
            break
    assert first_fail is not None and first_fail > 5


def test_per_env_counters_make_streams_independent():
    """Philox noise keyed by each env's own counter: an env's trajectory depends only on the steps it
    took, not on which other envs stepped in the same calls (the advisor's auto-reset finding)."""
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    B = 6
    st = Stepper(ph, B, 0, seed=13)
    psi = st.new_state()
    st.reset(psi, 1, arg0=8)
    psi0 = psi.clone()
    acts = torch.tensor([10, 11, 9, 10, 12, 8], dtype=torch.int32, device="cuda")
    b1 = torch.tensor([80, 0, 40, 80, 0, 10], dtype=torch.int32, device="cuda")
    st.step(psi, acts, 80, env_steps=b1)
    st.step(psi, acts, 80)
    assert st.env_counters().tolist() == [160, 80, 120, 160, 80, 90]
    for e in range(B):   # the same calls on env e alone
        one = Stepper(ph, 1, 0, seed=13, env_offset=e)
        y = psi0[e:e + 1].clone()
        one.step(y, acts[e:e + 1], 80, env_steps=b1[e:e + 1].clone())
        one.step(y, acts[e:e + 1], 80)
        torch.cuda.synchronize()
        assert torch.equal(y[0], psi[e]), e
    # checkpoint / resume of the counters
    c = st.env_counters()
    st.step_counter = 7
    assert st.env_counters().tolist() == [7] * B
    st.env_counters(c)
    assert torch.equal(st.env_counters(), c)


def test_batched_env_shards_equal_single_run_with_auto_reset():
    """BatchedEnv with auto-reset: two shards (env_offset 0 and 4) reproduce a one-shard run bit for bit,
    although the shards' episodes end (and restart) at different control steps."""
    ph = cfg.DEFAULTS[cfg.IHO]
    full = BatchedEnv(ph, 8, 0, seed=3)
    halves = [BatchedEnv(ph, 4, 0, seed=3, env_offset=o) for o in (0, 4)]
    full.reset()
    for h in halves:
        h.reset()
    a = torch.tensor([20, 10, 10, 0, 10, 20, 11, 10], dtype=torch.int32, device="cuda")
    n_done = 0
    for _ in range(12):
        _, _, d, _ = full.step(a)
        n_done += int(d.sum())
        for i, h in enumerate(halves):
            h.step(a[4 * i:4 * i + 4])
    torch.cuda.synchronize()
    assert n_done > 0
    assert torch.equal(full.psi[:4], halves[0].psi) and torch.equal(full.psi[4:], halves[1].psi)


FIX2 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mkl_v2.npz")


@pytest.mark.parametrize("name", ["ho71", "ho256", "qo171", "iqo513"])
def test_dropin_set_seed_reproduces_mkl_reference_trajectory_v2(name):
    """The harmonic and grid modules through the drop-in with the drivers' call sequence — load(family,
    ...), set_seed(seed), then step(state, dt, force, gamma) 1000 times, get_moments(state, data) at the
    snapshots — against the MKL-call-ordered steppers (tests/golden/mklref.py HoMkl / GridMkl, fixtures
    mkl_v2.npz): psi to 1e-9 (grid norm weighted by sqrt(h)) after 100 / 500 / 1000 steps, every step's q and
    x_mean to 1e-9, Fail never raised, and compute_statistics' 20 moments to 1e-9 relative."""
    import json
    with np.load(FIX2) as z:
        c = json.loads(bytes(z[f"traj/{name}/params"]).decode())
        acts, psi0 = z[f"traj/{name}/actions"], z[f"traj/{name}/psi0"]
        ref_q, ref_x, ref_psi = z[f"traj/{name}/q"], z[f"traj/{name}/x_mean"], z[f"traj/{name}/psi"]
        ref_m = z[f"traj/{name}/moments"] if c["kind"] == "grid" else None
    ts = int(round(1 / c["dt"]))
    if c["kind"] == "ho":
        sim = S.load(cfg.HO, n_max=c["n_max"], omega=c["omega"], gamma=c["gamma"], time_steps=ts,
                     f_max=c["f_max"])
        w = 1.0
    else:
        fam = cfg.IQO if c["lam"] < 0 else cfg.QO
        sim = S.load(fam, x_max=c["x_max"], grid_size=c["h"], lambda_=c["lam"], mass=c["mass"],
                     gamma=c["gamma"], time_steps=ts, f_max=c["f_max"])
        w = np.sqrt(c["h"])
    sim.set_seed(int(c["seed"]))
    state = psi0.copy()
    qs, xs, errs, merrs = [], [], [], []
    snap = 0
    for k in range(len(ref_q)):
        F = (int(acts[k // c["ci"]]) - 10) * (c["f_max"] / 10.)
        q, xm, fail = sim.step(state, c["dt"], F, c["gamma"])
        assert fail == 0, k
        qs.append(q)
        xs.append(xm)
        if k + 1 in (100, 500, 1000):
            errs.append(np.linalg.norm(state - ref_psi[snap]) * w)
            if ref_m is not None:
                data = np.zeros(20)
                sim.get_moments(state, data)
                merrs.append(np.abs(data - ref_m[snap]).max() / max(1.0, np.abs(ref_m[snap]).max()))
            snap += 1
    assert np.abs(np.array(qs) - ref_q).max() < 1e-9
    assert np.abs(np.array(xs) - ref_x).max() < 1e-9
    assert max(errs) < 1e-9, errs
    if ref_m is not None:
        assert max(merrs) < 1e-9, merrs
    print(f"{name}: |psi - psi_mkl| = {errs[-1]:.2e} after 1000 steps" +
          (f", moments {max(merrs):.1e}" if merrs else ""))


def test_injected_and_mt19937_noise_leave_philox_counters_alone():
    """qcart.h: an injected noise array (and the MT19937 stream, whose normals reach the step kernel the
    same way) advances neither stream — the per-env Philox counters stay where they were."""
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    B = 4
    st = Stepper(ph, B, 0, seed=3)
    psi = st.new_state()
    st.reset(psi, 1, arg0=8)
    acts = torch.full((B,), 10, dtype=torch.int32, device="cuda")
    st.step(psi, acts, 7)
    assert st.env_counters().tolist() == [7] * B
    nz = torch.randn((5, B, 2), dtype=torch.float64, device="cuda")
    st.step(psi, acts, 5, noise=nz)
    assert st.env_counters().tolist() == [7] * B
    st.set_seed_mt19937([1, 2, 3, 4])
    c = st.env_counters()
    st.step(psi, acts, 6)
    assert torch.equal(st.env_counters(), c)


def test_mt19937_zero_word_matches_mkl(oracle_mod):
    """Device MT19937 states with planted zero words (mkl_v2.npz zero/*, saved from MKL's own stream):
    the step kernel consumes MKL's normals for them — finite at u1 = 0 (MKL's radius 3.4244955099270222),
    0 at u2 = 0 — so the trajectories equal the oracle fed MKL's normals (1e-12) and stay finite."""
    with np.load(FIX2) as z:
        states, normals = z["zero/state"], z["zero/normals"]
    B = len(states)
    ph = cfg.DEFAULTS[cfg.IHO].with_(n_max=63)
    st = Stepper(ph, B, 0)
    st.set_seed_mt19937(list(range(B)))
    W = 626
    new = np.zeros((B, W), np.uint32)
    new[:, :625] = states
    st.mt19937_state(torch.from_numpy(new.view(np.int32)))
    psi = st.new_state()
    psi[:, 0] = 1.0
    psi0 = psi.cpu().numpy()
    acts = np.full(B, 13, np.int32)
    n = normals.shape[1] // 2
    st.step(psi, torch.from_numpy(acts).cuda(), n)
    got = psi.cpu().numpy()
    assert np.all(np.isfinite(got))
    o = oracle_mod.OracleSystem(1, n_max=63)
    ref = psi0.copy()
    o.run_batch(ref, acts, ph.f_max, n, ph.dt, ph.gamma, noise=normals.reshape(B, n, 2).transpose(1, 0, 2).copy(),
                n_threads=1)
    assert np.abs(got - ref).max() < 1e-12


FIX3 = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "mkl_v3.npz")


def _fix3(name):
    import json
    with np.load(FIX3) as z:
        c = json.loads(bytes(z[f"traj/{name}/params"]).decode())
        d = {k.split("/")[-1]: z[k] for k in z.files if k.startswith(f"traj/{name}/")}
    return c, d


def _v3_physics(c, **kw):
    ts = int(round(1 / c["dt"]))
    if c["kind"] == "iho":
        return cfg.DEFAULTS[cfg.IHO].with_(n_max=c["n_max"], omega=c["omega"], gamma=c["gamma"], time_steps=ts,
                                           f_max=c["f_max"], **kw)
    return cfg.DEFAULTS[cfg.QO].with_(x_max=c["x_max"], grid_size=c["h"], lambda_=c["lam"], mass=c["mass"],
                                      gamma=c["gamma"], time_steps=ts, f_max=c["f_max"], **kw)


@pytest.mark.parametrize("name", ["qo1025", "iho1024"])
def test_dropin_set_seed_reproduces_mkl_reference_trajectory_v3(name):
    """The large configurations' sizes through the drop-in (load, set_seed, 1000 step calls, get_moments):
    C3's QO x_n = 1025 grid at dt 1/11520 and IHO N = 1024, against the MKL-call-ordered steppers
    (mkl_v3.npz, make_mkl_fixtures_v3.py): psi to 1e-9 (grid weighted by sqrt(h)) after 100 / 500 / 1000
    steps, every step's q and x_mean to 1e-9, Fail never raised, the grid's 20 moments to 1e-9 relative."""
    c, d = _fix3(name)
    ph = _v3_physics(c)
    kw = ph.asdict()
    fam = kw.pop("family")
    sim = S.load(fam, **kw)
    w = 1.0 if c["kind"] == "iho" else np.sqrt(c["h"])
    sim.set_seed(int(c["seed"]))
    state = d["psi0"].copy()
    qs, xs, errs, merrs = [], [], [], []
    snap = 0
    for k in range(len(d["q"])):
        F = (int(d["actions"][k // c["ci"]]) - 10) * (c["f_max"] / 10.)
        q, xm, fail = sim.step(state, c["dt"], F, c["gamma"])
        assert fail == 0, k
        qs.append(q)
        xs.append(xm)
        if k + 1 in (100, 500, 1000):
            errs.append(np.linalg.norm(state - d["psi"][snap]) * w)
            if c["kind"] == "grid":
                data = np.zeros(20)
                sim.get_moments(state, data)
                ref = d["moments"][snap]
                merrs.append(np.abs(data - ref).max() / max(1.0, np.abs(ref).max()))
            snap += 1
    assert np.abs(np.array(qs) - d["q"]).max() < 1e-9
    assert np.abs(np.array(xs) - d["x_mean"]).max() < 1e-9
    assert max(errs) < 1e-9, errs
    if merrs:
        assert max(merrs) < 1e-9, merrs
    print(f"{name}: |psi - psi_mkl| = {errs[-1]:.2e} after 1000 steps" + (f", moments {max(merrs):.1e}" if merrs else ""))


def _batched_on_fixture(c, d, ph, B):
    """B copies of the fixture's env through the batched Stepper (fused control-interval launches of the
    config's own step kernel, every copy on MKL's MT19937 stream of the case's seed)."""
    st = Stepper(ph, B, 0)
    st.set_seed_mt19937([int(c["seed"])] * B)
    psi = torch.from_numpy(np.tile(d["psi0"], (B, 1))).to(st.state_dtype).cuda()
    qs, xs = [], []
    k0, steps = 0, len(d["q"])
    for a in d["actions"]:
        n = min(c["ci"], steps - k0)
        out = st.step(psi, torch.full((B,), int(a), dtype=torch.int32, device="cuda"), n, want_q=True)
        assert int(out["fail_step"].max()) == 0
        qs.append(out["q"].cpu().numpy())
        xs.append(out["x_mean"].cpu().numpy())
        k0 += n
    return psi.cpu().numpy().astype(np.complex128), np.concatenate(qs), np.concatenate(xs)


@pytest.mark.parametrize("name", ["qo1025", "iho1024"])
def test_stepper_tracks_mkl_reference_trajectory_v3(name):
    """The batched path at the large sizes — k_step<…, R = 17> (C3) / R = 16, fused 160 / 80-step launches,
    8 envs per workgroup on one force slot — on MKL's stream: every copy equals the MKL-call-ordered
    trajectory to 1e-9 in psi after 1000 steps and in every step's q / x_mean."""
    c, d = _fix3(name)
    B = 8
    psi, q, xm = _batched_on_fixture(c, d, _v3_physics(c), B)
    w = 1.0 if c["kind"] == "iho" else np.sqrt(c["h"])
    err = np.linalg.norm(psi - d["psi"][-1], axis=1).max() * w
    assert np.abs(q - d["q"][:, None]).max() < 1e-9
    assert np.abs(xm - d["x_mean"][:, None]).max() < 1e-9
    assert err < 1e-9, err
    print(f"{name}: batched |psi - psi_mkl| = {err:.2e} after 1000 steps")


# fp32 working precision (C5) against the fp64 MKL reference, 1000 steps at N = 2048: a complex64 state
# carries ~6e-8 relative rounding per step; the measured drift stays below 1e-5 in psi
FP32_MKL_TOL_PSI = 2e-5
FP32_MKL_TOL_X = 2e-5


def test_fp32_tracks_mkl_reference_trajectory_iho2048():
    """C5's kernel (k_step<1, 32, 1, float>: IHO N = 2048, fp32 state and tables, fp64 reductions) on MKL's
    MT19937 stream against the fp64 MKL-call-ordered trajectory (mkl_v3.npz iho2048, gamma 2 pi,
    dt 1/11520): ||psi - psi_mkl||_2 < 2e-5 after 1000 steps and |x_mean - x_mean_mkl| < 2e-5 at every
    step (the fp32 bound stated above), 8 copies per launch."""
    c, d = _fix3("iho2048")
    psi, q, xm = _batched_on_fixture(c, d, _v3_physics(c, precision=1), 8)
    err = np.linalg.norm(psi - d["psi"][-1], axis=1).max()
    xerr = np.abs(xm - d["x_mean"][:, None]).max()
    print(f"iho2048 fp32: |psi - psi_mkl| = {err:.2e}, max |x_mean - ref| = {xerr:.2e} after 1000 steps")
    assert err < FP32_MKL_TOL_PSI, err
    assert xerr < FP32_MKL_TOL_X, xerr


# simulate_10_steps of the harmonic and grid modules (HO/simulation.cpp:372-402, QO/simulation_quart.cpp:526-558):
# (family, load params, force of call c, expect a Fail). The quartic cooling well confines the packet (no Fail);
# the inverted quartic's packet falls off the grid at the end the force pushes it to, so the grid's two-ended
# boundary test (QO/simulation_quart.cpp:559-565) is exercised at each end
S10_CASES = {
    "ho31": (cfg.HO, dict(n_max=31), lambda c: 5.0 if c >= 3 else 0.5, True),
    "qo171": (cfg.QO, dict(), lambda c: 5.0 if (c // 10) % 2 == 0 else -5.0, False),
    "iqo301_right": (cfg.IQO, dict(x_max=7.5), lambda c: 5.0, True),
    "iqo301_left": (cfg.IQO, dict(x_max=7.5), lambda c: -5.0, True),
}


@pytest.mark.parametrize("name", list(S10_CASES))
def test_dropin_simulate_10_steps_matches_oracle_other_modules(oracle_mod, name):
    """simulate_10_steps for HO and the grid modules: ten go_one_step calls, the last step's (q, x_mean) and
    the Fail test of the FINAL state only (HO: top-5 Fock amplitudes > 1e-3; grid: either end's 6 points >
    5e-3) — against the oracle on the same MT19937 stream, call by call, up to and including the call where the
    state first reaches the boundary."""
    fam, params, force_of, expect_fail = S10_CASES[name]
    sim = S.load(fam, **params)
    ph = sim._impl.physics
    seed = 11
    sim.set_seed(seed)
    mt = oracle_mod.MT19937(seed)
    if ph.fock:
        o = oracle_mod.OracleSystem(fam, n_max=ph.n_max, omega=ph.omega)
        state = np.zeros(o.N, np.complex128)
        state[0] = 1.0
    else:
        o = oracle_mod.OracleSystem(fam, x_max=ph.x_max, grid_size=ph.grid_size, lambda_=ph.lambda_, mass=ph.mass)
        x = ph.grid_size * (np.arange(o.N) - o.N // 2)
        state = (np.exp(-x * x / 4.) / (2 * pi) ** 0.25).astype(np.complex128)
    ref = state.copy()
    w = 1.0 if ph.fock else np.sqrt(ph.grid_size)
    first_fail = None
    n_calls = 400 if expect_fail else 30
    for call in range(n_calls):
        force = force_of(call)
        q, xm, fail = sim.simulate_10_steps(state, ph.dt, force, ph.gamma)
        for k in range(10):
            q2, xm2, f2 = o.step(ref, ph.dt, force, ph.gamma, mt.normals(2))
        assert abs(q - q2) < 1e-9 and abs(xm - xm2) < 1e-9, call
        assert fail == f2, call
        assert np.linalg.norm(state - ref) * w < 1e-9, call
        if fail:
            first_fail = call
            break
    if expect_fail:
        assert first_fail is not None, "never reached the boundary"
        if name.startswith("iqo"):
            # the end the packet fell off
            side = np.sign(o.x_expectation(ref))
            assert side == (1 if name.endswith("right") else -1)
    else:
        assert first_fail is None
    print(f"{name}: first Fail at call {first_fail}")
