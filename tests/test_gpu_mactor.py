"""GPU: the measurement-input actor (DQN_measurement on f32 MFMA, qc_mactor_act) against the numpy
restatement (oracle/dqn.forward_measurement) on identical parameters, measurement records and noise.

Tolerance: fp32 with exact-f32 MFMA accumulation over up to 4480-term sums vs fp64:
|q_dev - q_ref| <= 5e-5 * max|q_ref| + 1e-5; actions equal the oracle's argmax wherever the top-two gap
exceeds twice that."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from oracle import dqn  # noqa: E402
from deepreinforcementlearningcontrolofquantumcartpoles_amd.actor import MeasurementActor, random_dqn_measurement  # noqa: E402


def make_records(B, L, seed=0, scaling=0.5):
    """Measurement records shaped like MeasurementRecord.hist: q ~ N(0, 6^2) (the IHO measurement noise
    1/sqrt(2 gamma dt)) and piecewise-constant forces on the 0.8 grid, both times input_scaling."""
    rng = np.random.default_rng(seed)
    obs = np.empty((B, 2, L), np.float32)
    obs[:, 0] = rng.normal(0.0, 6.0, (B, L)) * scaling
    f = rng.integers(-10, 11, (B, L // 80 + 1)) * 0.8 * scaling
    obs[:, 1] = np.repeat(f, 80, axis=1)[:, :L]
    return obs


def check(q_dev, q_ref, act):
    scale = np.abs(q_ref).max()
    tol = 5e-5 * scale + 1e-5
    err = np.abs(q_dev - q_ref).max()
    assert err <= tol, (err, tol)
    srt = np.sort(q_ref, axis=1)
    clear = (srt[:, -1] - srt[:, -2]) > 2 * tol
    assert clear.mean() > 0.8
    np.testing.assert_array_equal(act[clear], q_ref.argmax(1)[clear])
    return err / scale


@pytest.mark.parametrize("L,B,chunk", [(5760, 100, 32), (4320, 37, 0), (5760, 2048, 0)])
def test_mactor_matches_oracle(L, B, chunk):
    p = random_dqn_measurement(read_length=L, seed=21)
    g = torch.Generator().manual_seed(1)
    for j in (1, 2, 3):
        p[f"conv{j}.bias"] = torch.randn(p[f"conv{j}.bias"].shape, generator=g) * 0.1
    actor = MeasurementActor({k: v.cuda() for k, v in p.items()}, read_length=L, max_batch=B, seed=3, chunk=chunk)
    obs = make_records(B, L, seed=B)
    rng = np.random.default_rng(2)
    noise = dqn.f_noise(rng.standard_normal((B, actor.noise_len))).astype(np.float32)
    act, ex = actor.act(torch.from_numpy(obs).cuda(), noise=torch.from_numpy(noise).cuda(), want_q=True,
                        want_random=True)
    sub = np.arange(B) if B <= 128 else np.unique(np.r_[0, 1, B - 1, np.linspace(0, B - 1, 61).astype(int)])
    q_ref = dqn.forward_measurement(p, obs[sub].astype(np.float64), noise[sub].astype(np.float64))
    check(ex["q"].cpu().numpy()[sub], q_ref, act.cpu().numpy()[sub])
    assert int(ex["random"].sum()) == 0


def test_mactor_mean_weights_and_keyed_noise():
    L, B = 5760, 64
    p = random_dqn_measurement(read_length=L, seed=4)
    actor = MeasurementActor({k: v.cuda() for k, v in p.items()}, read_length=L, max_batch=B, seed=9)
    obs = torch.from_numpy(make_records(B, L, seed=7)).cuda()
    act, ex = actor.act(obs, noisy=False, want_q=True)
    q_ref = dqn.forward_measurement(p, obs.cpu().double().numpy(), None)
    check(ex["q"].cpu().numpy(), q_ref, act.cpu().numpy())
    # in-kernel noise: the same counter reproduces, another counter differs
    _, a1 = actor.act(obs, counter=5, want_q=True)
    _, a2 = actor.act(obs, counter=5, want_q=True)
    _, a3 = actor.act(obs, counter=6, want_q=True)
    assert torch.equal(a1["q"], a2["q"]) and not torch.equal(a1["q"], a3["q"])


def test_mactor_drives_the_measurement_env():
    """One control step of BatchedEnv(input='measurements') with actions from the measurement actor."""
    from deepreinforcementlearningcontrolofquantumcartpoles_amd import config as cfg
    from deepreinforcementlearningcontrolofquantumcartpoles_amd.env import BatchedEnv
    env = BatchedEnv(cfg.DEFAULTS[cfg.IHO].with_(n_max=63), 64, 0, seed=2, input="measurements")
    obs = env.reset()
    actor = MeasurementActor({k: v.cuda() for k, v in random_dqn_measurement(seed=1).items()}, max_batch=64)
    for _ in range(2):
        a = actor.act(obs, eps=0.1)
        assert a.dtype == torch.int32 and bool(((a >= 0) & (a < 21)).all())
        obs, r, done, info = env.step(a)
    assert obs.shape == (64, 2, 5760)


def test_mactor_edge_cases_and_reload():
    """B = 0 is a no-op; wrong shapes and B > max_batch are refused; a weight of the wrong shape is refused
    at load; reloading other weights changes the answer to the oracle's for those weights."""
    L, B = 4320, 16
    p = random_dqn_measurement(read_length=L, seed=30)
    actor = MeasurementActor({k: v.cuda() for k, v in p.items()}, read_length=L, max_batch=B, seed=1)
    a0 = actor.act(torch.zeros((0, 2, L), device="cuda"))
    assert a0.shape == (0,)
    with pytest.raises(ValueError):
        actor.act(torch.zeros((B + 1, 2, L), device="cuda"))
    with pytest.raises(ValueError):
        actor.act(torch.zeros((4, 2, L - 1), device="cuda"))
    with pytest.raises(ValueError):
        actor.act(torch.zeros((4, 1, L), device="cuda"))
    bad = dict(p)
    bad["fc1.weight"] = torch.zeros(256, 17)
    with pytest.raises(ValueError):
        actor.load({k: v.cuda() for k, v in bad.items()})
    obs = make_records(B, L, seed=5)
    p2 = random_dqn_measurement(read_length=L, seed=31)
    actor.load({k: v.cuda() for k, v in p2.items()})
    act, ex = actor.act(torch.from_numpy(obs).cuda(), noisy=False, want_q=True)
    check(ex["q"].cpu().numpy(), dqn.forward_measurement(p2, obs.astype(np.float64), None), act.cpu().numpy())
