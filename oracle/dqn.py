"""numpy restatement of the reference direct_DQN forward pass and the actor's action choice.

TEST INFRASTRUCTURE ONLY (the checker of the device actor, csrc/qcart_actor.hip): imported by tests/
and tools/, never by the product package. fp64 throughout.

Follows, in the reference tree `implementation codes/inverted harmonic oscillator/`:
  RL.py:96-102     direct_DQN.forward: relu(fc1) -> relu(fc2) -> fc31 -> relu -> fc41 (action values);
                   the mean branch fc32/fc42 does not enter the action
  layers.py:97-103 Linear_weight_normalize: F.linear(x, W / ||W||_F * weight_norm, b)
  layers.py:31-59  FactorizedNoisy (per-sample noise): w = u_w + sigma_w * (eps_out eps_in^T),
                   b = u_b + sigma_b * eps_out, eps = f(z) = sign(z) sqrt|z| (layers.py:77-79)
  main_parallel.py:436 actions = action_values.max(1)[1]
Parity anchor: no reference outputs exist for the network; the restatement is pinned by
the tests' hand-built cases (identity-like layers, explicit outer-product noise).
"""
from __future__ import annotations

import numpy as np

HIDDEN = (512, 256, 256)


def noise_len(n_actions: int = 21) -> int:
    return 2 * HIDDEN[1] + HIDDEN[2] + n_actions


def _np(v):
    try:
        return v.detach().cpu().double().numpy()
    except AttributeError:
        return np.asarray(v, dtype=np.float64)


def layer(params, name):
    """('wn', W_eff, b) or ('noisy', u_w, u_b, sigma_w, sigma_b) for one layer of a state_dict."""
    if f"{name}.u_w" in params:
        return ("noisy", _np(params[f"{name}.u_w"]), _np(params[f"{name}.u_b"]), _np(params[f"{name}.sigma_w"]),
                _np(params[f"{name}.sigma_b"]))
    w = _np(params[f"{name}.weight"])
    g = float(_np(params[f"{name}.weight_norm"]).reshape(-1)[0])
    return ("wn", w / np.linalg.norm(w) * g, _np(params[f"{name}.bias"]))


def _apply(lay, x, eps_in=None, eps_out=None):
    if lay[0] == "wn" or eps_in is None:
        w, b = (lay[1], lay[2])
        return x @ w.T + b
    _, u, ub, s, sb = lay
    # per-sample w_e = u + s * outer(eps_out_e, eps_in_e): y_e = u x_e + eps_out_e * (s (eps_in_e x_e) + sb) + ub
    return x @ u.T + ub + eps_out * ((x * eps_in) @ s.T + sb)


def forward(params, obs, noise=None, n_actions: int = 21):
    """Action values [B, n_actions] for obs [B, in]; noise [B, noise_len] (f-transformed) or None for
    the mean weights."""
    x = np.asarray(obs, dtype=np.float64)
    h1, h2, h3 = HIDDEN
    if noise is not None:
        nz = np.asarray(noise, dtype=np.float64)
        e_in31, e_out31 = nz[:, :h2], nz[:, h2:2 * h2]
        e_in41, e_out41 = nz[:, 2 * h2:2 * h2 + h3], nz[:, 2 * h2 + h3:2 * h2 + h3 + n_actions]
    else:
        e_in31 = e_out31 = e_in41 = e_out41 = None
    x = np.maximum(_apply(layer(params, "fc1"), x), 0.0)
    x = np.maximum(_apply(layer(params, "fc2"), x), 0.0)
    x = np.maximum(_apply(layer(params, "fc31"), x, e_in31, e_out31), 0.0)
    return _apply(layer(params, "fc41"), x, e_in41, e_out41)


def f_noise(z):
    """layers.py:77-79"""
    return np.sign(z) * np.sqrt(np.abs(z))


# ---- DQN_measurement (RL.py:29-78): conv1 -> relu -> conv2 -> relu -> conv3 -> relu -> view -> fc1 -> relu
#      -> fc21 (noisy) -> relu -> fc31 (noisy)
M_CONV = ((13, 5), (11, 4), (9, 4))   # (kernel, stride) of conv1..3, no padding


def conv1d(x, w, b, stride):
    """F.conv1d(x [B, ci, L], w [co, ci, k], b, stride) without padding, fp64."""
    k = w.shape[2]
    win = np.lib.stride_tricks.sliding_window_view(x, k, axis=2)[:, :, ::stride, :]   # [B, ci, T, k]
    return np.einsum("bctk,ock->bot", win, w, optimize=True) + b[None, :, None]


def forward_measurement(params, obs, noise=None, n_actions: int = 21):
    """Action values [B, n_actions] for obs [B, 2, L]; noise [B, 789] (f-transformed) or None."""
    x = np.asarray(obs, dtype=np.float64)
    for j, (_, s) in enumerate(M_CONV):
        x = np.maximum(conv1d(x, _np(params[f"conv{j + 1}.weight"]), _np(params[f"conv{j + 1}.bias"]), s), 0.0)
    x = x.reshape(x.shape[0], -1)
    x = np.maximum(x @ _np(params["fc1.weight"]).T + _np(params["fc1.bias"]), 0.0)
    h = 256
    if noise is not None:
        nz = np.asarray(noise, dtype=np.float64)
        e_in21, e_out21 = nz[:, :h], nz[:, h:2 * h]
        e_in31, e_out31 = nz[:, 2 * h:3 * h], nz[:, 3 * h:3 * h + n_actions]
    else:
        e_in21 = e_out21 = e_in31 = e_out31 = None
    x = np.maximum(_apply(layer(params, "fc21"), x, e_in21, e_out21), 0.0)
    return _apply(layer(params, "fc31"), x, e_in31, e_out31)
