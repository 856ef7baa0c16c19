"""ctypes binding of libqcart.so (include/qcart.h).

The library is the only compute path: if it is missing or no HIP device is present, every call
raises. There is deliberately no CPU fallback in this package.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# QCART_LIB selects an alternative in-tree build (A/B experiments); default: the package's libqcart.so
LIB_PATH = os.environ.get("QCART_LIB") or os.path.join(_HERE, "libqcart.so")

QC_HO, QC_IHO, QC_QO, QC_IQO = 0, 1, 2, 3
QC_A_REFERENCE, QC_A_EXACT = 0, 1
QC_RESET_GROUND, QC_RESET_RANDOM, QC_RESET_GAUSSIAN = 0, 1, 2
QC_CTL_LQG, QC_CTL_DAMPING, QC_CTL_SEMICLASSICAL = 0, 1, 2
QC_NOISE_PHILOX, QC_NOISE_MT19937 = 0, 1
CONTROL_STRATEGIES = {"LQG": QC_CTL_LQG, "damping": QC_CTL_DAMPING, "semiclassical": QC_CTL_SEMICLASSICAL}

STATUS = {
    0: "QC_OK", -1: "QC_EINVAL", -2: "QC_ENOMEM", -3: "QC_EHIP", -4: "QC_EPIVOT", -5: "QC_ESINGULAR",
    -6: "QC_ENOTBUILT",
}

# every symbol include/qcart.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "qc_create", "qc_destroy", "qc_last_error", "qc_abi_version", "qc_get_params", "qc_dim", "qc_n_obs",
    "qc_set_stream", "qc_sync", "qc_set_seed", "qc_set_step_counter", "qc_get_step_counter",
    "qc_env_counters", "qc_set_seed_mt19937", "qc_noise_mode", "qc_mt19937_state", "qc_mt19937_words",
    "qc_set_dynamics", "qc_add_force", "qc_step", "qc_moments", "qc_x_expectation", "qc_outside_prob",
    "qc_boundary_fail", "qc_energy", "qc_hamiltonian_dot_psi", "qc_phonon_number", "qc_reset", "qc_control", "qc_record_row_len", "qc_record",
    "qc_scan_levels", "qc_take_errors", "qc_step_group_size", "qc_group_layout", "qc_wavefunction_len", "qc_wavefunction_obs", "qc_set_timing", "qc_step_kernel_time",
    "qc_actor_create", "qc_actor_destroy", "qc_actor_last_error", "qc_actor_set_stream", "qc_actor_load",
    "qc_actor_noise_len", "qc_actor_act",
    "qc_mactor_create", "qc_mactor_destroy", "qc_mactor_last_error", "qc_mactor_set_stream", "qc_mactor_noise_len",
    "qc_mactor_flat_len", "qc_mactor_load", "qc_mactor_act",
    "qc_replay_create", "qc_replay_destroy", "qc_replay_last_error", "qc_replay_set_stream", "qc_replay_store",
    "qc_replay_store_xp", "qc_replay_sample", "qc_replay_update", "qc_replay_rebuild", "qc_replay_stats",
    "qc_replay_buffers", "qc_set_seed_mt19937_envs", "qc_mt19937_normals",
    "qc_server_create", "qc_server_run", "qc_server_stop", "qc_server_stats", "qc_server_timing", "qc_server_resident",
    "qc_server_last_error",
    "qc_server_destroy", "qc_env_tail",
)


class QcParams(ctypes.Structure):
    _fields_ = [
        ("family", ctypes.c_int32),
        ("n_max", ctypes.c_int32),
        ("omega", ctypes.c_double),
        ("x_max", ctypes.c_double),
        ("grid_size", ctypes.c_double),
        ("lambda_", ctypes.c_double),
        ("mass", ctypes.c_double),
        ("moment_order", ctypes.c_int32),
        ("a_mode", ctypes.c_int32),
        ("gamma", ctypes.c_double),
        ("dt", ctypes.c_double),
        ("f_max", ctypes.c_double),
        ("n_actions", ctypes.c_int32),
        ("precision", ctypes.c_int32),   # 0 fp64, 1 fp32 (Fock families; complex64 states)
        ("batch", ctypes.c_int64),
        ("env_offset", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("xth", ctypes.c_double),
    ]


class QcEnvTailArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int64),
        ("kind", ctypes.c_int32),
        ("n_obs", ctypes.c_int32),
        ("interval", ctypes.c_int32),
        ("pad", ctypes.c_int32),
        ("dt", ctypes.c_double),
        ("xth", ctypes.c_double),
        ("input_scaling", ctypes.c_double),
        ("failing_reward", ctypes.c_double),
        ("fail_step", ctypes.c_void_p),
        ("term_step", ctypes.c_void_p),
        ("obs", ctypes.c_void_p),
        ("pending", ctypes.c_void_p),
        ("t", ctypes.c_void_p),
        ("steps", ctypes.c_void_p),
        ("episode_return", ctypes.c_void_p),
        ("obs32", ctypes.c_void_p),
        ("reward", ctypes.c_void_p),
        ("done", ctypes.c_void_p),
        ("valid", ctypes.c_void_p),
        ("fin", ctypes.c_void_p),
        ("fin_cap", ctypes.c_int64),
        ("fin_n", ctypes.c_void_p),
    ]


class QcDqnParams(ctypes.Structure):
    _fields_ = [
        ("data_length", ctypes.c_int32),
        ("n_actions", ctypes.c_int32),
        ("max_batch", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
    ]


class QcMdqnParams(ctypes.Structure):
    _fields_ = [
        ("read_length", ctypes.c_int32),
        ("n_actions", ctypes.c_int32),
        ("max_batch", ctypes.c_int64),
        ("seed", ctypes.c_uint64),
        ("chunk", ctypes.c_int32),
    ]


class QcDqnLayer(ctypes.Structure):
    _fields_ = [
        ("weight", ctypes.c_void_p),
        ("bias", ctypes.c_void_p),
        ("weight_norm", ctypes.c_void_p),
        ("sigma_w", ctypes.c_void_p),
        ("sigma_b", ctypes.c_void_p),
    ]


class QcReplayParams(ctypes.Structure):
    _fields_ = [
        ("capacity", ctypes.c_int64),
        ("row_len", ctypes.c_int32),
        ("policy", ctypes.c_int32),
        ("passes_before_random", ctypes.c_double),
        ("alpha", ctypes.c_double),
        ("beta", ctypes.c_double),
        ("beta_increment", ctypes.c_double),
        ("abs_err_upper", ctypes.c_double),
        ("epsilon_scale", ctypes.c_double),
        ("seed", ctypes.c_uint64),
    ]


class QcReplayStats(ctypes.Structure):
    _fields_ = [
        ("len", ctypes.c_int64),
        ("data_pointer", ctypes.c_int64),
        ("passes", ctypes.c_double),
        ("max", ctypes.c_double),
        ("beta", ctypes.c_double),
        ("total_p", ctypes.c_double),
        ("n_nodes", ctypes.c_int64),
        ("tree_size", ctypes.c_int64),
    ]


class QCartError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{STATUS.get(code, code)}: {msg}")
        self.code = code


_lib = None


def _preload_torch_hip():
    # Reuse torch's HIP runtime (same SONAME libamdhip64.so.7) so that torch tensors and libqcart
    # share one runtime, one context and one stream namespace.
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not built: run `make` (or __graft_entry__.build()); this package has no CPU fallback")
    _preload_torch_hip()
    L = _Tolerant(ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)) if os.environ.get("QCART_LIB") else \
        ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    P, vp = ctypes.POINTER, ctypes.c_void_p
    i32, i64, u64, d = ctypes.c_int32, ctypes.c_int64, ctypes.c_uint64, ctypes.c_double
    L.qc_create.argtypes = [P(QcParams), ctypes.c_int, P(vp)]
    L.qc_destroy.argtypes = [vp]
    L.qc_destroy.restype = None
    L.qc_last_error.argtypes = [vp]
    L.qc_last_error.restype = ctypes.c_char_p
    L.qc_abi_version.argtypes = []
    L.qc_get_params.argtypes = [vp, P(QcParams)]
    L.qc_dim.argtypes = [vp]
    L.qc_n_obs.argtypes = [vp]
    L.qc_set_stream.argtypes = [vp, vp]
    L.qc_sync.argtypes = [vp]
    L.qc_set_seed.argtypes = [vp, u64]
    L.qc_set_step_counter.argtypes = [vp, u64]
    L.qc_get_step_counter.argtypes = [vp]
    L.qc_get_step_counter.restype = u64
    L.qc_env_counters.argtypes = [vp, vp, vp]
    L.qc_set_seed_mt19937.argtypes = [vp, vp]
    L.qc_set_seed_mt19937_envs.argtypes = [vp, vp, vp]
    L.qc_mt19937_normals.argtypes = [vp, ctypes.c_int32, vp, vp, vp, vp]
    L.qc_env_tail.argtypes = [vp, P(QcEnvTailArgs)]
    L.qc_server_create.argtypes = [P(QcParams), ctypes.c_int, i32, ctypes.c_char_p, d, P(vp)]
    L.qc_server_run.argtypes = [vp, d]
    L.qc_server_stop.argtypes = [vp]
    L.qc_server_stats.argtypes = [vp, P(i64), P(i64)]
    L.qc_server_timing.argtypes = [vp, vp]
    L.qc_server_resident.argtypes = [vp, P(i64), P(i64)]
    L.qc_server_last_error.argtypes = [vp]
    L.qc_server_last_error.restype = ctypes.c_char_p
    L.qc_server_destroy.argtypes = [vp]
    L.qc_server_destroy.restype = None
    L.qc_noise_mode.argtypes = [vp]
    L.qc_mt19937_state.argtypes = [vp, vp, vp]
    L.qc_mt19937_words.argtypes = []
    L.qc_set_dynamics.argtypes = [vp, d, d]
    L.qc_add_force.argtypes = [vp, d]
    L.qc_step.argtypes = [vp, vp, vp, i32, i32, vp, vp, vp, vp, vp, vp, vp]
    L.qc_moments.argtypes = [vp, vp, vp]
    L.qc_x_expectation.argtypes = [vp, vp, vp]
    L.qc_outside_prob.argtypes = [vp, vp, d, vp]
    L.qc_boundary_fail.argtypes = [vp, vp, vp]
    L.qc_energy.argtypes = [vp, vp, vp]
    L.qc_hamiltonian_dot_psi.argtypes = [vp, vp]
    L.qc_phonon_number.argtypes = [vp, vp, vp]
    L.qc_reset.argtypes = [vp, vp, i32, vp, d, d, d, vp, vp, vp]
    L.qc_control.argtypes = [vp, vp, i32, d, d, d, vp, vp]
    L.qc_record_row_len.argtypes = [i32, i32, i32]
    L.qc_record.argtypes = [vp, i32, i32, d, vp, i32, vp, i32, vp, vp, vp, vp, vp]
    L.qc_set_timing.argtypes = [vp, i32]
    L.qc_step_kernel_time.argtypes = [vp, P(d), P(i64)]
    L.qc_wavefunction_len.argtypes = [vp]
    L.qc_wavefunction_obs.argtypes = [vp, vp, d, vp]
    L.qc_scan_levels.argtypes = [vp, i32, P(i32), P(i32)]
    L.qc_step_group_size.argtypes = [vp]
    L.qc_group_layout.argtypes = [vp, vp, i64, vp, i64]
    for name in ("qc_take_errors",):   # (older in-tree builds in A/B runs lack them)
        if hasattr(L, name):
            getattr(L, name).argtypes = [vp]
    L.qc_actor_create.argtypes = [P(QcDqnParams), ctypes.c_int, P(vp)]
    L.qc_actor_destroy.argtypes = [vp]
    L.qc_actor_destroy.restype = None
    L.qc_actor_last_error.argtypes = [vp]
    L.qc_actor_last_error.restype = ctypes.c_char_p
    L.qc_actor_set_stream.argtypes = [vp, vp]
    L.qc_actor_load.argtypes = [vp, P(QcDqnLayer)]
    L.qc_actor_noise_len.argtypes = [vp]
    L.qc_actor_act.argtypes = [vp, i64, i64, vp, i32, vp, d, u64, vp, vp, vp]
    L.qc_mactor_create.argtypes = [P(QcMdqnParams), ctypes.c_int, P(vp)]
    L.qc_mactor_destroy.argtypes = [vp]
    L.qc_mactor_destroy.restype = None
    L.qc_mactor_last_error.argtypes = [vp]
    L.qc_mactor_last_error.restype = ctypes.c_char_p
    L.qc_mactor_set_stream.argtypes = [vp, vp]
    L.qc_mactor_noise_len.argtypes = [vp]
    L.qc_mactor_flat_len.argtypes = [vp]
    L.qc_mactor_load.argtypes = [vp, P(QcDqnLayer)]
    L.qc_mactor_act.argtypes = [vp, i64, i64, vp, i32, vp, d, u64, vp, vp, vp]
    L.qc_replay_create.argtypes = [P(QcReplayParams), ctypes.c_int, P(vp)]
    L.qc_replay_destroy.argtypes = [vp]
    L.qc_replay_destroy.restype = None
    L.qc_replay_last_error.argtypes = [vp]
    L.qc_replay_last_error.restype = ctypes.c_char_p
    L.qc_replay_set_stream.argtypes = [vp, vp]
    L.qc_replay_store.argtypes = [vp, i64, vp, vp]
    L.qc_replay_store_xp.argtypes = [vp, i64, vp, vp, vp, i32, vp, vp]
    L.qc_replay_sample.argtypes = [vp, i32, vp, vp, vp, vp]
    L.qc_replay_update.argtypes = [vp, i32, vp, vp]
    L.qc_replay_rebuild.argtypes = [vp]
    L.qc_replay_stats.argtypes = [vp, P(QcReplayStats)]
    L.qc_replay_buffers.argtypes = [vp, P(vp), P(vp)]
    if isinstance(L, _Tolerant):
        L = L.lib
    for name in EXPORTS:
        # every declared entry point must resolve in the shipped library (a stale build fails here); an
        # explicit QCART_LIB (A/B runs against older builds) may lack the newest ones
        if os.environ.get("QCART_LIB") and not hasattr(L, name):
            continue
        fn = getattr(L, name)
        if fn.restype is ctypes.c_int:   # default
            fn.restype = ctypes.c_int
    _lib = L
    return L


class _Tolerant:
    """An older in-tree build named by QCART_LIB (A/B runs): signatures of entry points it lacks are skipped."""

    class _Sink:
        argtypes = restype = None

    def __init__(self, lib):
        object.__setattr__(self, "lib", lib)

    def __getattr__(self, name):
        return getattr(self.lib, name) if hasattr(self.lib, name) else _Tolerant._Sink()


def check_actor(rc: int, handle=None) -> int:
    if rc < 0:
        msg = lib().qc_actor_last_error(handle)
        raise QCartError(rc, msg.decode() if msg else "")
    return rc


def check_mactor(rc: int, handle=None) -> int:
    if rc < 0:
        msg = lib().qc_mactor_last_error(handle)
        raise QCartError(rc, msg.decode() if msg else "")
    return rc


def check_replay(rc: int, handle=None) -> int:
    if rc < 0:
        msg = lib().qc_replay_last_error(handle)
        raise QCartError(rc, msg.decode() if msg else "")
    return rc


def check(rc: int, handle=None) -> int:
    if rc < 0:
        msg = lib().qc_last_error(handle)
        raise QCartError(rc, msg.decode() if msg else "")
    return rc
