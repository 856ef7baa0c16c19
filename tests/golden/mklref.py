"""The reference's third-party arithmetic (Intel MKL), driven through ctypes — TEST INFRASTRUCTURE ONLY.

The reference stepper is C++ glue over MKL: sparse BLAS for H, x̂ and the correction
factor A, LAPACKE band LU, VSL for the noise. Compiling or running the reference itself was denied
here, but the MKL runtime it links is in this image (/opt/conda/lib/libmkl_rt.so,
MKL 2021.4.0, conda-meta mkl-2021.4.0-h06a4308_640). This module restates the reference's call
sequences — the same MKL routines with the same descriptors, operations and order — so the fixtures
it produces (make_mkl_fixtures.py) pin the oracle at the MKL boundary:

  * IhoMkl: Set_World (IHO/simulation_i.cpp:44-152), reset_ab (:222-277) and go_one_step with D1 /
    D1ImRe / D2 / simple_sum_up / zgbtrs / normalize / check_boundary_error (:168-220, :279-333,
    :422-489, :546-573), every vector operation the same cblas / mkl_sparse call as the reference;
  * band_lu: LAPACKE_zgbtrf / zgbtrs row-major as reset_ab calls them (IHO:250-251,487; QO:410-411,622);
  * grid_p_relative: the quartic p̂ - p̄ I of compute_statistics (QO/simulation_quart.cpp:170-178,
    :326-337, :283-286) with the identity copied under {HERMITIAN, UPPER, DIAG_UNIT};
  * vsl_*: vslNewStream(VSL_BRNG_MT19937) + viRngUniformBits / vdRngGaussian(BOXMULLER) (:435,:577).

Loaded only by tests/golden/make_mkl_fixtures.py (fixture generation, in this container) and by the
CPU tests that re-derive a fixture when MKL is present; never by the product or a GPU run.
"""
from __future__ import annotations

import ctypes
import os
from math import pi, sqrt

import numpy as np

MKL_PATH = os.environ.get("QCART_MKL_RT", "/opt/conda/lib/libmkl_rt.so")

# mkl_spblas.h / mkl_vsl_defines.h / lapacke.h constants
OP_N, OP_T, OP_C = 10, 11, 12
T_GENERAL, T_SYMMETRIC, T_HERMITIAN, T_DIAGONAL = 20, 21, 22, 24
F_UPPER = 41
D_NON_UNIT, D_UNIT = 50, 51
BASE0 = 0
BRNG_MT19937 = 8 << 20
GAUSS_BOXMULLER = 0
ROW_MAJOR = 101


class Z(ctypes.Structure):
    _fields_ = [("re", ctypes.c_double), ("im", ctypes.c_double)]


class Descr(ctypes.Structure):
    _fields_ = [("type", ctypes.c_int), ("mode", ctypes.c_int), ("diag", ctypes.c_int)]


_mkl = None


def available() -> bool:
    return os.path.exists(MKL_PATH)


def mkl():
    global _mkl
    if _mkl is None:
        m = ctypes.CDLL(MKL_PATH)
        vp, i, d = ctypes.c_void_p, ctypes.c_int, ctypes.c_double
        P = ctypes.POINTER
        m.mkl_sparse_z_create_csr.argtypes = [P(vp), i, i, i, vp, vp, vp, vp]
        m.mkl_sparse_copy.argtypes = [vp, Descr, P(vp)]
        m.mkl_sparse_z_add.argtypes = [i, vp, Z, vp, P(vp)]
        m.mkl_sparse_spmm.argtypes = [i, vp, vp, P(vp)]
        m.mkl_sparse_z_mv.argtypes = [i, Z, vp, Descr, vp, Z, vp]
        m.mkl_sparse_set_mv_hint.argtypes = [vp, i, Descr, i]
        m.mkl_sparse_optimize.argtypes = [vp]
        m.mkl_sparse_order.argtypes = [vp]
        m.mkl_sparse_destroy.argtypes = [vp]
        m.mkl_sparse_z_export_csr.argtypes = [vp, P(i), P(i), P(i), P(P(ctypes.c_int)), P(P(ctypes.c_int)),
                                              P(P(ctypes.c_int)), P(P(Z))]
        m.LAPACKE_zgbtrf.argtypes = [i, i, i, i, i, vp, i, vp]
        m.LAPACKE_zgbtrs.argtypes = [i, ctypes.c_char, i, i, i, i, vp, i, vp, vp, i]
        m.cblas_zdotc_sub.argtypes = [i, vp, i, vp, i, vp]
        m.cblas_dznrm2.argtypes = [i, vp, i]
        m.cblas_dznrm2.restype = d
        m.cblas_zdscal.argtypes = [i, d, vp, i]
        m.cblas_daxpy.argtypes = [i, d, vp, i, vp, i]
        m.cblas_dcopy.argtypes = [i, vp, i, vp, i]
        m.cblas_dscal.argtypes = [i, d, vp, i]
        m.cblas_zcopy.argtypes = [i, vp, i, vp, i]
        m.MKL_Set_Num_Threads.argtypes = [i]
        m.vslNewStream.argtypes = [P(vp), i, ctypes.c_uint]
        m.vslDeleteStream.argtypes = [P(vp)]
        m.viRngUniformBits.argtypes = [i, vp, i, vp]
        m.vdRngGaussian.argtypes = [i, vp, i, vp, d, d]
        m.vslGetStreamSize.argtypes = [vp]
        m.vslSaveStreamM.argtypes = [vp, vp]
        m.vslLoadStreamM.argtypes = [P(vp), vp]
        m.MKL_Set_Num_Threads(1)   # mkl_set_num_threads(1), IHO/simulation_i.cpp:15-16
        _mkl = m
    return _mkl


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ok(st, what):
    if st != 0:
        raise RuntimeError(f"{what} failed: status {st}")


# ------------------------------------------------------------------------------------------- sparse
class Sparse:
    """An MKL sparse handle plus the host arrays it borrows (create_csr does not copy)."""

    def __init__(self, h, keep=()):
        self.h = h
        self.keep = keep

    @staticmethod
    def csr(dense: np.ndarray) -> "Sparse":
        n = dense.shape[0]
        rows, cols = np.nonzero(dense)
        ia = np.zeros(n + 1, np.int32)
        np.add.at(ia, rows + 1, 1)
        ia = np.cumsum(ia).astype(np.int32)
        ja = cols.astype(np.int32)
        val = np.ascontiguousarray(dense[rows, cols].astype(np.complex128))
        if val.size == 0:   # the reference's "empty_matrix": one stored explicit zero (IHO:53-62)
            ia = np.ones(n + 1, np.int32)
            ia[0] = 0
            ja = np.zeros(1, np.int32)
            val = np.zeros(1, np.complex128)
        h = ctypes.c_void_p()
        _ok(mkl().mkl_sparse_z_create_csr(ctypes.byref(h), BASE0, n, n, _p(ia), _p(ia[1:]), _p(ja), _p(val)),
            "create_csr")
        return Sparse(h, (ia, ja, val))

    def copy(self, t, mode, diag) -> "Sparse":
        h = ctypes.c_void_p()
        _ok(mkl().mkl_sparse_copy(self.h, Descr(t, mode, diag), ctypes.byref(h)), "copy")
        return Sparse(h)

    def add(self, op, alpha: complex, other: "Sparse") -> "Sparse":
        """op(self) * alpha + other (mkl_sparse_z_add)."""
        h = ctypes.c_void_p()
        _ok(mkl().mkl_sparse_z_add(op, self.h, Z(alpha.real, alpha.imag), other.h, ctypes.byref(h)), "z_add")
        return Sparse(h)

    def mm(self, other: "Sparse") -> "Sparse":
        h = ctypes.c_void_p()
        _ok(mkl().mkl_sparse_spmm(OP_N, self.h, other.h, ctypes.byref(h)), "spmm")
        return Sparse(h)

    def hint_optimize(self, descr: Descr, calls: int, order: bool = False):
        _ok(mkl().mkl_sparse_set_mv_hint(self.h, OP_N, descr, calls), "set_mv_hint")
        if order:
            _ok(mkl().mkl_sparse_order(self.h), "order")
        _ok(mkl().mkl_sparse_optimize(self.h), "optimize")

    def mv(self, alpha: complex, descr: Descr, x: np.ndarray, beta: complex, y: np.ndarray):
        _ok(mkl().mkl_sparse_z_mv(OP_N, Z(alpha.real, alpha.imag), self.h, descr, _p(x),
                                  Z(beta.real, beta.imag), _p(y)), "z_mv")

    def dense(self) -> np.ndarray:
        m = mkl()
        base, r, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        rs, re_, ci = ctypes.POINTER(ctypes.c_int)(), ctypes.POINTER(ctypes.c_int)(), ctypes.POINTER(ctypes.c_int)()
        v = ctypes.POINTER(Z)()
        _ok(m.mkl_sparse_z_export_csr(self.h, ctypes.byref(base), ctypes.byref(r), ctypes.byref(c), ctypes.byref(rs),
                                      ctypes.byref(re_), ctypes.byref(ci), ctypes.byref(v)), "export_csr")
        out = np.zeros((r.value, c.value), np.complex128)
        for i in range(r.value):
            for k in range(rs[i] - base.value, re_[i] - base.value):
                out[i, ci[k] - base.value] += complex(v[k].re, v[k].im)
        return out

    def __del__(self):
        try:
            if self.h:
                mkl().mkl_sparse_destroy(self.h)
        except Exception:
            pass


# --------------------------------------------------------------------------------------- LAPACKE
def band_lu(A_band_rows: np.ndarray, kl: int):
    """LAPACKE_zgbtrf(ROW_MAJOR, n, n, kl, kl, ab_LU, ldab = n, ipiv) as reset_ab calls it: ab_LU has
    3kl+1 rows, the 2kl+1 band rows of ab copied from row kl down (IHO:249-251, QO:410-411).
    A_band_rows[r][j] = A(j + kl - r... ) i.e. the LAPACKE row-major band: row kl+ku+i-j of column j = A(i, j)
    counted from the copy offset. Returns (ab_LU [3kl+1][n], ipiv 1-based [n])."""
    n = A_band_rows.shape[1]
    ab = np.zeros((3 * kl + 1, n), np.complex128)
    ab[kl:] = A_band_rows
    ipiv = np.zeros(n, np.int32)
    _ok(mkl().LAPACKE_zgbtrf(ROW_MAJOR, n, n, kl, kl, _p(ab), n, _p(ipiv)), "zgbtrf")
    return ab, ipiv


def band_solve(ab: np.ndarray, ipiv: np.ndarray, kl: int, b: np.ndarray) -> np.ndarray:
    """LAPACKE_zgbtrs(ROW_MAJOR, 'N', n, kl, kl, 1, ab_LU, n, ipiv, b, 1) (IHO:487, QO:622)"""
    x = np.ascontiguousarray(b.astype(np.complex128)).copy()
    n = ab.shape[1]
    _ok(mkl().LAPACKE_zgbtrs(ROW_MAJOR, b"N", n, kl, kl, 1, _p(ab), n, _p(ipiv), _p(x), 1), "zgbtrs")
    return x


def band_rows(M: np.ndarray, kl: int) -> np.ndarray:
    """The reference's row-major ab[2kl+1][n]: ab[kl + i - j][j] = M(i, j) (upper diagonals first)."""
    n = M.shape[0]
    ab = np.zeros((2 * kl + 1, n), np.complex128)
    for d in range(-kl, kl + 1):          # d = i - j
        for j in range(max(0, -d), min(n, n - d)):
            ab[kl + d][j] = M[j + d, j]
    return ab


# ------------------------------------------------------------------------------------------- VSL
def vsl_stream(seed: int):
    s = ctypes.c_void_p()
    _ok(mkl().vslNewStream(ctypes.byref(s), BRNG_MT19937, ctypes.c_uint(seed & 0xFFFFFFFF)), "vslNewStream")
    return s


def vsl_bits(seed: int, n: int) -> np.ndarray:
    s = vsl_stream(seed)
    out = np.zeros(n, np.uint32)
    _ok(mkl().viRngUniformBits(0, s, n, _p(out)), "viRngUniformBits")
    mkl().vslDeleteStream(ctypes.byref(s))
    return out


def vsl_gaussian(seed: int, n: int) -> np.ndarray:
    """n normals as the reference draws them: vdRngGaussian(BOXMULLER, stream, 2, r, 0, 1) per step."""
    s = vsl_stream(seed)
    out = np.zeros(n, np.float64)
    for k in range(0, n, 2):
        _ok(mkl().vdRngGaussian(GAUSS_BOXMULLER, s, 2, _p(out[k:]), 0.0, 1.0), "vdRngGaussian")
    mkl().vslDeleteStream(ctypes.byref(s))
    return out


# MT19937 stream memory (vslSaveStreamM, MKL 2021.4): 32-bit words 5..628 are mt19937ar's state array, word
# 629 its read index (the next output is temper(mt[index]); 624 = a twist is due) — found by comparing the
# saved memory with mt19937ar at several positions
_MT_OFF, _MT_IDX = 5, 629


def vsl_planted_zero(seed: int, k: int, zero_at, n_normals: int):
    """The stream of `seed` after k words with the state words at positions k + z (z in zero_at) set to 0
    (their tempered output is then 0), loaded back by vslLoadStreamM: returns (state [625] = mt[624] +
    index, the same layout as the oracle's MT19937.st, and the next n_normals vdRngGaussian(BOXMULLER)
    normals, drawn 2 per call like the reference)."""
    m = mkl()
    s = vsl_stream(seed)
    if k:
        buf = np.zeros(k, np.uint32)
        _ok(m.viRngUniformBits(0, s, k, _p(buf)), "viRngUniformBits")
    mem = np.zeros(m.vslGetStreamSize(s), np.uint8)
    _ok(m.vslSaveStreamM(s, _p(mem)), "vslSaveStreamM")
    m.vslDeleteStream(ctypes.byref(s))
    w = mem[: len(mem) // 4 * 4].view(np.uint32)
    assert 0 < k < 624 and int(w[_MT_IDX]) == k and all(k + z < 624 for z in zero_at)
    for z in zero_at:
        w[_MT_OFF + k + z] = 0
    state = np.concatenate([w[_MT_OFF:_MT_OFF + 624], w[_MT_IDX:_MT_IDX + 1]]).copy()
    s2 = ctypes.c_void_p()
    _ok(m.vslLoadStreamM(ctypes.byref(s2), _p(mem)), "vslLoadStreamM")
    out = np.zeros(n_normals, np.float64)
    for j in range(0, n_normals, 2):
        _ok(m.vdRngGaussian(GAUSS_BOXMULLER, s2, 2, _p(out[j:]), 0.0, 1.0), "vdRngGaussian")
    m.vslDeleteStream(ctypes.byref(s2))
    return state, out


# -------------------------------------------------------------------------------------- IHO stepper
class IhoMkl:
    """The inverted-harmonic `simulation` module (N_MAX = n_max, OMEGA = omega) in its own MKL calls."""

    def __init__(self, n_max: int, omega: float):
        self.n_max, self.N, self.omega = n_max, n_max + 1, omega
        n = self.N
        self.descr = Descr(T_HERMITIAN, F_UPPER, D_NON_UNIT)       # IHO:23
        self.h_descr = self.a_descr = self.descr                    # H mv (IHO:292,314), term7 mv (:551)
        self.fcoef, self.x_w = omega, None                          # -omega F x ; <x> unweighted (Fock)
        empty = Sparse.csr(np.zeros((n, n)))
        self.empty = empty
        # annihilation: the distance-1 diagonal sqrt(i+1) (mkl_dcsrdia of sqrt_n_append1, IHO:80-94)
        ann_d = np.zeros((n, n), np.complex128)
        for i in range(n - 1):
            ann_d[i, i + 1] = sqrt(float(i + 1))
        tmp = Sparse.csr(ann_d)
        ann = tmp.copy(T_GENERAL, F_UPPER, D_NON_UNIT)
        cre = ann.add(OP_T, 1.0, empty)
        t = cre.add(OP_N, complex(sqrt(0.5), 0.0), empty)
        self.x_hat = ann.add(OP_N, complex(sqrt(0.5), 0.0), t)
        t2 = cre.mm(cre)
        t3 = ann.mm(ann)
        t4 = t2.add(OP_N, complex(-0.5 * omega, 0.0), empty)
        self.H = t3.add(OP_N, complex(-0.5 * omega, 0.0), t4)
        mkl().mkl_sparse_order(self.H.h)
        mkl().mkl_sparse_order(self.x_hat.h)
        self.H.hint_optimize(self.descr, 100000000)
        mkl().mkl_sparse_optimize(self.x_hat.h)
        # x_upper/lower_diag (IHO:70-76); ab_upper2 = H's +2 diagonal * 0.5 (IHO:132-140)
        sq1 = np.array([sqrt(float(i + 1)) for i in range(n - 1)] + [0.0])
        self.x_lower = sq1 * sqrt(0.5)
        self.x_lower_ab = -self.x_lower * 0.5 * omega
        Hd = self.H.dense()
        self.ab_upper2 = np.array([Hd[i, i + 2].real * 0.5 for i in range(n - 2)])
        self._dt = self._force = None

    # compute_x_hat_state (IHO:168-196) — the reference's own loops, elementwise in the same order
    def x_state(self, alpha: float, psi: np.ndarray, beta: float, result: np.ndarray | None):
        p = psi.view(np.float64)
        xl = self.x_lower
        n_max = self.n_max
        out = np.zeros(2 * self.N) if result is None else result.view(np.float64)
        new = np.empty(2 * self.N)
        new[0] = alpha * (p[2] * xl[0])
        new[1] = alpha * (p[3] * xl[0])
        i = np.arange(1, n_max)
        new[2 * i] = alpha * (p[2 * i + 2] * xl[i] + p[2 * i - 2] * xl[i - 1])
        new[2 * i + 1] = alpha * (p[2 * i + 3] * xl[i] + p[2 * i - 1] * xl[i - 1])
        new[2 * n_max] = alpha * (p[2 * n_max - 2] * xl[n_max - 1])
        new[2 * n_max + 1] = alpha * (p[2 * n_max - 1] * xl[n_max - 1])
        if beta == 0.0:
            out[:] = new
        else:
            out *= beta
            out += new
        return out.view(np.complex128)

    def zdotc_re(self, a, b) -> float:
        r = np.zeros(1, np.complex128)
        mkl().cblas_zdotc_sub(self.N, _p(a), 1, _p(b), 1, _p(r))
        return float(r[0].real)

    def _avg(self, a, b) -> float:
        """temp.real (Fock) or temp.real * grid_size (grid, QO:235,460,482) of zdotc(a, b)"""
        v = self.zdotc_re(a, b)
        return v if self.x_w is None else v * self.x_w

    def daxpy(self, a: float, x, y):
        mkl().cblas_daxpy(2 * self.N, a, _p(x), 1, _p(y), 1)

    def x_expct(self, psi) -> float:
        xs = self.x_state(1.0, psi, 0.0, None)
        return self._avg(psi, xs)

    def reset_ab(self, dt: float, force: float):
        """IHO:222-277: ab (5 x N, imaginary parts), its LU, and the correction factor A."""
        n, om = self.N, self.omega
        ab = np.zeros((5, n), np.complex128)
        ab[2].real = 1.0
        coef = dt * force
        up1 = self.x_lower_ab[:n - 1] * coef           # ab[3][0..], copied to ab[1][1..] (IHO:229-235)
        ab[3, :n - 1].imag = up1
        ab[1, 1:].imag = up1
        up2 = self.ab_upper2 * dt                       # ab[4][0..], copied to ab[0][2..] (IHO:236-244)
        ab[4, :n - 2].imag = up2
        ab[0, 2:].imag = up2
        self.ab_LU, self.ipiv = band_lu(ab, 2)
        h0 = self.x_hat.add(OP_N, complex(-om * force, 0.0), self.H)
        h2 = h0.mm(h0)
        h3 = h2.mm(h0)
        h4 = h2.mm(h2)
        h5 = h2.mm(h3)
        d3, d4, d5, d6 = dt * dt * dt, dt * dt * dt * dt, dt * dt * dt * dt * dt, dt * dt * dt * dt * dt * dt
        a5 = h2.add(OP_N, complex(d3 / 12., 0.), self.empty)
        a6 = h3.add(OP_N, complex(0., -d4 / 24.), a5)
        a7 = h4.add(OP_N, complex(-d5 / 80., 0.), a6)
        self.A = h5.add(OP_N, complex(0., d6 / 360.), a7)
        self.A.hint_optimize(Descr(T_SYMMETRIC, F_UPPER, D_NON_UNIT), 80, order=True)
        self._dt, self._force = dt, force

    def D1(self, state, force, gamma, x_avg):
        """IHO:279-298 -> (result, relative_state)"""
        xs = self.x_state(1.0, state, 0.0, None).copy()
        rel = xs.copy()
        self.daxpy(-x_avg, state, rel)
        self.H.mv(complex(0., -1.), self.h_descr, state, complex(0., self.fcoef * force), xs)
        result = xs.copy()
        xs = rel.copy()
        self.x_state(1.0, rel, -x_avg, xs)
        self.daxpy(-gamma / 4., xs, result)
        return result, rel

    def D1ImRe(self, state, force, gamma):
        """IHO:301-318 -> (resultIm, resultRe, relative_state)"""
        rIm = self.x_state(1.0, state, 0.0, None).copy()
        x_avg = self._avg(state, rIm)
        rel = rIm.copy()
        self.daxpy(-x_avg, state, rel)
        self.H.mv(complex(0., -1.), self.h_descr, state, complex(0., self.fcoef * force), rIm)
        rRe = rel.copy()
        self.x_state(-gamma / 4., rel, x_avg * gamma / 4., rRe)
        return rIm, rRe, rel

    def D2(self, state, gamma, rr, precomputed: bool):
        """IHO:321-333 (in place on rr)"""
        if not precomputed:
            rr[:] = self.x_state(1.0, state, 0.0, None)
            x_avg = self._avg(state, rr)
            self.daxpy(-x_avg, state, rr)
        mkl().cblas_zdscal(self.N, sqrt(gamma / 2.), _p(rr), 1)

    def step(self, psi: np.ndarray, dt: float, force: float, gamma: float, r):
        """step() (IHO:358-389): reset_ab on a dt / force change, go_one_step, check_boundary_error."""
        if dt != self._dt or force != self._force:
            self.reset_ab(dt, force)
        n = self.N
        r0, r1 = float(r[0]), float(r[1])
        dW = r0 * sqrt(dt)
        dZ = sqrt(dt) * dt * 0.5 * (r0 + r1 / sqrt(3.))
        x_mean = self.x_expct(psi)
        q = x_mean + dW / sqrt(2. * gamma) / dt
        D1s, D2s = self.D1(psi, force, gamma, x_mean)
        self.D2(psi, gamma, D2s, True)
        D2drt = np.zeros(n, np.complex128)
        self.daxpy(sqrt(dt), D2s, D2drt)
        Yp = psi.copy()
        self.daxpy(dt, D1s, Yp)
        Ym = Yp.copy()
        self.daxpy(1., D2drt, Yp)
        self.daxpy(-1., D2drt, Ym)
        D1pIm, D1pRe, D2Yp = self.D1ImRe(Yp, force, gamma)
        D1mIm, D1mRe, D2Ym = self.D1ImRe(Ym, force, gamma)
        self.D2(Yp, gamma, D2Yp, True)
        self.D2(Ym, gamma, D2Ym, True)
        self.daxpy(-1., D1mIm, D1pIm)                    # D1_Y_plusIm_substract_D1_Y_minusIm
        Phim = Yp.copy()
        self.daxpy(-sqrt(dt), D2Yp, Phim)
        Phip = Yp
        self.daxpy(sqrt(dt), D2Yp, Phip)
        D2Pp = np.zeros(n, np.complex128)
        D2Pm = np.zeros(n, np.complex128)
        self.D2(Phip, gamma, D2Pp, False)
        self.D2(Phim, gamma, D2Pm, False)
        # simple_sum_up (IHO:546-573), the loop over the 2N doubles written in the same order
        term7 = np.zeros(n, np.complex128)
        self.A.mv(complex(1., 0.), self.a_descr, D1s, complex(0., 0.), term7)
        s = psi.view(np.float64)
        d2, sub, pRe, mRe = D2s.view(np.float64), D1pIm.view(np.float64), D1pRe.view(np.float64), D1mRe.view(np.float64)
        d1, yp, ym = D1s.view(np.float64), D2Yp.view(np.float64), D2Ym.view(np.float64)
        pp, pm, t7 = D2Pp.view(np.float64), D2Pm.view(np.float64), term7.view(np.float64)
        s += (d2 * dW + 0.5 / sqrt(dt) * dZ * (sub + pRe - mRe)
              + 0.25 * dt * (pRe + 2 * d1 + mRe)
              + 0.25 / sqrt(dt) * (dW * dW - dt) * (yp - ym)
              + 0.5 / dt * (dW * dt - dZ) * (yp + ym - 2 * d2)
              + 0.25 / dt * (dW * dW / 3 - dt) * dW * (pp - pm - yp + ym)
              - 0.25 * sqrt(dt) * dW * (sub)
              + t7)
        psi[:] = band_solve(self.ab_LU, self.ipiv, self.kl, psi)
        self.normalize(psi)
        return q, x_mean, self.fail(psi)

    kl = 2

    def normalize(self, psi):
        """IHO:216-220"""
        norm = mkl().cblas_dznrm2(self.N, _p(psi), 1)
        mkl().cblas_zdscal(self.N, 1. / norm, _p(psi), 1)

    def fail(self, psi) -> int:
        """check_boundary_error, IHO:422-426"""
        n = self.N
        return int(mkl().cblas_dznrm2(5, _p(psi[n - 5:]), 1) > 2.e-3)


# --------------------------------------------------------------------------------------- HO stepper
class HoMkl(IhoMkl):
    """The harmonic `simulation` module (HO/simulation.cpp) in its own MKL calls. The step is IHO's
    go_one_step (HO:413-470, simple_sum_up :527-544) with the harmonic Hamiltonian: a diagonal CSR H
    multiplied under the {DIAGONAL, UPPER} descriptor (HO:23,272,294), term7 under {SYMMETRIC, UPPER}
    (HO:532), the tridiagonal ab (kl = 1, HO:208-232) and Fail at |psi[N-5:]| > 1e-3 (HO:403-407)."""

    kl = 1

    def __init__(self, n_max: int, omega: float):
        self.n_max, self.N, self.omega = n_max, n_max + 1, omega
        n = self.N
        self.h_descr = Descr(T_DIAGONAL, F_UPPER, D_NON_UNIT)      # HO:23
        self.a_descr = Descr(T_SYMMETRIC, F_UPPER, D_NON_UNIT)     # HO:252,532
        self.descr = self.h_descr
        self.fcoef, self.x_w = omega, None
        empty = Sparse.csr(np.zeros((n, n)))
        self.empty = empty
        ann_d = np.zeros((n, n), np.complex128)                     # mkl_dcsrdia of sqrt_n_append1 (HO:86-97)
        for i in range(n - 1):
            ann_d[i, i + 1] = sqrt(float(i + 1))
        ann = Sparse.csr(ann_d).copy(T_GENERAL, F_UPPER, D_NON_UNIT)
        cre = ann.add(OP_T, 1.0, empty)                             # HO:98
        t = cre.add(OP_N, complex(sqrt(0.5), 0.0), empty)           # HO:101-102
        self.x_hat = ann.add(OP_N, complex(sqrt(0.5), 0.0), t)
        # H = omega (0.5 + n) on the diagonal (mkl_zcsrdia, HO:119-124)
        self.H = Sparse.csr(np.diag([omega * (0.5 + float(i)) for i in range(n)]).astype(np.complex128))
        mkl().mkl_sparse_order(self.H.h)                            # HO:125-131
        mkl().mkl_sparse_order(self.x_hat.h)
        self.H.hint_optimize(self.h_descr, 100000000)
        mkl().mkl_sparse_optimize(self.x_hat.h)
        sq1 = np.array([sqrt(float(i + 1)) for i in range(n - 1)] + [0.0])
        self.x_lower = sq1 * sqrt(0.5)                              # x_lower_diag (HO:70-75)
        self.x_lower_ab = -self.x_lower * 0.5 * omega
        self.ab_center = np.array([omega * (0.5 + float(i)) * 0.5 for i in range(n)])
        self._dt = self._force = None

    def reset_ab(self, dt: float, force: float):
        """HO:208-258: ab (3 x N, imaginary parts: the x coupling on +-1, H dt / 2 on the diagonal), its LU,
        and the correction factor A (same spmm / z_add chain as the IHO, SYMMETRIC hint)."""
        n, om = self.N, self.omega
        ab = np.zeros((3, n), np.complex128)
        ab[1].real = 1.0
        ab[2, :n - 1].imag = self.x_lower_ab[:n - 1] * (dt * force)    # dcopy + dscal (HO:213-214)
        ab[0, 1:].imag = ab[2, :n - 1].imag                           # HO:216
        ab[1].imag = self.ab_center * dt                              # HO:222-224
        self.ab_LU, self.ipiv = band_lu(ab, 1)
        self.A = _a_chain(self.x_hat.add(OP_N, complex(-om * force, 0.0), self.H), dt, self.empty)
        self.A.hint_optimize(self.a_descr, 80, order=True)
        self._dt, self._force = dt, force

    def fail(self, psi) -> int:
        n = self.N
        return int(mkl().cblas_dznrm2(5, _p(psi[n - 5:]), 1) > 1.e-3)


def _a_chain(h0: Sparse, dt: float, empty: Sparse) -> Sparse:
    """The correction factor dt^3/12 H^2 - i dt^4/24 H^3 - dt^5/80 H^4 + i dt^6/360 H^5 as the reference
    builds it: spmm powers, then z_add from the lowest order up (IHO:253-272, HO:234-245, QO:414-425)."""
    h2 = h0.mm(h0)
    h3 = h2.mm(h0)
    h4 = h2.mm(h2)
    h5 = h2.mm(h3)
    d3, d4, d5, d6 = dt * dt * dt, dt * dt * dt * dt, dt * dt * dt * dt * dt, dt * dt * dt * dt * dt * dt
    a5 = h2.add(OP_N, complex(d3 / 12., 0.), empty)
    a6 = h3.add(OP_N, complex(0., -d4 / 24.), a5)
    a7 = h4.add(OP_N, complex(-d5 / 80., 0.), a6)
    return h5.add(OP_N, complex(0., d6 / 360.), a7)


# ------------------------------------------------------------------------------------- grid stepper
class GridMkl(IhoMkl):
    """The quartic `simulation` module (QO/simulation_quart.cpp; the inverted quartic's file is the same
    code with lambda < 0) in its own MKL calls: Set_World's dense -> CSR operators (QO:46-200), reset_ab
    (:394-432), D1 / D1ImRe / D2 with the diagonal x and the 9-band H under {SYMMETRIC, UPPER} (:434-486,
    :25), simple_sum_up (:626-644), zgbtrs with kl = 4 (:622), normalize with sqrt(h) (:259-263), the
    two-ended check_boundary_error (:559-565) and compute_statistics (:326-362)."""

    kl = 4

    def __init__(self, x_max: float, grid_size: float, lambda_: float, mass: float, moment_order: int = 5):
        h = grid_size
        xc = int(x_max / h + 0.5)
        n = 2 * xc + 1
        self.N, self.h, self.mass, self.lam, self.moment_order = n, h, mass, lambda_, moment_order
        self.omega = None
        self.descr = Descr(T_SYMMETRIC, F_UPPER, D_NON_UNIT)       # QO:25
        self.h_descr = self.a_descr = self.descr
        self.herm = Descr(T_HERMITIAN, F_UPPER, D_NON_UNIT)         # p_hat (QO:198,239,285)
        self.fcoef, self.x_w = pi, h
        self.x = np.array([h * float(i - xc) for i in range(n)])     # QO:48-50
        x2 = self.x * self.x
        V = x2 * x2 * lambda_
        dx = np.zeros((n, n), np.complex128)                         # QO:59-70
        for k, v in ((1, 672.), (2, -168.), (3, 32.), (4, -3.)):
            for i in range(k, n - k):
                dx[i, i - k] = -v / 840. / h
                dx[i - k, i] = v / 840. / h
        d2 = np.zeros((n, n), np.complex128)                         # QO:71-93
        self.ab_upper = np.zeros((4, n))
        self.ab_lower = np.zeros((4, n))
        hh = h * h
        for i in range(n):
            d2[i, i] = -14350. / 5040. / hh
        self.ab_center = (d2.diagonal().real * (-1.) / (2. * mass) + V) * 0.5
        for k, v in ((1, 8064.), (2, -1008.), (3, 128.), (4, -9.)):
            for i in range(k, n):
                d2[i, i - k] = v / 5040. / hh
                d2[i - k, i] = v / 5040. / hh
                c = 0.5 * d2[i, i - k].real * (-1.) / (2. * mass)
                self.ab_upper[4 - k, i] = c
                self.ab_lower[k - 1, i - k] = c
        self.empty = empty = Sparse.csr(np.zeros((n, n)))
        # mkl_zdnscsr / mkl_zcsrdia keep the nonzero entries (zeros left out); then mkl_sparse_copy
        delta_x = Sparse.csr(dx).copy(T_GENERAL, F_UPPER, D_NON_UNIT)                       # QO:118-126
        delta_2_x = Sparse.csr(d2).copy(T_SYMMETRIC, F_UPPER, D_NON_UNIT)                   # QO:130-137
        self.x_hat = Sparse.csr(np.diag(self.x).astype(np.complex128)).copy(T_DIAGONAL, F_UPPER, D_NON_UNIT)
        V_hat = Sparse.csr(np.diag(V).astype(np.complex128)).copy(T_DIAGONAL, F_UPPER, D_NON_UNIT)
        self.identity = Sparse.csr(np.eye(n, dtype=np.complex128)).copy(T_HERMITIAN, F_UPPER, D_UNIT)
        self.p_hat = delta_x.add(OP_N, complex(0., -1.), empty)                              # QO:181-182
        p_hat_2 = delta_2_x.add(OP_N, complex(-1., 0.), empty)
        self.H = p_hat_2.add(OP_N, complex(1. / (2. * mass), 0.), V_hat)                     # QO:191-199
        mkl().mkl_sparse_order(self.H.h)
        mkl().mkl_sparse_order(self.x_hat.h)
        mkl().mkl_sparse_order(self.p_hat.h)
        self.H.hint_optimize(self.descr, 10000000)
        self.p_hat.hint_optimize(self.herm, 1000000)
        self._keep = (delta_x, delta_2_x, V_hat, p_hat_2)
        self._dt = self._force = None

    # compute_x_hat_state (QO:214-229): x diagonal, element by element in the reference's order
    def x_state(self, alpha: float, psi: np.ndarray, beta: float, result):
        p = psi.view(np.float64).reshape(-1, 2)
        xs = self.x[:, None]
        if beta == 0.0:
            return np.ascontiguousarray((alpha * p) * xs).view(np.complex128).reshape(-1)
        out = result.view(np.float64).reshape(-1, 2)
        out *= beta
        out += (alpha * p) * xs
        return result

    def reset_ab(self, dt: float, force: float):
        """QO:394-432. The diagonal's imaginary part is dcopy + dscal + daxpy in MKL (:397-399); the
        off-diagonals dt * ab_upper / ab_lower (:402-405)."""
        n, m = self.N, mkl()
        ab = np.zeros((9, n), np.complex128)
        ab[4].real = 1.0
        abd = ab.view(np.float64)                      # [9][2n]: imaginary parts at odd offsets
        row = 2 * n
        m.cblas_dcopy(n, _p(self.ab_center), 1, abd[4:].ctypes.data + 8, 2)
        m.cblas_dscal(n, dt, abd[4:].ctypes.data + 8, 2)
        m.cblas_daxpy(n, -dt * force * 0.5 * pi, _p(self.x), 1, abd[4:].ctypes.data + 8, 2)
        up = np.ascontiguousarray(self.ab_upper.reshape(-1))
        lo = np.ascontiguousarray(self.ab_lower.reshape(-1))
        m.cblas_dcopy(4 * n, _p(up), 1, abd.ctypes.data + 8, 2)
        m.cblas_dscal(4 * n, dt, abd.ctypes.data + 8, 2)
        m.cblas_dcopy(4 * n, _p(lo), 1, abd[5:].ctypes.data + 8, 2)
        m.cblas_dscal(4 * n, dt, abd[5:].ctypes.data + 8, 2)
        assert abd.shape[1] == row
        self.ab = ab
        self.ab_LU, self.ipiv = band_lu(ab, 4)
        self.A = _a_chain(self.x_hat.add(OP_N, complex(-pi * force, 0.), self.H), dt, self.empty)
        self.A.hint_optimize(self.descr, 80, order=True)
        self._dt, self._force = dt, force

    def normalize(self, psi):
        norm = mkl().cblas_dznrm2(self.N, _p(psi), 1)
        mkl().cblas_zdscal(self.N, 1. / norm / sqrt(self.h), _p(psi), 1)

    def fail(self, psi) -> int:
        n = self.N
        return int(mkl().cblas_dznrm2(6, _p(psi[n - 6:]), 1) > 5.e-3 or mkl().cblas_dznrm2(6, _p(psi), 1) > 5.e-3)

    def p_expct(self, psi) -> float:
        """QO:237-243"""
        y = np.zeros(self.N, np.complex128)
        self.p_hat.mv(complex(1., 0.), self.herm, psi, complex(0., 0.), y)
        return self.zdotc_re(psi, y) * self.h

    def moments(self, psi: np.ndarray) -> np.ndarray:
        """compute_statistics (QO:326-362): <x>, <p>, then the centred moments of orders 2..m."""
        psi = np.ascontiguousarray(psi, np.complex128)
        mo, n, h = self.moment_order, self.N, self.h
        data = [self.x_expct(psi), self.p_expct(psi)]
        x_rel = self.x - data[0]
        p_rel = self.identity.add(OP_N, complex(-data[1], 0.), self.p_hat)
        p_rel.hint_optimize(self.herm, 5)
        temp = np.zeros((mo + 1, n), np.complex128)
        tv = temp.view(np.float64).reshape(mo + 1, n, 2)
        pv = psi.view(np.float64).reshape(n, 2)
        tv[0] = pv * x_rel[:, None]
        p_rel.mv(complex(1., 0.), self.herm, psi, complex(0., 0.), temp[1])
        for i in range(2, mo + 1):
            p_rel.mv(complex(1., 0.), self.herm, temp[i - 1], complex(0., 0.), temp[i])
        for j in range(2, mo + 1):
            for i in range(j):
                tv[i] *= x_rel[:, None]
            for i in range(j + 1):
                data.append(self.zdotc_re(psi, temp[i]) * h)
        return np.array(data)


# ------------------------------------------------------------------------------- quartic p̂ - p̄ I
def grid_delta_x(x_n: int, h: float) -> np.ndarray:
    """delta_x_dense of QO/simulation_quart.cpp:63-76, with the reference's loop bounds."""
    d = np.zeros((x_n, x_n))
    for k, v in ((1, 672.), (2, -168.), (3, 32.), (4, -3.)):
        for i in range(k, x_n - k):
            d[i, i - k] = -v / 840. / h
            d[i - k, i] = v / 840. / h
    return d


def grid_p_relative(x_n: int, h: float, pbar: float, v: np.ndarray) -> np.ndarray:
    """(p̂ - p̄ I) v as compute_statistics applies it: p_hat = delta_x * (-i) (QO:180), identity copied
    with {HERMITIAN, UPPER, DIAG_UNIT} (:170-178), p_hat_relative = identity * (-p̄) + p_hat (:337) under
    the {HERMITIAN, UPPER, NON_UNIT} hint, mv with that descriptor (:283-286)."""
    empty = Sparse.csr(np.zeros((x_n, x_n)))
    dx = Sparse.csr(grid_delta_x(x_n, h).astype(np.complex128))
    p_hat = dx.add(OP_N, complex(0., -1.), empty)
    ident = Sparse.csr(np.eye(x_n, dtype=np.complex128)).copy(T_HERMITIAN, F_UPPER, D_UNIT)
    prel = ident.add(OP_N, complex(-pbar, 0.), p_hat)
    d = Descr(T_HERMITIAN, F_UPPER, D_NON_UNIT)
    prel.hint_optimize(d, 5)
    y = np.zeros(x_n, np.complex128)
    prel.mv(complex(1., 0.), d, np.ascontiguousarray(v, np.complex128), complex(0., 0.), y)
    return y
