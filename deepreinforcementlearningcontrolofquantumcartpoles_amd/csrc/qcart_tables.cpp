// qcart_tables.cpp — see qcart_tables.hpp.
#include "qcart_tables.hpp"

#include <algorithm>
#include <cmath>

#include "../../include/qcart.h"

namespace qcart {

namespace {

// Fortran/Smith complex reciprocal-free division a / b (as LAPACK's ZSCAL(ONE / pivot)).
cplx cdiv(cplx a, cplx b) {
    double ar = a.real(), ai = a.imag(), br = b.real(), bi = b.imag();
    if (std::fabs(br) >= std::fabs(bi)) {
        double t = bi / br, d = br + bi * t;
        return cplx((ar + ai * t) / d, (ai - ar * t) / d);
    }
    double t = br / bi, d = br * t + bi;
    return cplx((ar * t + ai) / d, (ai * t - ar) / d);
}
inline double cabs1(cplx a) { return std::fabs(a.real()) + std::fabs(a.imag()); }
inline cplx cm(cplx a, cplx b) {  // plain (a.re b.re - a.im b.im, a.re b.im + a.im b.re)
    return cplx(a.real() * b.real() - a.imag() * b.imag(), a.real() * b.imag() + a.imag() * b.real());
}

// real band product C = A B (half-widths ka, kb), layout [(d+k)*N + i] = M[i][i+d]
std::vector<double> band_mul(int N, const std::vector<double>& A, int ka, const std::vector<double>& B,
                             int kb, int& kc) {
    kc = ka + kb;
    std::vector<double> C((size_t)(2 * kc + 1) * N, 0.0);
    for (int i = 0; i < N; i++)
        for (int da = -ka; da <= ka; da++) {
            int k = i + da;
            if (k < 0 || k >= N) continue;
            double a = A[(size_t)(da + ka) * N + i];
            if (a == 0.0) continue;
            for (int db = -kb; db <= kb; db++) {
                int j = k + db;
                if (j < 0 || j >= N) continue;
                C[(size_t)(da + db + kc) * N + i] += a * B[(size_t)(db + kb) * N + k];
            }
        }
    return C;
}

// kl x kl complex matrices, row-major
using Mat = std::vector<cplx>;
Mat matmul(const Mat& A, const Mat& B, int n) {
    Mat C((size_t)n * n, cplx(0, 0));
    for (int i = 0; i < n; i++)
        for (int k = 0; k < n; k++) {
            cplx a = A[i * n + k];
            for (int j = 0; j < n; j++) C[i * n + j] += a * B[k * n + j];
        }
    return C;
}
Mat eye(int n) {
    Mat I((size_t)n * n, cplx(0, 0));
    for (int i = 0; i < n; i++) I[i * n + i] = 1.0;
    return I;
}
double maxabs(const Mat& A) {
    double m = 0;
    for (auto& v : A) m = std::max(m, std::abs(v));
    return m;
}

}  // namespace

// Set_World: IHO/simulation_i.cpp:45-151, HO/simulation.cpp:45-141, QO/simulation_quart.cpp:46-200
int build_ops(int family, int n_max, double omega, double x_max, double grid_size, double lambda_,
              double mass, int R, OpHost& op, std::string& err) {
    op = OpHost();
    op.family = family;
    op.fock = (family == QC_HO || family == QC_IHO);
    if (op.fock) {
        if (n_max < 4) { err = "n_max must be >= 4"; return QC_EINVAL; }
        op.N = n_max + 1;
        op.kl = (family == QC_HO) ? 1 : 2;
        op.w = 1.0;
        op.c = omega;
    } else if (family == QC_QO || family == QC_IQO) {
        if (!(grid_size > 0) || !(x_max > 0) || !(mass > 0)) { err = "bad grid parameters"; return QC_EINVAL; }
        op.x0 = (int)(x_max / grid_size + 0.5);     // QO/simulation_quart.cpp:21
        op.N = op.x0 * 2 + 1;
        op.kl = 4;
        op.w = grid_size;
        op.h = grid_size;
        op.c = M_PI;
    } else {
        err = "unknown family";
        return QC_EINVAL;
    }
    const int N = op.N, kl = op.kl;
    op.R = R;
    op.Npad = kWave * R;
    op.lanes = kWave;
    op.Rs = R;
    if (op.Npad < N) { err = "rows-per-lane too small"; return QC_EINVAL; }
    const int Np = op.Npad;
    op.hband.assign((size_t)(2 * kl + 1) * N, 0.0);
    op.abim.assign((size_t)(2 * kl + 1) * N, 0.0);
    op.xu.assign(Np, 0.0);
    op.xg.assign(Np, 0.0);
    op.hu.assign(Np, 0.0);
    auto HB = [&](int i, int d) -> double& { return op.hband[(size_t)(d + kl) * N + i]; };
    auto AB = [&](int i, int d) -> double& { return op.abim[(size_t)(d + kl) * N + i]; };
    if (op.fock) {
        // x_lower_diag[i] = sqrt(i+1) * sqrt(0.5)   IHO/simulation_i.cpp:65-75
        for (int i = 0; i + 1 < N; i++) op.xu[i] = std::sqrt((double)(i + 1)) * std::sqrt(0.5);
        if (family == QC_HO) {
            for (int i = 0; i < N; i++) {
                HB(i, 0) = omega * (0.5 + (double)i);          // HO/simulation.cpp:121
                AB(i, 0) = omega * (0.5 + (double)i) * 0.5;    // ab_center
                op.hu[i] = HB(i, 0);
            }
        } else {
            for (int i = 0; i + 2 < N; i++) {
                // H = -omega/2 (a+ a+ + a a): IHO/simulation_i.cpp:119-124
                double v = (-0.5 * omega) * (std::sqrt((double)(i + 1)) * std::sqrt((double)(i + 2)));
                HB(i, 2) = v;
                HB(i + 2, -2) = v;
                AB(i, 2) = v * 0.5;                             // ab_upper2, IHO :143-146
                AB(i + 2, -2) = v * 0.5;
                op.hu[i] = v;                                   // H[r][r+2]
            }
        }
    } else {
        const double h = grid_size;
        static const double num[5] = {-14350., 8064., -1008., 128., -9.};
        double d2[5];
        for (int d = 0; d < 5; d++) d2[d] = num[d] / 5040. / (h * h);      // QO :71-93
        for (int i = 0; i < N; i++) {
            double x = h * ((double)(i - op.x0));                          // QO :48
            op.xg[i] = x;
            double x2 = x * x, V = x2 * x2 * lambda_;                      // QO :49-50
            HB(i, 0) = (1. / (2. * mass)) * (-d2[0]) + V;                  // QO :182,191
            AB(i, 0) = (d2[0] * (-1.) / (2. * mass) + V) * 0.5;            // ab_center :73
            op.hu[i] = HB(i, 0);
            for (int d = 1; d <= 4; d++)
                if (i + d < N) {
                    double hv = (1. / (2. * mass)) * (-d2[d]);
                    HB(i, d) = hv;
                    HB(i + d, -d) = hv;
                    double av = 0.5 * d2[d] * (-1.) / (2. * mass);         // ab_upper/lower :77-93
                    AB(i, d) = av;
                    AB(i + d, -d) = av;
                }
        }
        for (int d = 1; d <= 4; d++) op.hoff[d] = (1. / (2. * mass)) * (-d2[d]);
    }
    return QC_OK;
}

// reset_ab(): IHO/simulation_i.cpp:227-277, HO/simulation.cpp:208-258, QO/simulation_quart.cpp:394-432
int build_action(const OpHost& op, double dt, double force, bool mirror, ActHost& act, std::string& err) {
    const int N = op.N, kl = op.kl, Np = op.Npad;
    act = ActHost();
    act.force = force;
    // ---- ab = I + i dt/2 H_F, dense band W[i][d], d in [-kl, kl]
    std::vector<cplx> W((size_t)N * (2 * kl + 1), cplx(0, 0));
    auto Wat = [&](int i, int d) -> cplx& { return W[(size_t)i * (2 * kl + 1) + (d + kl)]; };
    for (int i = 0; i < N; i++)
        for (int d = -kl; d <= kl; d++) {
            int j = i + d;
            if (j < 0 || j >= N) continue;
            double im = 0.0;
            if (op.fock) {
                if (d == 1 || d == -1) {
                    int lo = std::min(i, j);
                    // x_lower_diag_ab * (dt * F)   IHO :73-74, :230-235
                    im = ((-op.xu[lo]) * 0.5 * op.c) * (dt * force);
                } else {
                    im = op.abim[(size_t)(d + kl) * N + i] * dt;
                }
            } else {
                im = op.abim[(size_t)(d + kl) * N + i] * dt;
                if (d == 0) im += (-dt * force * 0.5 * M_PI) * op.xg[i];     // QO :397-399
            }
            Wat(i, d) = cplx(d == 0 ? 1.0 : 0.0, im);
        }
    // ---- pivot-free right-looking band LU (zgbtf2 arithmetic without interchanges)
    for (int j = 0; j < N; j++) {
        int km = std::min(kl, N - 1 - j);
        cplx piv = Wat(j, 0);
        for (int t = 1; t <= km; t++)
            if (cabs1(Wat(j + t, -t)) > cabs1(piv)) {
                err = "band LU would pivot (row " + std::to_string(j + t) + "); reduce dt";
                return QC_EPIVOT;
            }
        if (piv == cplx(0, 0)) { err = "singular band matrix"; return QC_ESINGULAR; }
        cplx rp = cdiv(cplx(1, 0), piv);
        for (int t = 1; t <= km; t++) Wat(j + t, -t) = cm(rp, Wat(j + t, -t));
        for (int cc = 1; cc <= km; cc++) {
            cplx y = Wat(j, cc);
            if (y == cplx(0, 0)) continue;
            for (int t = 1; t <= km; t++) Wat(j + t, cc - t) -= cm(Wat(j + t, -t), y);
        }
    }
    act.lc.assign((size_t)kl * Np, cplx(0, 0));
    act.uc.assign((size_t)kl * Np, cplx(0, 0));
    act.dinv.assign(Np, cplx(1, 0));
    for (int r = 0; r < N; r++) {
        cplx di = cdiv(cplx(1, 0), Wat(r, 0));
        act.dinv[r] = di;
        for (int k = 1; k <= kl; k++) {
            if (r - k >= 0) act.lc[(size_t)(k - 1) * Np + r] = Wat(r, -k);
            if (r + k < N) act.uc[(size_t)(k - 1) * Np + r] = cm(Wat(r, k), di);
        }
    }
    // ab is complex symmetric (H_F real symmetric), so U[r][r+k] / U[r][r] = L[r+k][r] up to rounding;
    // with L D L^T tables (op.sym) the step kernel reads the backward factors from the lc band, so the
    // backward composites are built from exactly those values
    if (op.sym)
        for (int k = 1; k <= kl; k++)
            for (int r = 0; r < Np; r++)
                act.uc[(size_t)(k - 1) * Np + r] = (r + k < Np) ? act.lc[(size_t)(k - 1) * Np + r + k] : cplx(0, 0);
    const int LN = op.lanes, RS = op.Rs;   // step-kernel lanes per env, rows per lane
    // ---- Kogge-Stone composites. Forward state s_r = (y_r, ..., y_{r-kl+1}),
    // s_r = A_r s_{r-1} + b_r e1, A_r = [[-l_1 .. -l_kl], shift]. Lane transition Phi_l = A_{lR+R-1}..A_{lR}.
    auto fwd_row = [&](int r) {
        Mat A((size_t)kl * kl, cplx(0, 0));
        for (int k = 0; k < kl; k++) A[k] = -act.lc[(size_t)k * Np + r];
        for (int i = 1; i < kl; i++) A[i * kl + (i - 1)] = 1.0;
        return A;
    };
    auto bwd_row = [&](int r) {
        Mat B((size_t)kl * kl, cplx(0, 0));
        for (int k = 0; k < kl; k++) B[k] = -act.uc[(size_t)k * Np + r];
        for (int i = 1; i < kl; i++) B[i * kl + (i - 1)] = 1.0;
        return B;
    };
    std::vector<Mat> Tk(LN), Qk(LN);
    for (int l = 0; l < LN; l++) {
        Mat P = eye(kl);
        for (int j = 0; j < RS; j++) P = matmul(fwd_row(l * RS + j), P, kl);
        Tk[l] = P;
        Mat Q = eye(kl);
        for (int j = RS - 1; j >= 0; j--) Q = matmul(bwd_row(l * RS + j), Q, kl);
        Qk[l] = Q;
    }
    const size_t blk = (size_t)kl * kl;
    act.tf.assign((size_t)kTabLevels * LN * blk, cplx(0, 0));
    act.tb.assign((size_t)kTabLevels * LN * blk, cplx(0, 0));
    // in-row (16-lane DPP row) products for the two-level scan: forward Pf(l) = Phi_l .. Phi_{row start},
    // backward Pb(l) = Psi_l .. Psi_{row end}; they carry a neighbouring row's end state into the row
    {
        std::vector<Mat> Pf(LN), Pb(LN);
        for (int l = 0; l < LN; l++) Pf[l] = (l % 16 == 0) ? Tk[l] : matmul(Tk[l], Pf[l - 1], kl);
        for (int l = LN - 1; l >= 0; l--) Pb[l] = (l % 16 == 15) ? Qk[l] : matmul(Qk[l], Pb[l + 1], kl);
        for (int l = 0; l < LN; l++) {
            std::copy(Pf[l].begin(), Pf[l].end(), act.tf.begin() + ((size_t)kRowPrefix * LN + l) * blk);
            std::copy(Pb[l].begin(), Pb[l].end(), act.tb.begin() + ((size_t)kRowPrefix * LN + l) * blk);
        }
    }
    for (int lvl = 0; lvl < kMaxLevels; lvl++) {
        const int d = 1 << lvl;
        double mf = 0, mb = 0;
        for (int l = 0; l < LN; l++) {
            if (l >= d) mf = std::max(mf, maxabs(Tk[l]));
            if (l + d < LN) mb = std::max(mb, maxabs(Qk[l]));
            std::copy(Tk[l].begin(), Tk[l].end(), act.tf.begin() + ((size_t)lvl * LN + l) * blk);
            std::copy(Qk[l].begin(), Qk[l].end(), act.tb.begin() + ((size_t)lvl * LN + l) * blk);
        }
        act.max_tf[lvl] = mf;
        act.max_tb[lvl] = mb;
        // next level: T_{k+1}(l) = T_k(l) T_k(l - d);  Q_{k+1}(l) = Q_k(l) Q_k(l + d)
        std::vector<Mat> T2(LN), Q2(LN);
        for (int l = 0; l < LN; l++) {
            T2[l] = (l - d >= 0) ? matmul(Tk[l], Tk[l - d], kl) : Tk[l];
            Q2[l] = (l + d < LN) ? matmul(Qk[l], Qk[l + d], kl) : Qk[l];
        }
        Tk.swap(T2);
        Qk.swap(Q2);
    }
    act.kf = kMaxLevels;
    act.kb = kMaxLevels;
    for (int lvl = kMaxLevels - 1; lvl >= 0; lvl--) {
        if (act.max_tf[lvl] <= kScanTol) act.kf = lvl; else break;
    }
    for (int lvl = kMaxLevels - 1; lvl >= 0; lvl--) {
        if (act.max_tb[lvl] <= kScanTol) act.kb = lvl; else break;
    }
    // ---- IHO reference (MKL HERMITIAN/UPPER) correction: A_eff = A - 2i tril(Im A, -1)
    act.m2.assign((size_t)kMirrorBands * Np, 0.0);
    if (mirror) {
        std::vector<double> HF((size_t)(2 * kl + 1) * N, 0.0);
        for (int i = 0; i < N; i++)
            for (int d = -kl; d <= kl; d++) {
                int j = i + d;
                if (j < 0 || j >= N) continue;
                double x = 0.0;
                if (op.fock) { if (d == 1) x = op.xu[i]; else if (d == -1) x = op.xu[j]; }
                else if (d == 0) x = op.xg[i];
                HF[(size_t)(d + kl) * N + i] = (-op.c * force) * x + op.hband[(size_t)(d + kl) * N + i];
            }
        int k2, k3, k5;
        auto P2 = band_mul(N, HF, kl, HF, kl, k2);
        auto P3 = band_mul(N, P2, k2, HF, kl, k3);
        auto P5 = band_mul(N, P2, k2, P3, k3, k5);
        const double c3 = dt * dt * dt * dt / 24., c5 = dt * dt * dt * dt * dt * dt / 360.;
        const int nb = std::min(kMirrorBands, 5 * kl);
        // MKL reads only the stored upper entry A[j][i] (j = i - d) and mirrors conj(A[j][i]) into
        // row i, so the correction uses Im of the UPPER entry: A_eff[i][j] = A[i][j] - 2i Im A[j][i].
        for (int i = 0; i < N; i++)
            for (int d = 1; d <= nb; d++) {
                int j = i - d;
                if (j < 0) continue;
                double p3 = (d <= k3) ? P3[(size_t)(d + k3) * N + j] : 0.0;
                double p5 = P5[(size_t)(d + k5) * N + j];
                double imA = (c5 * p5) + (-c3 * p3);          // Im A[j][j+d] (IHO :259-264)
                act.m2[(size_t)(d - 1) * Np + i] = 2.0 * imA;
            }
    }
    return QC_OK;
}

}  // namespace qcart
