// qcart_tables.hpp — host-side construction of the operator rows and per-action factor tables that
// the HIP step kernel streams. This is the MI355X-native replacement of the reference's
// Set_World constructor and reset_ab() (IHO/simulation_i.cpp:26-151, :227-277;
// HO/simulation.cpp:26-141, :208-258; QO/simulation_quart.cpp:28-209, :394-432).
//
// Instead of a per-call MKL banded LU + sparse spmm chain, every discrete force
// F_a = (a - 10) F_max / 10 (IHO/RL.py:107-111) gets, once per (dt, params):
//   * a pivot-free LU of ab = I + i dt/2 (H - c F X) (zgbtf2 arithmetic; refused with QC_EPIVOT if
//     partial pivoting would swap a row),
//   * the lane-composite transfer matrices of the Kogge-Stone scan that parallelises the banded
//     forward/backward substitutions across the 64 lanes of a wavefront,
//   * for the IHO reference mode, the strictly-lower band of Im(A) that turns the exact product
//     A.D1 (evaluated on device by Horner in H_F) into MKL's HERMITIAN/UPPER mirrored product.
#pragma once

#include <complex>
#include <cstdint>
#include <string>
#include <vector>

namespace qcart {

using cplx = std::complex<double>;

constexpr int kWave = 64;
constexpr int kMaxLevels = 6;     // log2(64)
constexpr int kTabLevels = 7;     // per direction: 6 Kogge-Stone levels + the in-row prefix product
constexpr int kRowPrefix = 6;     // table level holding the in-row prefix product (16-lane rows)
constexpr int kMirrorBands = 10;  // offsets -1..-10 of tril(Im A, -1) for the IHO (5*kl)
constexpr double kScanTol = 1e-22;  // drop Kogge-Stone levels whose composites are below this

struct OpHost {
    int family = 0;      // 0 HO, 1 IHO, 2 QO, 3 IQO
    bool fock = true;
    int N = 0, kl = 0, R = 0, Npad = 0, x0 = 0;
    // step-kernel factor tables: lanes per env and rows per lane (64 x R; 128 x R/2 for the two-waves-
    // per-env step kernel, the same Npad)
    int lanes = 64, Rs = 0;
    bool sym = false;    // L D L^T tables (slot_sym): the backward factors are read from the lc band
    double w = 1.0;      // dot weight (1 or h)
    double c = 0.0;      // force coupling (omega or pi)
    double h = 0.0;
    std::vector<double> xu;    // Fock: X[r][r+1], r in [0, Npad)
    std::vector<double> xg;    // grid: x_r
    std::vector<double> hu;    // IHO: H[r][r+2]; HO/grid: H[r][r] (diag incl. V)
    std::vector<double> hband; // full real band (2kl+1) x N, [(d+kl)*N + i] = H[i][i+d]
    std::vector<double> abim;  // imag(ab) at F = 0 by the reference's own construction, (2kl+1) x N
    double hoff[5] = {0, 0, 0, 0, 0};  // grid constant H[r][r+d], d = 1..4
};

struct ActHost {
    double force = 0.0;
    int kf = 0, kb = 0;               // Kogge-Stone levels kept (forward, backward)
    std::vector<cplx> lc;             // [kl][Npad]  L[r][r-k]
    std::vector<cplx> uc;             // [kl][Npad]  U[r][r+k] / U[r][r]
    std::vector<cplx> dinv;           // [Npad]      1 / U[r][r]
    std::vector<double> m2;           // [10][Npad]  2 Im A[r][r-d]   (IHO reference mode only)
    std::vector<cplx> tf;             // [7][64][kl*kl] forward composites  T_k(l); [6]: row prefix
    std::vector<cplx> tb;             // [7][64][kl*kl] backward composites Q_k(l); [6]: row suffix
    double max_tf[kMaxLevels] = {0}, max_tb[kMaxLevels] = {0};
};

// Returns 0 or a qc_status code; err receives a message.
int build_ops(int family, int n_max, double omega, double x_max, double grid_size, double lambda_,
              double mass, int R, OpHost& op, std::string& err);
int build_action(const OpHost& op, double dt, double force, bool mirror, ActHost& act,
                 std::string& err);

}  // namespace qcart
