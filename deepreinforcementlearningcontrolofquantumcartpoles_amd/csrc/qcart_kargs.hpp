// qcart_kargs.hpp — the by-value argument block of the step / observation kernels (host+device).
#pragma once
#include <stdint.h>

namespace qcart {

struct KArgs {
    // state and I/O (device pointers)
    double* psi;               // [B][N] complex interleaved
    const int32_t* actions;    // [B] or null
    const int32_t* env_steps;  // [B] per-env step budget (min with n_steps) or null
    const double* noise;       // [n_steps][B][2] or null
    double* q_out;             // [n_steps][B] or null
    double* xm_out;            // [n_steps][B] or null
    int32_t* fail_step;        // [B] or null
    int32_t* term_step;        // [B] or null
    double* obs_out;           // [B][n_obs] or null
    int64_t B;
    int64_t env_offset;
    uint64_t seed;
    uint64_t step0;
    int32_t N;
    int32_t Npad;
    int32_t n_steps;
    int32_t default_action;
    int32_t n_slots;
    int32_t mirror;            // IHO reference-mode Hermitian mirror correction
    int32_t bnd_len;           // 5 (Fock) or 6 (grid)
    int32_t win_lo, win_hi;    // IQO outside-probability window [lo, hi); win_hi <= win_lo: off
    int32_t moment_order;
    int32_t n_obs;
    int32_t scan_lds;          // step kernel stages Kogge-Stone composites in LDS (Fock families)
    int32_t lv_f, lv_b;        // max forward / backward scan levels over the slots (LDS image size)
    uint32_t scan_lds_bytes;   // dynamic LDS per 4-wave block
    // physics scalars
    double dt, sqrt_dt, gamma, g4, beta, inv_sqrt2g, w, inv_sqrt_w, c, h;
    double a2, a3, a4, a5;     // Horner coefficients dt^3/12, dt^4/24, dt^5/80, dt^6/360
    double fail_thr;
    double hoff[5];            // grid constant H[r][r+d]
    // operator rows [Npad]
    const double* xu;          // Fock X[r][r+1]
    const double* xg;          // grid x_r
    const double* hu;          // IHO H[r][r+2]; HO / grid H[r][r]
    // per-slot factor tables
    const double* lc;          // complex [slot][kl][Npad]
    const double* uc;          // complex [slot][kl][Npad]
    const double* dinv;        // complex [slot][Npad]
    const double* m2;          // real    [slot][10][Npad]
    const double* tf;          // complex [slot][6][64][kl*kl]
    const double* tb;          // complex [slot][6][64][kl*kl]
    const int32_t* kf;         // [slot]
    const int32_t* kb;         // [slot]
    const double* force;       // [slot]
};

// host-side launchers (qcart_kernels.hip)
int launch_step(int family, int R, const KArgs& a, void* stream);
int launch_obs(int family, int R, const KArgs& a, void* stream);   // moments into obs_out
int launch_aux(int family, int R, int what, const KArgs& a, double xth, void* out, void* stream);
int launch_reset(int family, int R, const KArgs& a, int kind, const uint8_t* mask, double a0,
                 double a1, double a2, const double* k_arr, const double* m_arr, const double* s_arr,
                 void* stream);
bool have_kernel(int family, int R);

}  // namespace qcart
