// qcart_kargs.hpp — the by-value argument block of the step / observation kernels (host+device).
#pragma once
#include <stdint.h>

namespace qcart {

// One force slot's factor tables as one contiguous block, every band / level lane-interleaved:
// row r = l*R + j of band b at element (b*R + j)*64 + l, scan composite e of level v of lane l at
// (v*kl*kl + e)*64 + l. A wave's j-th read of a band is then one contiguous 64-element run, and the
// step kernel addresses the block with one buffer descriptor and constant offsets.
//   lc   complex [kl][R][64]    L[r][r-k]                      (zgbtrs forward)
//   uc   complex [kl][R][64]    U[r][r+k] / U[r][r]            (zgbtrs backward; absent when sym)
//   di   complex [R][64]        1 / U[r][r]
//   m2   real    [10][R][64]    2 Im A[r-d][r] (IHO only; zero unless the reference mirror mode)
//   tf   complex [7][kl*kl][64] forward Kogge-Stone composites, level 6 = in-row prefix product
//   tb   complex [7][kl*kl][64] backward composites, level 6 = in-row suffix product
// sym (slot_sym): ab = I + i dt/2 H_F is complex symmetric, so its pivot-free LU is L D L^T and
// U[r][r+k] / U[r][r] = L[r+k][r]: the backward substitution reads the lc band at row r + k (the next
// lane's run for rows past the lane) and the block carries no uc band.
struct SlotLayout {
    uint32_t lc, uc, di, m2, tf, tb, bytes;
};
// es: bytes of one complex element (16 fp64, 8 fp32); real bands use es / 2
// lanes: lanes per env (64) — the run length of every band
constexpr SlotLayout slot_layout(int kl, int R, bool has_m2, uint32_t es = 16, bool sym = false, int lanes = 64) {
    SlotLayout L{};
    const uint32_t ln = (uint32_t)lanes;
    L.lc = 0;
    L.uc = L.lc + es * ln * (uint32_t)(kl * R);
    L.di = L.uc + (sym ? 0u : es * ln * (uint32_t)(kl * R));
    L.m2 = L.di + es * ln * (uint32_t)R;
    L.tf = L.m2 + (has_m2 ? (es / 2) * ln * 10u * (uint32_t)R : 0u);
    L.tb = L.tf + es * ln * 7u * (uint32_t)(kl * kl);
    L.bytes = L.tb + es * ln * 7u * (uint32_t)(kl * kl);
    return L;
}

// L D L^T tables (no uc band): every fp64 family (ab = I + i dt/2 H_F is complex symmetric for every
// Hamiltonian here); the fp32 kernel (C5) keeps the uc band (its L D L^T layout was measured slower:
// DESIGN.md §4). lanes: the run length of the tables (64 = one wave per env)
constexpr bool slot_sym(bool fock, uint32_t es, int lanes) { return !fock || lanes > 64 || es == 16; }

// scan levels per direction the MODE 2 LDS image keeps (forward levels, prefix, backward levels, suffix):
// 4 for the Fock bands (kl <= 2), 2 for the grid's kl = 4 (its 16-element composites)
constexpr int mode2_levels(int kl) { return kl >= 4 ? 2 : 4; }
// grid step kernels that read their per-row constants (H_F's folded diagonal, x_r) from the LDS image
// instead of holding them in registers: the R = 17 kernel, whose step spills (for R <= 9 the registers
// are there and the LDS reads cost more than they save: C4 12.6 -> 14.9 ms, C3 29.4 -> 27.9 ms)
constexpr bool grid_rows_in_lds(int R) { return R >= 17; }
// bytes of LDS per wave for the step loop's noise refill (64 steps x 2 normals): fp64 kernels with LDS tables
constexpr uint32_t kNzLds = 1024;

// boundary bands of check_boundary_error: the top kFockBnd Fock levels (IHO/simulation_i.cpp:422-426,
// HO/simulation.cpp:403-407), kGridBnd points at either end of the grid (QO/simulation_quart.cpp:559-565). The
// grid step kernel's normalise is specialised on kGridBnd at compile time (qcart_kernels.hpp)
constexpr int kFockBnd = 5;
// grid moment orders (get_moments' MOMENT, QO/setupC.py:16,38): up to kMaxMomentOrder the observation kernel holds
// observable i in lane i of the env's wave, (2 + m + 1) m / 2 <= 64 (m = 9: 54 observables); its second instantiation
// holds observable i in lane i % 64, register i / 64, up to kMaxMomentOrderHi (m = 16: 152 observables, 3 per lane).
// The step server's shared-object rows hold 64 observables (QCS_MAX_OBS): it serves orders up to kMaxMomentOrder
constexpr int kMaxMomentOrder = 9;
constexpr int kMaxMomentOrderHi = 16;
// the step kernel's fused observation epilogue covers orders up to this one (qc_step runs the observation kernel
// after the step for higher orders)
constexpr int kStepMaxMomentOrder = 6;
constexpr int kGridBnd = 6;

struct KArgs {
    // state and I/O (device pointers)
    void* psi;                 // [B][N] complex interleaved, fp64 or fp32 (precision)
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
    uint64_t* ctr;             // [B] per-env noise counters: env e's Philox counter of its next step
    int32_t N;
    int32_t Npad;
    int32_t n_steps;
    int32_t default_action;
    int32_t n_slots;
    int32_t mirror;            // IHO reference-mode Hermitian mirror correction
    int32_t bnd_len;           // kFockBnd (Fock) or kGridBnd (grid)
    int32_t win_lo, win_hi;    // IQO outside-probability window [lo, hi); win_hi <= win_lo: off
    int32_t moment_order;
    int32_t n_obs;
    int32_t precision;         // 0 fp64, 1 fp32 (psi storage and step arithmetic)
    int32_t tab_mode;          // step kernel factor tables: 0 global, 1 LDS (lc/uc/di/m2), 2 + composites, 4 + forward composites
    uint32_t lds_bytes;        // dynamic LDS per block for tab_mode >= 1
    uint32_t lds_fx;           // LDS offset of the H_F force coefficients (Fock, tab_mode >= 1)
    const int32_t* order;      // [n_blocks*W] envs grouped by force slot (-1 idle) or null (identity)
    uint32_t n_blocks;         // step kernel grid (single-slot workgroups)
    const int32_t* order_mixed;   // [n_mixed*W] k_group's two-slot remainder workgroups (-1 idle)
    uint32_t n_mixed;          // capacity of two-slot blocks (0: none; launch_step DUAL); grid n_mixed + n_blocks
    const int32_t* n_mixed_used;   // device: k_group's two-slot workgroup count (blocks [0, it) run them)
    uint32_t lds_img;          // bytes of one slot's MODE 3 image (tables + H_F force coefficients)
    uint32_t lds_nz;           // LDS offset of the per-wave noise buffers (fp64, tab_mode >= 1: kNzLds bytes per wave)
    // physics scalars
    double dt, sqrt_dt, gamma, g4, beta, inv_sqrt2g, w, inv_sqrt_w, c, h;
    double a2, a3, a4, a5;     // Horner coefficients dt^3/12, dt^4/24, dt^5/80, dt^6/360
    double fail_thr;
    double hoff[5];            // grid constant H[r][r+d]
    // operator rows [Npad]
    const double* xu;          // Fock X[r][r+1]
    const double* xg;          // grid x_r
    const double* hu;          // IHO H[r][r+2]; HO / grid H[r][r]
    // per-slot factor blocks (see SlotLayout), slot s at tab + s * slot_bytes
    const double* tab;
    uint32_t slot_bytes;
    const int32_t* kf;         // [slot]
    const int32_t* kb;         // [slot]
    const double* force;       // [slot]
    // analytic controllers (qc_control)
    int32_t* act_out;          // [B]
    double* force_out;         // [B] or null
    int32_t ctl_strategy;      // enum qc_control_strategy
    int32_t ctl_half;          // no_action_choice (10)
    double ctl_param, ctl_time, ctl_scaling, ctl_fmax, ctl_lambda, ctl_mass;
    // step constants folded on the host (kernel arguments live in SGPRs; computed on the device they
    // were wave-uniform VGPR values that the step kernel spilled): 1/sqrt(dt), 1/dt, the SRK coefficient
    // prefactors 0.5/sqrt(dt), 0.25/sqrt(dt), 0.5/dt, 0.25/dt, 0.25 dt, 0.25 sqrt(dt), sqrt(dt) dt 0.5,
    // sqrt(dt) beta and the Horner ratios a2/a5, a3/a5, a4/a5 — each the same fp64 expression as before
    double inv_sdt, inv_dt, k_hisdt, k_qisdt, k_hidt, k_qidt, k_qdt, k_qsdt, k_dz, k_sb, b2, b3, b4;
    double x2h;                // IHO: -1/omega, X^2's +-2 bands as a multiple of H's (k_step X2H)
    int32_t* bad;              // the handle's error word: an out-of-range action of an ungrouped call (MODE 0)
    int32_t spread;            // MODE 0 without order: one env per block (wave 0; the block's other waves idle)
};

// the step server's resident kernel (k_resident, qcart_server.cpp): the per-request view of ONE step of ONE env that
// the step body takes in registers (RES) instead of through the KArgs arrays
struct ResIO {
    int32_t slot;               // in: the force slot (the request's action)
    int32_t reload;             // in: the block's LDS slot image holds another slot (MODE >= 1: copy it again)
    int32_t row_lds;            // in: take the row from the block's LDS copy (the one it returned last), not the client's
    uint32_t lds_row;           // in: byte offset of that copy in the dynamic LDS ([R][64] complex, written every step)
    double z0, z1;              // in: the step's two normals (the env's MT19937 stream)
    double q, xm;               // out: the step's q and x_mean
    int32_t fail;               // out: Fail (0 / 1)
};
// k_resident's second argument (KArgs stays the first: the step loop reads it through the kernarg segment, KAR)
struct ResArgs {
    void* slots;                // device address of the shm object's qcs_slot array (qcart_shm.h), slot e = block e
    const uint32_t* ctl;        // device address of the header's r_quit word; ctl[1] = r_beat
    uint32_t* mt;               // [B][kMtWords] the handle's MT19937 states (shared with the tick path's kernels)
    uint64_t beat_ticks;        // s_memrealtime ticks (100 MHz) without a heartbeat change before a wave exits
    uint64_t lease_ticks;       // s_memrealtime ticks after which an idle wave exits (the server relaunches the kernel)
    uint32_t gen;               // the server's dynamics generation (6 bits): a request of another one bounces
    uint32_t lds_row;           // byte offset of the row copy in the dynamic LDS
    double* obs;                // device address of the shm object's obs rows ([B][QCS_MAX_OBS])
};
int launch_resident(int family, int R, const KArgs& a, const ResArgs& r, void* stream);
bool have_resident(int family, int R);

// measurement-record update (qcart_record.hip, qc_record)
struct RecArgs {
    const double* q;            // [n_steps][B] step() q outputs of the interval
    const int32_t* actions;     // [B] or null (default_action)
    int32_t default_action;
    const double* slot_force;   // [slot] force of each action slot
    const uint8_t* mode;        // [B] 0 frozen, 1 record, 2 record into a fresh (zero) history; null = 1
    float* hist;                // [B][2][L] in place
    float* forces;              // [B][K + 1] in place
    float* rows;                // [B][row_len] or null
    const float* reward;        // [B] or null
    int64_t B;
    int32_t n_slots;            // action slots (out-of-range actions clamp like k_step's)
    int32_t* bad;               // the handle's error word: raised on an out-of-range action (qc_take_errors)
    int32_t L, m, K, cg, row_len;
    int32_t vec4;               // L, m multiples of 4: float4 history traffic
    double scaling;
};
int launch_record(const RecArgs& a, void* stream);
int launch_wavefunction(const void* psi, int precision, int64_t B, int32_t N, int32_t lo, int32_t cnt, double scaling,
                        float* out, void* stream);

// the batched episode loop's bookkeeping (qcart_env.hip, qc_env_tail): see qc_env_tail_args in qcart.h
struct EnvTailArgs {
    int64_t B;
    int32_t kind, n_obs, interval, pad;
    double dt, xth, input_scaling, failing_reward;
    const int32_t* fail_step;
    const int32_t* term_step;
    const double* obs;
    uint8_t* pending;
    double* t;
    int64_t* steps;
    double* episode_return;
    float* obs32;
    float* reward;
    uint8_t* done;
    uint8_t* valid;
    double* fin;
    int64_t fin_cap;
    int64_t* fin_n;
};
int launch_env_tail(const EnvTailArgs& a, void* stream);

// reference noise stream (qcart_noise.hip): per-env MT19937 state [B][kMtWords] uint32 (624 words,
// the read index, one pad word)
constexpr int kMtWords = 626;
int launch_mt_seed(const uint32_t* seeds, const uint8_t* mask, int64_t B, uint32_t* st, void* stream);
int launch_mt_normals(uint32_t* st, int64_t B, int32_t n_steps, const int32_t* env_steps, double* noise,
                      void* stream, const double* pre = nullptr, const uint8_t* has_pre = nullptr);
int launch_fill_u64(uint64_t* p, int64_t n, uint64_t v, void* stream);

// host-side launchers (qcart_kernels.hip)
// (the kernel precision is a.precision)
int launch_step(int family, int R, const KArgs& a, void* stream);
int launch_obs(int family, int R, const KArgs& a, void* stream);   // moments into obs_out
int launch_aux(int family, int R, int what, const KArgs& a, double xth, void* out, void* stream);
int launch_reset(int family, int R, const KArgs& a, int kind, const uint8_t* mask, double a0,
                 double a1, double a2, const double* k_arr, const double* m_arr, const double* s_arr,
                 void* stream);
int launch_control(int family, int R, const KArgs& a, void* stream);   // qc_control (act_out / force_out)
bool have_kernel(int family, int R, int precision = 0);
int step_waves(int family, int R, int precision = 0);   // envs per step-kernel workgroup (<0: none)
int step_dual_img(int family, int R, int precision = 0);   // MODE 3 slot-image bytes (0: no two-slot blocks)
// envs grouped by force slot into order[cap] (gran-aligned groups, -1 padding); qcart_k_group.hip
// order_mixed (optional, [n_slots * gran] + 1 count word): slots with >= gran envs are laid out back to back
// and cut into gran-env workgroups; the ones that straddle two slots go to order_mixed (k_step DUAL), the rest
// to order, and their number to order_mixed[n_slots * gran]
int launch_group(const int32_t* actions, int32_t default_action, const int32_t* env_steps, int32_t n_steps, int64_t B,
                 int n_slots, int gran, int32_t* order, int32_t cap, int32_t* bad, int32_t* order_mixed, void* stream);

}  // namespace qcart
