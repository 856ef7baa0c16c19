// qcart_api.cpp — implementation of the C ABI declared in include/qcart.h.
//
// A handle is bound to one device and one HIP stream and owns the operator rows and the per-slot
// factor tables (21 discrete forces + registered custom forces). All compute runs in the HIP
// kernels of qcart_kernels.hip; there is no CPU fallback: a missing device or kernel is an error.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/qcart.h"
#include "qcart_kargs.hpp"
#include "qcart_tables.hpp"

using namespace qcart;

namespace {
constexpr int kMaxSlots = 64;
// qc_step calls of at most this many physics steps on at most this many envs read their tables from L2 (MODE 0)
constexpr int kShortCallSteps = 10;
constexpr int64_t kShortCallBatch = 4096;
constexpr int64_t kSpreadBatch = 1024;   // 4 envs per CU of MI355X's 256: one per SIMD
std::mutex g_err_mu;
std::string g_create_err;

void set_create_err(const std::string& s) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    g_create_err = s;
}
}  // namespace

namespace qcart {
void set_global_error(const std::string& m) { set_create_err(m); }
// the step server's resident kernel (qcart_server.cpp): declared here, defined after qc_handle
bool resident_available(const qc_handle* h);
int resident_launch(qc_handle* h, void* psi, void* slots, double* obs, const uint32_t* ctl, double beat_s,
                    double lease_s, uint32_t gen, void* stream);
}  // namespace qcart

struct qc_handle {
    qc_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    int R = 0;
    int wpb = 4;   // envs per step workgroup (step_waves)
    bool mirror = false;
    OpHost op;
    std::vector<ActHost> acts;
    std::string err;
    // noise: per-env Philox counters [B] (always allocated); MT19937 mode: per-env states + the
    // call's normals buffer
    uint64_t* d_ctr = nullptr;
    int noise_mode = QC_NOISE_PHILOX;
    uint32_t* d_mt = nullptr;
    double* d_noise = nullptr;
    size_t noise_cap = 0;
    // step-kernel timing (qc_set_timing): a HIP event pair around every k_step launch on the handle's stream
    bool timing = false;
    std::vector<hipEvent_t> ev;   // [2 * n] start / stop
    size_t ev_used = 0;
    // device buffers
    double *d_xu = nullptr, *d_xg = nullptr, *d_hu = nullptr;
    double *d_tab = nullptr, *d_force = nullptr;
    uint32_t slot_bytes = 0;
    int32_t* d_order = nullptr;   // envs grouped by force slot (step kernel with per-block LDS tables)
    size_t order_cap = 0;
    // two-slot remainder workgroups (k_group order_mixed, k_step DUAL): bytes of one slot's MODE 3 LDS
    // image, 0 = not used by this handle (QCART_DUAL=0 turns them off, for A/B)
    uint32_t dual_img = 0;
    int32_t* d_order_mixed = nullptr;   // [kMaxSlots][wpb]
    int32_t *d_kf = nullptr, *d_kb = nullptr;
    // raised by k_group / the MODE 0 step kernel on an out-of-range action (qc_take_errors): one word of pinned,
    // coherent host memory mapped into the device, so that reading it after a stream synchronisation is a host
    // load (a 4-byte device-to-host copy cost a copy kernel and a second synchronisation per step-server tick)
    int32_t* d_bad = nullptr;
    volatile int32_t* h_bad = nullptr;
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int fail(qc_handle* h, int code, const std::string& msg) {
    if (h) h->err = msg;
    return code;
}

int hip_check(qc_handle* h, hipError_t e, const char* what) {
    if (e == hipSuccess) return QC_OK;
    return fail(h, QC_EHIP, std::string(what) + ": " + hipGetErrorString(e));
}

// the rows-per-lane instantiations compiled in qcart_kernels.hip
int pick_R(int family, int N, int precision) {
    static const int r_fock_ho[] = {1, 2, 4, 8};
    static const int r_fock_iho[] = {1, 2, 3, 4, 8, 16};
    static const int r_grid[] = {1, 2, 3, 5, 9, 17};
    static const int r_f32_ho[] = {4, 8, 32}, r_f32_iho[] = {8, 16, 32};
    const int need = (N + kWave - 1) / kWave;
    const int* list = family == QC_HO ? r_fock_ho : (family == QC_IHO ? r_fock_iho : r_grid);
    int n = family == QC_HO ? 4 : 6;
    if (precision == QC_FP32) {
        list = family == QC_HO ? r_f32_ho : r_f32_iho;
        n = 3;
    }
    for (int i = 0; i < n; i++)
        if (list[i] >= need) return list[i];
    return -1;
}

void free_dev(qc_handle* h) {
    double** dp[] = {&h->d_xu, &h->d_xg, &h->d_hu, &h->d_tab,
                     &h->d_force};
    for (auto p : dp)
        if (*p) { (void)hipFree(*p); *p = nullptr; }
    if (h->h_bad) { (void)hipHostFree((void*)h->h_bad); h->h_bad = nullptr; h->d_bad = nullptr; }
    if (h->d_kf) { (void)hipFree(h->d_kf); h->d_kf = nullptr; }
    if (h->d_order) { (void)hipFree(h->d_order); h->d_order = nullptr; h->order_cap = 0; }
    if (h->d_order_mixed) { (void)hipFree(h->d_order_mixed); h->d_order_mixed = nullptr; }
    if (h->d_kb) { (void)hipFree(h->d_kb); h->d_kb = nullptr; }
    if (h->d_ctr) { (void)hipFree(h->d_ctr); h->d_ctr = nullptr; }
    if (h->d_mt) { (void)hipFree(h->d_mt); h->d_mt = nullptr; }
    if (h->d_noise) { (void)hipFree(h->d_noise); h->d_noise = nullptr; h->noise_cap = 0; }
    for (auto e : h->ev) (void)hipEventDestroy(e);
    h->ev.clear();
    h->ev_used = 0;
}

template <typename T>
int upload(qc_handle* h, T** dst, const T* src, size_t n) {
    if (!*dst) {
        hipError_t e = hipMalloc((void**)dst, n * sizeof(T));
        if (e != hipSuccess) return fail(h, QC_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    return hip_check(h, hipMemcpy(*dst, src, n * sizeof(T), hipMemcpyHostToDevice), "hipMemcpy");
}

// (re)build every slot's factor block on the host (SlotLayout, lane-interleaved) and upload them
// (slot capacity kMaxSlots)
int upload_tables(qc_handle* h) {
    const int Np = h->op.Npad, kl = h->op.kl, R = h->op.Rs, LN = h->op.lanes;
    const bool f32 = h->p.precision == QC_FP32;   // fp32 blocks: the fp64 factors rounded once
    const bool sym = h->op.sym;   // L D L^T, no uc band (SlotLayout, slot_sym)
    const SlotLayout L = slot_layout(kl, R, h->op.family == QC_IHO, f32 ? 8u : 16u, sym, LN);
    h->slot_bytes = L.bytes;
    std::vector<uint8_t> tab((size_t)kMaxSlots * L.bytes, 0);
    std::vector<double> force(kMaxSlots, 0.0);
    std::vector<int32_t> kf(kMaxSlots, 0), kb(kMaxSlots, 0);
    auto ilv = [&](int b, int r) { return ((size_t)b * R + (r % R)) * LN + r / R; };   // row-band element
    auto putr = [&](uint8_t* blk, uint32_t off, size_t elem, double v) {
        if (f32) ((float*)(blk + off))[elem] = (float)v;
        else ((double*)(blk + off))[elem] = v;
    };
    auto put = [&](uint8_t* blk, uint32_t off, size_t elem, cplx v) {
        putr(blk, off, 2 * elem, v.real());
        putr(blk, off, 2 * elem + 1, v.imag());
    };
    for (size_t s = 0; s < h->acts.size(); s++) {
        const ActHost& a = h->acts[s];
        uint8_t* blk = tab.data() + s * L.bytes;
        for (int b = 0; b < kl; b++)
            for (int r = 0; r < Np; r++) {
                put(blk, L.lc, ilv(b, r), a.lc[(size_t)b * Np + r]);
                if (!sym) put(blk, L.uc, ilv(b, r), a.uc[(size_t)b * Np + r]);
            }
        for (int r = 0; r < Np; r++) put(blk, L.di, ilv(0, r), a.dinv[r]);
        if (h->op.family == QC_IHO)
            for (int b = 0; b < kMirrorBands; b++)
                for (int r = 0; r < Np; r++) putr(blk, L.m2, ilv(b, r), a.m2[(size_t)b * Np + r]);
        const size_t kk = (size_t)kl * kl;
        for (int v = 0; v < kTabLevels; v++)
            for (int l = 0; l < LN; l++)
                for (size_t e = 0; e < kk; e++) {
                    const size_t src = ((size_t)v * LN + l) * kk + e, dst = ((size_t)v * kk + e) * LN + l;
                    put(blk, L.tf, dst, a.tf[src]);
                    put(blk, L.tb, dst, a.tb[src]);
                }
        force[s] = a.force;
        kf[s] = a.kf;
        kb[s] = a.kb;
    }
    int rc;
    if ((rc = upload(h, &h->d_tab, (const double*)tab.data(), tab.size() / 8))) return rc;
    if ((rc = upload(h, &h->d_force, force.data(), force.size()))) return rc;
    if ((rc = upload(h, &h->d_kf, kf.data(), kf.size()))) return rc;
    if ((rc = upload(h, &h->d_kb, kb.data(), kb.size()))) return rc;
    return QC_OK;
}

int build_all_actions(qc_handle* h) {
    std::vector<double> forces;
    for (auto& a : h->acts) forces.push_back(a.force);
    if (forces.empty())
        for (int a = 0; a < h->p.n_actions; a++)
            forces.push_back((double)(a - h->p.n_actions / 2) * (h->p.f_max / (double)(h->p.n_actions / 2)));
    h->acts.assign(forces.size(), ActHost());
    for (size_t i = 0; i < forces.size(); i++) {
        int rc = build_action(h->op, h->p.dt, forces[i], h->mirror, h->acts[i], h->err);
        if (rc) return rc;
    }
    return QC_OK;
}

KArgs base_args(const qc_handle* h) {
    KArgs a;
    std::memset(&a, 0, sizeof(a));
    const qc_params& p = h->p;
    const OpHost& op = h->op;
    a.B = p.batch;
    a.env_offset = p.env_offset;
    a.seed = p.seed;
    a.ctr = h->d_ctr;
    a.N = op.N;
    a.Npad = op.Npad;
    a.n_slots = (int32_t)h->acts.size();
    a.mirror = h->mirror ? 1 : 0;
    a.bnd_len = op.fock ? kFockBnd : kGridBnd;
    a.win_lo = a.win_hi = 0;
    if (!op.fock && p.xth > 0) {
        const int c = op.N / 2, w = (int)std::nearbyint(p.xth / op.h);   // IQO/main_parallel.py:78-81
        a.win_lo = c - w;
        a.win_hi = c + w;
    }
    a.moment_order = op.fock ? 0 : p.moment_order;
    {
        // step-kernel table placement: the slot block's lc/uc/di/m2 (and the kept scan composites) in
        // the workgroup's LDS when they fit the 160 KiB of a CU (QCART_TAB_MODE overrides, for A/B)
        int lf = 0, lb = 0;
        for (auto& s : h->acts) {
            lf = std::max(lf, s.kf);
            lb = std::max(lb, s.kb);
        }
        const bool f32 = p.precision == QC_FP32;
        const uint32_t es = f32 ? 8u : 16u;   // bytes per complex table element
        const SlotLayout L = slot_layout(op.kl, op.Rs, op.family == QC_IHO, es, op.sym, op.lanes);
        // MODE 2 image: levels 0..NL-1 + the row prefix per direction at fixed places (needs kf, kb <= NL)
        const int NL = mode2_levels(op.kl);
        const size_t t1 = L.tf, t2 = L.tf + (size_t)(2 * NL + 2) * op.kl * op.kl * op.lanes * es;
        // fp64 Fock families append the slot's H_F force coefficients (R+1 doubles per lane), the grid its
        // row constants (H_F's folded diagonal and x_r: 2R doubles per lane, RowLds)
        // (IHO: and X^2's diagonal, R doubles per lane)
        const size_t fx = op.fock ? (f32 ? 0 : (size_t)(op.R + 1 + (op.family == QC_IHO ? op.R : 0)) * kWave * 8)
                                  : (grid_rows_in_lds(op.R) ? (size_t)2 * op.R * kWave * 8 : 0);
        // MODE 4 (grid R >= 17): the forward levels + prefix only, beside the row constants
        const size_t t4 = L.tf + (size_t)(NL + 1) * op.kl * op.kl * op.lanes * es;
        // fp64: each wave's noise buffer (kNzLds) after the image(s)
        const size_t nzb = f32 ? 0 : (size_t)h->wpb * kNzLds, cap = 160 * 1024 - nzb;
        const bool m4 = !op.fock && !f32 && grid_rows_in_lds(op.R) && lf <= NL && t4 + fx <= cap;
        int mode = (t2 + fx <= cap && lf <= NL && lb <= NL) ? 2 : m4 ? 4 : (t1 + fx <= cap ? 1 : 0);
        if (const char* e = std::getenv("QCART_TAB_MODE")) {   // a cap: 0 < 1 < 4 < 2 in LDS use
            const int c = std::atoi(e);
            if (mode != 4 || c < 2) mode = std::min(mode, c);
        }
        a.tab_mode = mode;
        a.lds_fx = (uint32_t)(mode == 2 ? t2 : mode == 4 ? t4 : t1);
        a.lds_bytes = mode ? (uint32_t)(a.lds_fx + fx) : 0u;
        // two-slot blocks (MODE 3) share the launch: the dynamic LDS covers two slot images
        if (h->dual_img && mode >= 1) {
            a.lds_img = h->dual_img;
            a.lds_bytes = std::max(a.lds_bytes, 2u * h->dual_img);
        }
        a.lds_nz = 0;
        if (mode >= 1 && nzb) {
            a.lds_nz = (a.lds_bytes + 15u) & ~15u;
            a.lds_bytes = a.lds_nz + (uint32_t)nzb;
        }
    }
    a.precision = p.precision;
    a.order = nullptr;
    a.n_blocks = (uint32_t)((p.batch + h->wpb - 1) / h->wpb);
    a.n_obs = qc_n_obs(h);
    a.dt = p.dt;
    a.sqrt_dt = std::sqrt(p.dt);
    a.gamma = p.gamma;
    a.g4 = p.gamma / 4.;
    a.beta = std::sqrt(p.gamma / 2.);
    a.inv_sqrt2g = 1.0 / std::sqrt(2. * p.gamma);
    a.w = op.w;
    a.inv_sqrt_w = 1.0 / std::sqrt(op.w);
    a.c = op.c;
    a.h = op.fock ? 1.0 : op.h;
    const double dt = p.dt;
    a.x2h = op.family == QC_IHO ? -1.0 / op.c : 0.0;
    a.a2 = dt * dt * dt / 12.;
    a.a3 = dt * dt * dt * dt / 24.;
    a.a4 = dt * dt * dt * dt * dt / 80.;
    a.a5 = dt * dt * dt * dt * dt * dt / 360.;
    // host-folded step constants (KArgs): the same expressions the kernel evaluated
    a.inv_sdt = 1.0 / a.sqrt_dt;
    a.inv_dt = 1.0 / dt;
    a.k_hisdt = 0.5 * a.inv_sdt;
    a.k_qisdt = 0.25 * a.inv_sdt;
    a.k_hidt = 0.5 * a.inv_dt;
    a.k_qidt = 0.25 * a.inv_dt;
    a.k_qdt = 0.25 * dt;
    a.k_qsdt = 0.25 * a.sqrt_dt;
    a.k_dz = a.sqrt_dt * dt * 0.5;
    a.k_sb = a.sqrt_dt * a.beta;
    a.b2 = a.a2 / a.a5;
    a.b3 = a.a3 / a.a5;
    a.b4 = a.a4 / a.a5;
    // check_boundary_error thresholds: IHO 2e-3 (IHO:423), HO 1e-3 (HO:404), grid 5e-3 (QO:561)
    a.fail_thr = p.family == QC_HO ? 1e-3 : (p.family == QC_IHO ? 2e-3 : 5e-3);
    for (int d = 0; d < 5; d++) a.hoff[d] = op.hoff[d];
    a.xu = h->d_xu;
    a.xg = h->d_xg;
    a.hu = h->d_hu;
    a.tab = h->d_tab;
    a.slot_bytes = h->slot_bytes;
    a.kf = h->d_kf;
    a.kb = h->d_kb;
    a.force = h->d_force;
    a.bad = h->d_bad;
    return a;
}

int validate_params(const qc_params* p, std::string& err) {
    if (!p) { err = "null params"; return QC_EINVAL; }
    if (p->family < QC_HO || p->family > QC_IQO) { err = "family must be 0..3"; return QC_EINVAL; }
    if (!(p->dt > 0) || !std::isfinite(p->dt)) { err = "dt must be > 0"; return QC_EINVAL; }
    if (!(p->gamma >= 0) || !std::isfinite(p->gamma)) { err = "gamma must be >= 0"; return QC_EINVAL; }
    if (p->batch < 0) { err = "batch must be >= 0"; return QC_EINVAL; }
    if (p->n_actions < 1 || p->n_actions > kMaxSlots || (p->n_actions % 2) == 0) {
        err = "n_actions must be odd and <= 64";
        return QC_EINVAL;
    }
    if (p->family >= QC_QO && (p->moment_order < 1 || p->moment_order > kMaxMomentOrderHi)) {
        // the observation kernel's instantiations: up to 3 observables per lane of the env's wave
        err = "moment_order must be in 1..16 (the (2+m+1)*m/2 observables, at most 3 per lane of a 64-lane wave)";
        return QC_EINVAL;
    }
    if (p->a_mode != QC_A_REFERENCE && p->a_mode != QC_A_EXACT) { err = "bad a_mode"; return QC_EINVAL; }
    if (p->precision != QC_FP64 && p->precision != QC_FP32) { err = "precision must be 0 (fp64) or 1 (fp32)"; return QC_EINVAL; }
    if (p->precision == QC_FP32 && p->family >= QC_QO) { err = "fp32 is built for the Fock families only"; return QC_EINVAL; }
    return QC_OK;
}

}  // namespace

namespace qcart {
// fp64 Fock modules with a resident kernel instantiated for their rows per lane, in MT19937 mode
bool resident_available(const qc_handle* h) {
    return h && h->p.precision == QC_FP64 && h->noise_mode == QC_NOISE_MT19937 && h->d_mt && h->p.batch > 0 &&
           h->p.batch <= kSpreadBatch && have_resident(h->p.family, h->op.Rs);
}
// k_resident over the handle's B envs (env e = slot e): the KArgs of qc_step's short one-step call (MODE 0, one env
// per block, no grouping) — the same step body and constants, so both paths step an env bitwise alike
int resident_launch(qc_handle* h, void* psi, void* slots, double* obs, const uint32_t* ctl, double beat_s,
                    double lease_s, uint32_t gen, void* stream) {
    if (!resident_available(h)) return fail(h, QC_EINVAL, "no resident kernel for this module");
    KArgs a = base_args(h);
    a.psi = psi;
    a.n_steps = 1;
    // MODE 2 (the request's slot image kept in LDS between requests) for the Fock modules where base_args places the
    // tables so and every block gets a CU of its own (<= 256 slots; one wave's noise buffer); else MODE 0 (tables from
    // L2; the grid's MODE 2 body contracts apart from its MODE 0 ticks)
    // (QCART_RESIDENT_MODE=0 forces the latter, for A/B)
    const char* rm = std::getenv("QCART_RESIDENT_MODE");   // (read per launch: a launch lives a 20 ms lease)
    const bool lds_ok = !(rm && std::atoi(rm) == 0);
    if (lds_ok && a.tab_mode == 2 && h->p.batch <= 256 && h->op.fock) {
        // one slot image per block (not the two-slot layout's), then one wave's noise buffer (base_args' layout)
        const OpHost& op = h->op;
        const uint32_t fx = op.fock ? (uint32_t)(op.R + 1 + (op.family == QC_IHO ? op.R : 0)) * kWave * 8u : 0u;
        a.lds_img = 0;
        a.lds_nz = (a.lds_fx + fx + 15u) & ~15u;
        a.lds_bytes = a.lds_nz + kNzLds;
    } else {
        a.tab_mode = 0;
        a.lds_bytes = 0;
        a.lds_img = 0;
        a.lds_nz = 0;
    }
    // the block's copy of the row it returned ([Rs][64] complex fp64), after the image and the noise buffer
    const uint32_t lds_row = a.lds_bytes;
    a.lds_bytes += (uint32_t)h->op.Rs * kWave * 16u;
    a.spread = 1;
    a.n_blocks = (uint32_t)h->p.batch;
    a.bad = nullptr;   // the client sends only actions of the grid (anything else bounces to the tick path)
    ResArgs r{};
    r.slots = slots;
    r.ctl = ctl;
    r.mt = h->d_mt;
    r.beat_ticks = (uint64_t)(beat_s * 1e8);   // s_memrealtime: 100 MHz
    r.lease_ticks = (uint64_t)(lease_s * 1e8);
    r.gen = gen & 63u;
    r.lds_row = lds_row;
    r.obs = obs;
    DeviceGuard g(h->device);
    const int rc = launch_resident(h->p.family, h->op.Rs, a, r, stream);
    return rc ? fail(h, QC_EHIP, "resident kernel launch failed") : QC_OK;
}
}  // namespace qcart

extern "C" {

int qc_abi_version(void) { return QC_ABI_VERSION; }

const char* qc_last_error(const qc_handle* h) {
    if (h) return h->err.c_str();
    std::lock_guard<std::mutex> lk(g_err_mu);
    return g_create_err.c_str();
}

int qc_create(const qc_params* p, int device, qc_handle** out) {
    if (!out) { set_create_err("null out"); return QC_EINVAL; }
    *out = nullptr;
    std::string err;
    int rc = validate_params(p, err);
    if (rc) { set_create_err(err); return rc; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        set_create_err("no HIP device available (libqcart has no CPU fallback)");
        return QC_EHIP;
    }
    if (device < 0 || device >= ndev) { set_create_err("device index out of range"); return QC_EINVAL; }
    qc_handle* h = new qc_handle();
    h->p = *p;
    h->device = device;
    h->mirror = (p->family == QC_IHO && p->a_mode == QC_A_REFERENCE);
    // probe N first to pick the rows-per-lane instantiation
    OpHost probe;
    rc = build_ops(p->family, p->n_max, p->omega, p->x_max, p->grid_size, p->lambda_, p->mass, 1 << 12, probe, err);
    if (rc) { set_create_err(err); delete h; return rc; }
    h->R = pick_R(p->family, probe.N, p->precision);
    if (h->R < 0 || !have_kernel(p->family, h->R, p->precision)) {
        set_create_err("no kernel instantiated for N = " + std::to_string(probe.N));
        delete h;
        return QC_ENOTBUILT;
    }
    h->wpb = step_waves(p->family, h->R, p->precision);
    if (h->wpb <= 0) {
        set_create_err("no step kernel for N = " + std::to_string(probe.N));
        delete h;
        return QC_ENOTBUILT;
    }
    rc = build_ops(p->family, p->n_max, p->omega, p->x_max, p->grid_size, p->lambda_, p->mass, h->R, h->op, err);
    if (rc) { set_create_err(err); delete h; return rc; }
    const uint32_t es = p->precision == QC_FP32 ? 8u : 16u;
    h->op.sym = slot_sym(h->op.fock, es, h->op.lanes);
    rc = build_all_actions(h);
    if (rc) { set_create_err(h->err); delete h; return rc; }
    DeviceGuard g(device);
    const int Np = h->op.Npad;
    if ((rc = upload(h, &h->d_xu, h->op.xu.data(), Np)) || (rc = upload(h, &h->d_xg, h->op.xg.data(), Np)) ||
        (rc = upload(h, &h->d_hu, h->op.hu.data(), Np)) || (rc = upload_tables(h))) {
        set_create_err(h->err);
        free_dev(h);
        delete h;
        return rc;
    }
    {
        const char* de = std::getenv("QCART_DUAL");
        if (!(de && std::atoi(de) == 0)) h->dual_img = (uint32_t)std::max(0, step_dual_img(p->family, h->R, p->precision));
    }
    {
        std::vector<uint64_t> zero((size_t)std::max<int64_t>(p->batch, 1), 0);
        rc = upload(h, &h->d_ctr, zero.data(), zero.size());
        void* hb = nullptr;
        if (!rc) rc = hip_check(h, hipHostMalloc(&hb, sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent),
                                "hipHostMalloc");
        if (!rc) {
            h->h_bad = (volatile int32_t*)hb;
            *h->h_bad = 0;
            void* dp = nullptr;
            rc = hip_check(h, hipHostGetDevicePointer(&dp, hb, 0), "hipHostGetDevicePointer");
            h->d_bad = (int32_t*)dp;
        }
    }
    if (rc) {
        set_create_err(h->err);
        free_dev(h);
        delete h;
        return rc;
    }
    *out = h;
    return QC_OK;
}

void qc_destroy(qc_handle* h) {
    if (!h) return;
    {
        DeviceGuard g(h->device);
        (void)hipDeviceSynchronize();
        free_dev(h);
    }
    delete h;
}

int qc_get_params(const qc_handle* h, qc_params* out) {
    if (!h || !out) return QC_EINVAL;
    *out = h->p;
    return QC_OK;
}

int qc_dim(const qc_handle* h) { return h ? h->op.N : QC_EINVAL; }

int qc_n_obs(const qc_handle* h) {
    if (!h) return QC_EINVAL;
    if (h->op.fock) return 5;
    const int m = h->p.moment_order;
    return (2 + m + 1) * m / 2;   // QO/simulation_quart.cpp:381
}

int qc_set_stream(qc_handle* h, void* stream) {
    if (!h) return QC_EINVAL;
    h->stream = (hipStream_t)stream;
    return QC_OK;
}

int qc_sync(qc_handle* h) {
    if (!h) return QC_EINVAL;
    DeviceGuard g(h->device);
    return hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize");
}

int qc_set_seed(qc_handle* h, uint64_t seed) {
    if (!h) return QC_EINVAL;
    h->p.seed = seed;
    h->noise_mode = QC_NOISE_PHILOX;
    return qc_set_step_counter(h, 0);
}
int qc_set_step_counter(qc_handle* h, uint64_t step) {
    if (!h) return QC_EINVAL;
    DeviceGuard g(h->device);
    if (launch_fill_u64(h->d_ctr, h->p.batch, step, h->stream)) return fail(h, QC_EHIP, "fill kernel launch failed");
    return QC_OK;
}
uint64_t qc_get_step_counter(const qc_handle* h) {
    if (!h || h->p.batch <= 0) return 0;
    DeviceGuard g(h->device);
    uint64_t v = 0;
    if (hipStreamSynchronize(h->stream) != hipSuccess) return 0;
    if (hipMemcpy(&v, h->d_ctr, sizeof(v), hipMemcpyDeviceToHost) != hipSuccess) return 0;
    return v;
}
int qc_env_counters(qc_handle* h, uint64_t* out, const uint64_t* in) {
    if (!h) return QC_EINVAL;
    if (h->p.batch == 0) return QC_OK;
    DeviceGuard g(h->device);
    const size_t bytes = (size_t)h->p.batch * sizeof(uint64_t);
    if (out && hip_check(h, hipMemcpyAsync(out, h->d_ctr, bytes, hipMemcpyDeviceToDevice, h->stream), "hipMemcpyAsync"))
        return QC_EHIP;
    if (in && hip_check(h, hipMemcpyAsync(h->d_ctr, in, bytes, hipMemcpyDeviceToDevice, h->stream), "hipMemcpyAsync"))
        return QC_EHIP;
    return QC_OK;
}
int qc_set_seed_mt19937_envs(qc_handle* h, const uint32_t* seeds, const uint8_t* mask) {
    if (!h) return QC_EINVAL;
    if (h->p.batch > 0 && !seeds) return fail(h, QC_EINVAL, "seeds is null");
    if (mask && h->noise_mode != QC_NOISE_MT19937)
        return fail(h, QC_EINVAL, "a masked reseed needs every env's MT19937 stream (qc_set_seed_mt19937 first)");
    DeviceGuard g(h->device);
    if (h->p.batch > 0) {
        if (!h->d_mt) {
            hipError_t e = hipMalloc((void**)&h->d_mt, (size_t)h->p.batch * kMtWords * sizeof(uint32_t));
            if (e != hipSuccess) { h->d_mt = nullptr; return fail(h, QC_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e)); }
        }
        if (launch_mt_seed(seeds, mask, h->p.batch, h->d_mt, h->stream))
            return fail(h, QC_EHIP, "MT19937 seed kernel launch failed");
    }
    h->noise_mode = QC_NOISE_MT19937;
    return QC_OK;
}
int qc_set_seed_mt19937(qc_handle* h, const uint32_t* seeds) { return qc_set_seed_mt19937_envs(h, seeds, nullptr); }
int qc_mt19937_normals(qc_handle* h, int32_t n_steps, const int32_t* env_steps, const double* pre,
                       const uint8_t* has_pre, double* noise) {
    if (!h) return QC_EINVAL;
    if (n_steps < 0) return fail(h, QC_EINVAL, "n_steps must be >= 0");
    if (h->noise_mode != QC_NOISE_MT19937 || !h->d_mt) return fail(h, QC_EINVAL, "no MT19937 state (qc_set_seed_mt19937 first)");
    if (!noise && h->p.batch > 0 && n_steps > 0) return fail(h, QC_EINVAL, "noise is null");
    if (!pre != !has_pre) return fail(h, QC_EINVAL, "pre and has_pre go together");
    DeviceGuard g(h->device);
    if (launch_mt_normals(h->d_mt, h->p.batch, n_steps, env_steps, noise, h->stream, pre, has_pre))
        return fail(h, QC_EHIP, "MT19937 normals kernel launch failed");
    return QC_OK;
}
int qc_noise_mode(const qc_handle* h) { return h ? h->noise_mode : QC_EINVAL; }
int qc_mt19937_state(qc_handle* h, uint32_t* out, const uint32_t* in) {
    if (!h) return QC_EINVAL;
    if (!h->d_mt) return fail(h, QC_EINVAL, "no MT19937 state (qc_set_seed_mt19937 first)");
    DeviceGuard g(h->device);
    const size_t bytes = (size_t)h->p.batch * kMtWords * sizeof(uint32_t);
    if (out && hip_check(h, hipMemcpyAsync(out, h->d_mt, bytes, hipMemcpyDeviceToDevice, h->stream), "hipMemcpyAsync"))
        return QC_EHIP;
    if (in && hip_check(h, hipMemcpyAsync(h->d_mt, in, bytes, hipMemcpyDeviceToDevice, h->stream), "hipMemcpyAsync"))
        return QC_EHIP;
    return QC_OK;
}
int qc_mt19937_words(void) { return kMtWords; }

int qc_set_dynamics(qc_handle* h, double dt, double gamma) {
    if (!h) return QC_EINVAL;
    if (!(dt > 0) || !(gamma >= 0)) return fail(h, QC_EINVAL, "dt must be > 0 and gamma >= 0");
    const bool change_t = dt != h->p.dt;
    h->p.gamma = gamma;
    if (!change_t) return QC_OK;
    const double old = h->p.dt;
    h->p.dt = dt;
    int rc = build_all_actions(h);
    if (rc) {
        h->p.dt = old;
        build_all_actions(h);
        return rc;
    }
    DeviceGuard g(h->device);
    (void)hipStreamSynchronize(h->stream);
    return upload_tables(h);
}

int qc_add_force(qc_handle* h, double force) {
    if (!h) return QC_EINVAL;
    for (size_t s = 0; s < h->acts.size(); s++)
        if (h->acts[s].force == force) return (int)s;
    if ((int)h->acts.size() >= kMaxSlots) return fail(h, QC_ENOMEM, "no free force slot");
    ActHost a;
    int rc = build_action(h->op, h->p.dt, force, h->mirror, a, h->err);
    if (rc) return rc;
    h->acts.push_back(a);
    DeviceGuard g(h->device);
    (void)hipStreamSynchronize(h->stream);
    rc = upload_tables(h);
    if (rc) { h->acts.pop_back(); return rc; }
    return (int)h->acts.size() - 1;
}

int qc_step(qc_handle* h, void* psi, const int32_t* actions, int32_t default_action, int32_t n_steps,
            const int32_t* env_steps, const double* noise, double* q_out, double* xmean_out, int32_t* fail_step, int32_t* term_step,
            double* obs_out) {
    if (!h) return QC_EINVAL;
    if (!psi && h->p.batch > 0) return fail(h, QC_EINVAL, "psi is null");
    if (n_steps < 0) return fail(h, QC_EINVAL, "n_steps must be >= 0");
    if (!actions && (default_action < 0 || default_action >= (int)h->acts.size()))
        return fail(h, QC_EINVAL, "default_action out of range");
    if (term_step && !(h->p.xth > 0 && !h->op.fock))
        return fail(h, QC_EINVAL, "term_step needs a grid family and params.xth > 0");
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    a.actions = actions;
    a.env_steps = env_steps;
    a.default_action = default_action;
    a.n_steps = n_steps;
    a.q_out = q_out;
    a.xm_out = xmean_out;
    a.fail_step = fail_step;
    a.term_step = term_step;
    a.obs_out = obs_out;
    // short calls on small batches (the drop-in's step / simulate_10_steps, the step server's ticks): the factor
    // tables are read from the slot blocks in L2 by each wave (MODE 0) — no per-workgroup LDS image of the slot
    // (120 KiB at IHO N = 512) for one or ten steps, and no slot-grouping launch (each wave has its own slot).
    // QCART_SHORT_MODE0=0 turns it off (A/B)
    {
        static const bool short_mode0 = !(std::getenv("QCART_SHORT_MODE0") && std::atoi(std::getenv("QCART_SHORT_MODE0")) == 0);
        if (short_mode0 && n_steps <= kShortCallSteps && h->p.batch <= kShortCallBatch && a.tab_mode != 0) {
            a.tab_mode = 0;
            a.lds_bytes = 0;
            a.lds_img = 0;
            a.lds_nz = 0;
        }
        // a short MODE 0 call on up to 4 envs per CU: one env per block (QCART_SPREAD=0 turns it off, A/B)
        static const bool spread = !(std::getenv("QCART_SPREAD") && std::atoi(std::getenv("QCART_SPREAD")) == 0);
        if (spread && a.tab_mode == 0 && n_steps <= kShortCallSteps && h->p.batch <= kSpreadBatch && h->wpb > 1) {
            a.spread = 1;
            a.n_blocks = (uint32_t)h->p.batch;
        }
    }
    // grid moment orders above the step kernel's fused epilogue: the observation kernel runs after the step
    const bool obs_after = obs_out && !h->op.fock && h->p.moment_order > kStepMaxMomentOrder;
    if (obs_after) a.obs_out = nullptr;
    DeviceGuard g(h->device);
    if (h->p.batch == 0) return QC_OK;
    if (!noise && h->noise_mode == QC_NOISE_MT19937 && n_steps > 0) {
        // the reference's stream: each env's MT19937 draws its steps' normals into the injected-noise
        // buffer first (the state advances by exactly the words the env consumes)
        const size_t need = (size_t)n_steps * (size_t)h->p.batch * 2;
        if (h->noise_cap < need) {
            if (h->d_noise) (void)hipFree(h->d_noise);
            h->d_noise = nullptr;
            h->noise_cap = 0;
            hipError_t e = hipMalloc((void**)&h->d_noise, need * sizeof(double));
            if (e != hipSuccess) return fail(h, QC_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
            h->noise_cap = need;
        }
        if (launch_mt_normals(h->d_mt, h->p.batch, n_steps, env_steps, h->d_noise, h->stream))
            return fail(h, QC_EHIP, "MT19937 normals kernel launch failed");
        noise = h->d_noise;
    }
    a.noise = noise;
    if ((actions || env_steps) && a.tab_mode != 0) {
        // group envs by force slot, padded to whole workgroups: every workgroup then shares one slot's
        // tables (the per-block LDS image); envs without a step budget form a last group of their own
        // (a reset interval of a few finished envs then costs in proportion to them); order within a
        // group does not change any result
        const size_t W = (size_t)h->wpb;
        const size_t cap = (size_t)((h->p.batch + W - 1) / W) * W + W * (size_t)(kMaxSlots + 1);
        if (h->order_cap < cap) {
            if (h->d_order) (void)hipFree(h->d_order);
            h->d_order = nullptr;
            h->order_cap = 0;
            hipError_t e = hipMalloc((void**)&h->d_order, cap * sizeof(int32_t));
            if (e != hipSuccess) return fail(h, QC_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
            h->order_cap = cap;
        }
        // two-slot remainder workgroups when the step kernel has them (tables in LDS, fp64, one wave per env)
        const bool dual = a.lds_img > 0;
        if (dual && !h->d_order_mixed) {
            hipError_t e = hipMalloc((void**)&h->d_order_mixed, ((size_t)kMaxSlots * W + 1) * sizeof(int32_t));
            if (e != hipSuccess) return fail(h, QC_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
        }
        if (launch_group(actions, default_action, env_steps, n_steps, h->p.batch, (int)h->acts.size(), (int)W,
                         h->d_order, (int32_t)cap, h->d_bad, dual ? h->d_order_mixed : nullptr, h->stream))
            return fail(h, QC_EHIP, "group kernel launch failed");
        a.order = h->d_order;
        a.n_blocks = (uint32_t)(cap / W);
        a.order_mixed = dual ? h->d_order_mixed : nullptr;
        a.n_mixed = dual ? (uint32_t)h->acts.size() : 0u;
        a.n_mixed_used = dual ? h->d_order_mixed + h->acts.size() * W : nullptr;
    }
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (h->timing) {
        if (h->ev_used + 2 > h->ev.size()) {
            for (int i = 0; i < 2; ++i) {
                hipEvent_t e;
                if (hipEventCreate(&e) != hipSuccess) return fail(h, QC_EHIP, "hipEventCreate failed");
                h->ev.push_back(e);
            }
        }
        ev0 = h->ev[h->ev_used];
        ev1 = h->ev[h->ev_used + 1];
        h->ev_used += 2;
        (void)hipEventRecord(ev0, h->stream);
    }
    int rc = launch_step(h->p.family, h->op.Rs, a, h->stream);
    if (h->timing) (void)hipEventRecord(ev1, h->stream);
    if (rc) return fail(h, rc, rc == QC_ENOTBUILT ? "kernel not built" : "step kernel launch failed");
    if (obs_after) {
        KArgs o = base_args(h);
        o.psi = (double*)psi;
        o.obs_out = obs_out;
        rc = launch_obs(h->p.family, h->R, o, h->stream);
        if (rc) return fail(h, rc, "obs kernel launch failed");
    }
    return QC_OK;
}

int qc_set_timing(qc_handle* h, int on) {
    if (!h) return QC_EINVAL;
    h->timing = on != 0;
    h->ev_used = 0;
    return QC_OK;
}

int qc_step_kernel_time(qc_handle* h, double* total_ms, int64_t* launches) {
    if (!h) return QC_EINVAL;
    DeviceGuard g(h->device);
    if (hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize")) return QC_EHIP;
    double tot = 0.0;
    for (size_t i = 0; i + 1 < h->ev_used; i += 2) {
        float ms = 0.f;
        if (hip_check(h, hipEventElapsedTime(&ms, h->ev[i], h->ev[i + 1]), "hipEventElapsedTime")) return QC_EHIP;
        tot += ms;
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = (int64_t)(h->ev_used / 2);
    h->ev_used = 0;
    return QC_OK;
}

int qc_moments(qc_handle* h, const void* psi, double* out) {
    if (!h || (!psi && h->p.batch > 0) || (!out && h->p.batch > 0)) return QC_EINVAL;
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    a.obs_out = out;
    DeviceGuard g(h->device);
    int rc = launch_obs(h->p.family, h->R, a, h->stream);
    return rc ? fail(h, rc, "obs kernel launch failed") : QC_OK;
}

int qc_x_expectation(qc_handle* h, const void* psi, double* out) {
    if (!h || (!psi && h->p.batch > 0)) return QC_EINVAL;
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    DeviceGuard g(h->device);
    int rc = launch_aux(h->p.family, h->R, 0, a, 0.0, out, h->stream);
    return rc ? fail(h, rc, "aux kernel launch failed") : QC_OK;
}

int qc_outside_prob(qc_handle* h, const void* psi, double xth, double* out) {
    if (!h || (!psi && h->p.batch > 0)) return QC_EINVAL;
    if (h->op.fock) return fail(h, QC_EINVAL, "outside probability is defined on grid families");
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    DeviceGuard g(h->device);
    int rc = launch_aux(h->p.family, h->R, 1, a, xth, out, h->stream);
    return rc ? fail(h, rc, "aux kernel launch failed") : QC_OK;
}

int qc_boundary_fail(qc_handle* h, const void* psi, int32_t* out) {
    if (!h || (!psi && h->p.batch > 0)) return QC_EINVAL;
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    DeviceGuard g(h->device);
    int rc = launch_aux(h->p.family, h->R, 2, a, 0.0, out, h->stream);
    return rc ? fail(h, rc, "aux kernel launch failed") : QC_OK;
}

int qc_energy(qc_handle* h, const void* psi, double* out) {
    if (!h || (!psi && h->p.batch > 0)) return QC_EINVAL;
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    DeviceGuard g(h->device);
    int rc = launch_aux(h->p.family, h->R, 3, a, 0.0, out, h->stream);
    return rc ? fail(h, rc, "aux kernel launch failed") : QC_OK;
}

int qc_hamiltonian_dot_psi(qc_handle* h, void* psi) {
    if (!h || (!psi && h->p.batch > 0)) return QC_EINVAL;
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    DeviceGuard g(h->device);
    int rc = launch_aux(h->p.family, h->R, 5, a, 0.0, nullptr, h->stream);
    return rc ? fail(h, rc, "aux kernel launch failed") : QC_OK;
}

int qc_phonon_number(qc_handle* h, const void* psi, double* out) {
    if (!h || (!psi && h->p.batch > 0)) return QC_EINVAL;
    if (!h->op.fock) return fail(h, QC_EINVAL, "phonon number is defined on Fock families");
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    DeviceGuard g(h->device);
    int rc = launch_aux(h->p.family, h->R, 4, a, 0.0, out, h->stream);
    return rc ? fail(h, rc, "aux kernel launch failed") : QC_OK;
}

int qc_reset(qc_handle* h, void* psi, int32_t kind, const uint8_t* mask, double arg0, double arg1, double arg2,
             const double* k_arr, const double* mean_arr, const double* std_arr) {
    if (!h || (!psi && h->p.batch > 0)) return QC_EINVAL;
    if (kind < QC_RESET_GROUND || kind > QC_RESET_GAUSSIAN) return fail(h, QC_EINVAL, "bad reset kind");
    if (kind == QC_RESET_GAUSSIAN && h->op.fock) return fail(h, QC_EINVAL, "Gaussian packet needs a grid family");
    if (kind != QC_RESET_GAUSSIAN && !h->op.fock) return fail(h, QC_EINVAL, "Fock reset needs a Fock family");
    if (kind == QC_RESET_RANDOM && !(arg0 >= 1)) return fail(h, QC_EINVAL, "levels must be >= 1");
    if (kind == QC_RESET_GAUSSIAN && !std_arr && !(arg2 > 0)) return fail(h, QC_EINVAL, "std must be > 0");
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    DeviceGuard g(h->device);
    int rc = launch_reset(h->p.family, h->R, a, kind, mask, arg0, arg1, arg2, k_arr, mean_arr, std_arr, h->stream);
    return rc ? fail(h, rc, "reset kernel launch failed") : QC_OK;
}

int qc_control(qc_handle* h, const void* psi, int32_t strategy, double con_parameter, double control_time,
               double input_scaling, int32_t* actions, double* force_out) {
    if (!h || (!psi && h->p.batch > 0) || (!actions && h->p.batch > 0)) return QC_EINVAL;
    if (strategy < QC_CTL_LQG || strategy > QC_CTL_SEMICLASSICAL) return fail(h, QC_EINVAL, "bad control strategy");
    if (h->op.fock && strategy != QC_CTL_LQG)
        return fail(h, QC_EINVAL, "the Fock families define the LQG controller only");
    if (!(control_time > 0)) return fail(h, QC_EINVAL, "control_time must be > 0");
    // LinearQuadratic takes sqrt(k * mass), k = lambda * con_parameter (controllers.py:20): the
    // reference raises a math domain error when that is negative
    if (!h->op.fock && strategy == QC_CTL_LQG && h->p.lambda_ * con_parameter * h->p.mass < 0)
        return fail(h, QC_EINVAL, "LQG: lambda * con_parameter * mass < 0 (math domain error)");
    KArgs a = base_args(h);
    a.psi = (double*)psi;
    a.act_out = actions;
    a.force_out = force_out;
    a.ctl_strategy = strategy;
    a.ctl_param = con_parameter;
    a.ctl_time = control_time;
    a.ctl_scaling = input_scaling;
    a.ctl_half = h->p.n_actions / 2;
    // force_max = net.convert_to_force(2 * no_action_choice) = round(2h - h) * (F_max / h) (RL.py:107-109)
    a.ctl_fmax = (double)a.ctl_half * (h->p.f_max / a.ctl_half);
    a.ctl_lambda = h->p.lambda_;
    a.ctl_mass = h->p.mass;
    DeviceGuard g(h->device);
    int rc = launch_control(h->p.family, h->R, a, h->stream);
    return rc ? fail(h, rc, "control kernel launch failed") : QC_OK;
}

int qc_record_row_len(int32_t read_length, int32_t interval, int32_t coarse_grain) {
    if (read_length <= 0 || interval <= 0 || coarse_grain <= 0 || interval % coarse_grain) return QC_EINVAL;
    const int m = interval / coarse_grain;
    if (read_length % m) return QC_EINVAL;
    return read_length + m + read_length / m + 1 + 2;
}

int qc_record(qc_handle* h, int32_t read_length, int32_t coarse_grain, double input_scaling, const double* q,
              int32_t n_steps, const int32_t* actions, int32_t default_action, const uint8_t* mode, float* hist,
              float* forces, const float* reward, float* rows) {
    if (!h) return QC_EINVAL;
    const int row_len = qc_record_row_len(read_length, n_steps, coarse_grain);
    if (row_len < 0)
        return fail(h, QC_EINVAL, "need n_steps % coarse_grain == 0 and read_length % (n_steps / coarse_grain) == 0");
    if (h->p.batch > 0 && (!q || !hist || !forces)) return fail(h, QC_EINVAL, "q, hist and forces are required");
    if (!actions && (default_action < 0 || default_action >= (int)h->acts.size()))
        return fail(h, QC_EINVAL, "default_action out of range");
    RecArgs a{};
    a.q = q;
    a.actions = actions;
    a.default_action = default_action;
    a.slot_force = h->d_force;
    a.mode = mode;
    a.hist = hist;
    a.forces = forces;
    a.rows = rows;
    a.reward = reward;
    a.B = h->p.batch;
    a.n_slots = (int32_t)h->acts.size();
    a.bad = h->d_bad;
    a.L = read_length;
    a.cg = coarse_grain;
    a.m = n_steps / coarse_grain;
    a.K = read_length / a.m;
    a.row_len = row_len;
    a.scaling = input_scaling;
    a.vec4 = (read_length % 4 == 0 && a.m % 4 == 0 && ((uintptr_t)hist & 15) == 0) ? 1 : 0;
    if (sizeof(float) * (size_t)(2 * a.L + a.K + 1) > 160 * 1024) return fail(h, QC_EINVAL, "read_length too large");
    DeviceGuard g(h->device);
    int rc = launch_record(a, h->stream);
    return rc ? fail(h, rc, "record kernel launch failed") : QC_OK;
}

// the rows get_data_wavefunction keeps: HO state[:-10] (HO/main_parallel.py:132-134), IHO state[:-20]
// (IHO/main_parallel.py:133-135), grid state[10:-10] (QO/main_parallel.py:132-133, IQO:136-137)
static int wavefunction_rows(const qc_handle* h, int* lo) {
    *lo = h->op.fock ? 0 : 10;
    return h->op.N - (h->op.family == QC_HO ? 10 : 20);
}

int qc_wavefunction_len(const qc_handle* h) {
    if (!h) return QC_EINVAL;
    int lo;
    return 2 * wavefunction_rows(h, &lo);
}

int qc_wavefunction_obs(qc_handle* h, const void* psi, double input_scaling, float* out) {
    if (!h) return QC_EINVAL;
    if (h->p.batch > 0 && (!psi || !out)) return fail(h, QC_EINVAL, "psi and out are required");
    int lo;
    const int rows = wavefunction_rows(h, &lo);
    if (rows <= 0) return fail(h, QC_EINVAL, "the wavefunction input needs more rows than it drops");
    DeviceGuard g(h->device);
    int rc = launch_wavefunction(psi, h->p.precision, h->p.batch, h->op.N, lo, rows, input_scaling, out,
                                 h->stream);
    return rc ? fail(h, QC_EHIP, "wavefunction kernel launch failed") : QC_OK;
}

int qc_step_group_size(const qc_handle* h) { return h ? h->wpb : QC_EINVAL; }

int qc_group_layout(qc_handle* h, int32_t* order, int64_t order_len, int32_t* mixed, int64_t mixed_len) {
    if (!h) return QC_EINVAL;
    DeviceGuard g(h->device);
    if (hip_check(h, hipStreamSynchronize(h->stream), "hipStreamSynchronize")) return QC_EHIP;
    if (order && order_len > 0 && h->d_order) {
        const size_t n = std::min((size_t)order_len, h->order_cap);
        if (hip_check(h, hipMemcpy(order, h->d_order, n * sizeof(int32_t), hipMemcpyDeviceToHost), "hipMemcpy"))
            return QC_EHIP;
    }
    const int64_t mcap = h->d_order_mixed ? (int64_t)kMaxSlots * h->wpb : 0;
    if (mixed && mixed_len > 0 && mcap > 0) {
        const size_t n = (size_t)std::min(mixed_len, mcap);
        if (hip_check(h, hipMemcpy(mixed, h->d_order_mixed, n * sizeof(int32_t), hipMemcpyDeviceToHost), "hipMemcpy"))
            return QC_EHIP;
    }
    return h->d_order_mixed ? (int)h->acts.size() : 0;
}

int qc_env_tail(qc_handle* h, const qc_env_tail_args* in) {
    if (!h || !in) return QC_EINVAL;
    const qc_env_tail_args& x = *in;
    if (x.B != h->p.batch) return fail(h, QC_EINVAL, "env tail: B must be the handle's batch");
    if (x.kind != QC_IHO && x.kind != QC_IQO) return fail(h, QC_EINVAL, "env tail: the cartpole families (IHO, IQO)");
    if (x.kind == QC_IQO && !x.term_step) return fail(h, QC_EINVAL, "env tail: IQO needs term_step");
    if (x.B > 0 && (!x.fail_step || !x.obs || !x.pending || !x.t || !x.steps || !x.episode_return || !x.reward ||
                    !x.done || !x.valid || !x.fin || !x.fin_n || x.fin_cap < 1 || x.n_obs < 1 || x.interval < 1))
        return fail(h, QC_EINVAL, "env tail: missing buffer or bad size");
    EnvTailArgs a;
    std::memset(&a, 0, sizeof(a));
    a.B = x.B;
    a.kind = x.kind;
    a.n_obs = x.n_obs;
    a.interval = x.interval;
    a.dt = x.dt;
    a.xth = x.xth;
    a.input_scaling = x.input_scaling;
    a.failing_reward = x.failing_reward;
    a.fail_step = x.fail_step;
    a.term_step = x.term_step;
    a.obs = x.obs;
    a.pending = x.pending;
    a.t = x.t;
    a.steps = x.steps;
    a.episode_return = x.episode_return;
    a.obs32 = x.obs32;
    a.reward = x.reward;
    a.done = x.done;
    a.valid = x.valid;
    a.fin = x.fin;
    a.fin_cap = x.fin_cap;
    a.fin_n = x.fin_n;
    DeviceGuard g(h->device);
    return launch_env_tail(a, h->stream) ? fail(h, QC_EHIP, "env tail kernel launch failed") : QC_OK;
}

int qc_take_errors(qc_handle* h) {
    if (!h) return QC_EINVAL;
    DeviceGuard g(h->device);
    if (hipStreamSynchronize(h->stream) != hipSuccess) return fail(h, QC_EHIP, "reading the error word failed");
    if (!*h->h_bad) return QC_OK;
    *h->h_bad = 0;
    return fail(h, QC_EINVAL, "an action out of [0, n_slots) reached qc_step (clamped by the kernels)");
}

int qc_scan_levels(const qc_handle* h, int32_t action, int32_t* fwd, int32_t* bwd) {
    if (!h || action < 0 || action >= (int)h->acts.size()) return QC_EINVAL;
    if (fwd) *fwd = h->acts[action].kf;
    if (bwd) *bwd = h->acts[action].kb;
    return QC_OK;
}

}  // extern "C"
