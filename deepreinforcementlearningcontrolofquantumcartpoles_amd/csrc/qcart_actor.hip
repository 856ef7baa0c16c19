// qcart_actor.hip — batched DQN actor: the reference's direct_DQN action selection
// for B envs per launch, fused fc1 -> fc2 -> fc31 -> fc41 -> argmax -> epsilon-greedy.
//
// Reference: inverted harmonic oscillator/RL.py:80-111 (direct_DQN), layers.py:7-79 (FactorizedNoisy),
// layers.py:97-103 (Linear_weight_normalize), main_parallel.py:208-219 (epsilon-greedy in the actor) and
// :414-440 (the inference process: argmax of the action values).
//
// Design (MI355X): one workgroup = 32 envs x 4 waves. Every layer is Y[o][env] = W[o][k] X[k][env] on
// the f32-input MFMA v_mfma_f32_32x32x2_f32 (exact f32 accumulation): A = the layer's weights, stored
// once per load in fragment order (one coalesced 256-B read per MFMA), B = the activations in LDS as
// [feature][32 envs] (one conflict-free ds_read_b32 per MFMA), D = a 32-feature x 32-env tile whose
// rows land in the 16 accumulator registers. The epilogue adds bias / noise, applies ReLU and writes
// the next layer's input back to LDS; activations never leave the CU. A factorised noisy layer is two
// GEMMs per tile: u_w X and sigma_w (eps_in o X), combined as
//   y = u_w x + u_b + eps_out o (sigma_w (eps_in o x) + sigma_b)   (== (u_w + sigma_w o eps_out eps_in^T) x + ...)
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <string>

#include "../../include/qcart.h"
#include "qcart_kernels.hpp"

namespace qcart {
namespace actor {

constexpr int kE = 32;                 // envs per workgroup (one MFMA column block)
constexpr int kH1 = 512, kH2 = 256, kH3 = 256;
constexpr int kMaxIn = 512;            // data_length limit (LDS: [in][32] fp32 within 64 KiB)
constexpr int kThreads = 256;
using f32x16 = float __attribute__((ext_vector_type(16)));

// fragment buffer of one [O][K] matrix: tiles of 32 outputs x K/2 steps x 64 lanes
__host__ __device__ constexpr int tiles(int O) { return (O + 31) / 32; }
__host__ __device__ constexpr int ksteps(int K) { return (K + 1) / 2; }

struct Layer {
    const float* u;      // fragments of the (effective) weight
    const float* s;      // fragments of sigma_w (noisy) or null
    const float* ub;     // bias, padded to tiles*32
    const float* sb;     // sigma_b, padded, or null
};

struct ActArgs {
    Layer L[4];
    int in_len, in_pad, n_act;
    int64_t B, env_offset;
    const float* obs;
    int noisy;
    const float* noise;   // [noise_len][B] feature-major (internal layout)
    int64_t noise_ld;     // leading dimension of the noise buffer (>= B)
    float eps;
    uint64_t seed, counter;
    int32_t* actions;
    float* q_out;
    int32_t* random_out;
    // measurement network (DQN_measurement): the 256-wide fc1 output, feature-major [256][h_ld], enters
    // as H2; fc1 / fc2 of direct_DQN are skipped and L[2] / L[3] hold fc21 / fc31
    const float* h_in;
    int64_t h_ld;
};

// acc += A_frag(W) . X  over `steps` k-steps (X: LDS [k][32]; lane reads X[2s + (lane>>5)][lane&31]).
// The weight fragments come from L2: batches of kP steps, the next batch's loads issued before the
// current batch's MFMAs (kP x 64 cycles of MFMA cover the L2 latency at one wave per SIMD).
constexpr int kP = 16;
__device__ __forceinline__ void gemm_tile(f32x16& acc, const float* __restrict__ wf, const float* x, int steps,
                                          int lane) {
    const float* xl = x + (lane >> 5) * kE + (lane & 31);
    const float* wl = wf + lane;
    const int full = steps / kP * kP;
    f32x16 acc1 = {};   // second accumulator chain (odd steps): halves the dependent-MFMA chain
    float a[kP];
    if (full > 0) {
#pragma unroll
        for (int u = 0; u < kP; ++u) a[u] = wl[u * 64];
    }
    for (int s = 0; s < full; s += kP) {
        float an[kP];
        const int sn = s + kP < full ? s + kP : s;   // last batch: harmless reload of the same fragments
#pragma unroll
        for (int u = 0; u < kP; ++u) an[u] = wl[(sn + u) * 64];
        __builtin_amdgcn_sched_barrier(0);   // keep the next batch's loads ahead of this batch's MFMAs
#pragma unroll
        for (int u = 0; u < kP; u += 2) {
            acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u], xl[(s + u) * 2 * kE], acc, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[u + 1], xl[(s + u + 1) * 2 * kE], acc1, 0, 0, 0);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int u = 0; u < kP; ++u) a[u] = an[u];
    }
    for (int s = full; s < steps; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(wl[s * 64], xl[s * 2 * kE], acc, 0, 0, 0);
    acc += acc1;
}

// D-tile element r of this lane: output row (within the tile) and env column
__device__ __forceinline__ int drow(int r, int lane) { return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5); }

__device__ __forceinline__ float noise_at(const ActArgs& a, int f, int64_t e) {
    return a.noise[(int64_t)f * a.noise_ld + e];
}

__global__ __launch_bounds__(kThreads) void k_actor_act(const ActArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* RA = lds;                      // H1 [512][32]; later H3 [256][32] + H3e [256][32]
    float* RB = lds + kH1 * kE;           // X0 [in_pad][32]; later H2 [256][32] + H2e [256][32]
    float* RC = lds + 2 * kH1 * kE;       // fc41 sigma partial [32 rows][64 lanes... as D regs]
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int64_t e0 = (int64_t)blockIdx.x * kE;
    const int env = lane & 31;
    const int64_t eg = e0 + env;          // this lane's env (D column)
    const bool env_ok = eg < a.B;

    float* H2 = RB;
    float* H2e = RB + kH2 * kE;
    const bool n31 = a.noisy && a.L[2].s != nullptr;
    if (a.h_in) {
        // DQN_measurement: relu(fc1(x)) from HBM (coalesced 32-env rows) -> H2, eps_in(fc21) o H2
        for (int i = tid; i < kH2 * kE; i += kThreads) {
            const int k = i / kE, e = i % kE;
            const bool ok = e0 + e < a.B;
            const float h = ok ? a.h_in[(int64_t)k * a.h_ld + e0 + e] : 0.f;
            H2[i] = h;
            if (n31) H2e[i] = ok ? h * noise_at(a, k, e0 + e) : 0.f;
        }
        __syncthreads();
        goto fc31;
    }
    // ---- input: the fp32 network input (IHO/main_parallel.py:131,241) -> X0[k][env]
    for (int i = tid; i < a.in_pad * kE; i += kThreads) {
        const int k = i / kE, e = i % kE;
        RB[i] = (k < a.in_len && e0 + e < a.B) ? a.obs[(e0 + e) * a.in_len + k] : 0.f;
    }
    __syncthreads();

    // ---- fc1: 512 outputs = 16 tiles, 4 per wave; ReLU
    for (int t = wave; t < tiles(kH1); t += 4) {
        f32x16 acc = {};
        gemm_tile(acc, a.L[0].u + (size_t)t * ksteps(a.in_pad) * 64, RB, ksteps(a.in_pad), lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = t * 32 + drow(r, lane);
            RA[o * kE + env] = fmaxf(acc[r] + a.L[0].ub[o], 0.f);
        }
    }
    __syncthreads();

    // ---- fc2: 256 outputs = 8 tiles, 2 per wave; ReLU; also eps_in(fc31) o H2 for the noisy GEMM
    for (int t = wave; t < tiles(kH2); t += 4) {
        f32x16 acc = {};
        gemm_tile(acc, a.L[1].u + (size_t)t * ksteps(kH1) * 64, RA, ksteps(kH1), lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = t * 32 + drow(r, lane);
            const float h = fmaxf(acc[r] + a.L[1].ub[o], 0.f);
            H2[o * kE + env] = h;
            if (n31) H2e[o * kE + env] = env_ok ? h * noise_at(a, o, eg) : 0.f;
        }
    }
    __syncthreads();

    // ---- fc31 (noisy or weight-normalised): 8 tiles, 2 per wave; ReLU; eps_in(fc41) o H3
fc31:
    float* H3 = RA;
    float* H3e = RA + kH3 * kE;
    const bool n41 = a.noisy && a.L[3].s != nullptr;
    for (int t = wave; t < tiles(kH3); t += 4) {
        f32x16 acc = {}, accs = {};
        gemm_tile(acc, a.L[2].u + (size_t)t * ksteps(kH2) * 64, H2, ksteps(kH2), lane);
        if (n31) gemm_tile(accs, a.L[2].s + (size_t)t * ksteps(kH2) * 64, H2e, ksteps(kH2), lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            const int o = t * 32 + drow(r, lane);
            float y = acc[r] + a.L[2].ub[o];
            if (n31) y += env_ok ? noise_at(a, kH2 + o, eg) * (accs[r] + a.L[2].sb[o]) : 0.f;
            const float h = fmaxf(y, 0.f);
            H3[o * kE + env] = h;
            if (n41) H3e[o * kE + env] = env_ok ? h * noise_at(a, 2 * kH2 + o, eg) : 0.f;
        }
    }
    __syncthreads();

    // ---- fc41: one 32-row tile; wave 0: u_w H3, wave 1: sigma_w (eps_in o H3) -> LDS partial
    if (wave == 1 && n41) {
        f32x16 accs = {};
        gemm_tile(accs, a.L[3].s, H3e, ksteps(kH3), lane);
#pragma unroll
        for (int r = 0; r < 16; ++r) RC[r * 64 + lane] = accs[r];
    }
    f32x16 acc = {};
    if (wave == 0) gemm_tile(acc, a.L[3].u, H3, ksteps(kH3), lane);
    __syncthreads();
    if (wave != 0) return;

    // ---- action values, argmax (lowest index among equal maxima), epsilon-greedy
    float best = -INFINITY;
    int besti = 0x7fffffff;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int o = drow(r, lane);
        if (o < a.n_act) {
            float q = acc[r] + a.L[3].ub[o];
            if (n41) q += env_ok ? noise_at(a, 2 * kH2 + kH3 + o, eg) * (RC[r * 64 + lane] + a.L[3].sb[o]) : 0.f;
            if (a.q_out && env_ok) a.q_out[eg * a.n_act + o] = q;
            if (q > best || (q == best && o < besti)) {
                best = q;
                besti = o;
            }
        }
    }
    const float ob = __shfl_xor(best, 32, 64);
    const int oi = __shfl_xor(besti, 32, 64);
    if (ob > best || (ob == best && oi < besti)) besti = oi;
    if (lane < 32 && env_ok) {
        int act = besti;
        int rnd = 0;
        if (a.eps > 0.f) {
            uint32_t c[4] = {(uint32_t)a.counter, (uint32_t)(a.counter >> 32), (uint32_t)(a.env_offset + eg), 0x200u};
            philox10(c, (uint32_t)a.seed, (uint32_t)(a.seed >> 32));
            const float u1 = (float)(c[0] >> 8) * 0x1.0p-24f, u2 = (float)(c[1] >> 8) * 0x1.0p-24f;
            if (u1 < a.eps) {   // random.random() < eps_threshold -> random.randrange(21)
                act = min((int)(u2 * (float)a.n_act), a.n_act - 1);
                rnd = 1;
            }
        }
        a.actions[eg] = act;
        if (a.random_out) a.random_out[eg] = rnd;
    }
}

// NoisyNet noise, feature-major [noise_len][ld]: f(z) = sign(z) sqrt|z| (layers.py:77-79) of Philox
// normals keyed by (seed, env_offset + e), counter, tag 0x100 + pair
__global__ __launch_bounds__(256) void k_actor_noise(float* out, int64_t ld, int64_t B, int noise_len,
                                                     int64_t env_offset, uint64_t seed, uint64_t counter) {
    const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int p = blockIdx.y;
    if (e >= B) return;
    // Box-Muller in fp32 (hardware log / sin / cos): the network noise is fp32 and has no oracle stream
    uint32_t c[4] = {(uint32_t)counter, (uint32_t)(counter >> 32), (uint32_t)(env_offset + e), 0x100u + (uint32_t)p};
    philox10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const float u1 = ((float)(c[0] >> 8) + 0.5f) * 0x1.0p-24f, u2 = (float)(c[1] >> 8) * 0x1.0p-24f;
    const float rad = sqrtf(-2.f * __logf(u1));
    float sn, cs;
    __sincosf(6.283185307f * u2, &sn, &cs);
    const float f0 = rad * cs, f1 = rad * sn;
    out[(int64_t)(2 * p) * ld + e] = copysignf(sqrtf(fabsf(f0)), f0);
    if (2 * p + 1 < noise_len) out[(int64_t)(2 * p + 1) * ld + e] = copysignf(sqrtf(fabsf(f1)), f1);
}

// injected noise [B][noise_len] -> feature-major [noise_len][ld]
__global__ __launch_bounds__(256) void k_actor_transpose(const float* in, float* out, int64_t ld, int64_t B,
                                                         int noise_len) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= B * noise_len) return;
    const int64_t e = i / noise_len;
    const int f = (int)(i % noise_len);
    out[(int64_t)f * ld + e] = in[i];
}

// effective weight (W g / ||W||_F, or W) -> fragments [tile][step][64]; bias padded to tiles*32
// split = 0: MFMA k-step s pairs k = 2s, 2s + 1 (lane halves); split = 1: k = s, s + Kpad / 2 (the
// convolutions: the upper half of K is then a fixed input offset, see k_mconv)
__global__ __launch_bounds__(1024) void k_actor_prep(const float* W, const float* g, int O, int K, int Kpad,
                                                     float* frag, const float* bias, float* bias_pad, int split) {
    __shared__ double part[1024];
    double ss = 0.0;
    if (g) {
        for (int i = threadIdx.x; i < O * K; i += 1024) ss += (double)W[i] * (double)W[i];
    }
    part[threadIdx.x] = ss;
    __syncthreads();
    for (int w = 512; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) part[threadIdx.x] += part[threadIdx.x + w];
        __syncthreads();
    }
    const float sc = g ? (float)((double)g[0] / sqrt(part[0])) : 1.f;
    const int T = tiles(O), S = ksteps(Kpad);
    for (int i = threadIdx.x; i < T * S * 64; i += 1024) {
        const int l = i & 63, s = (i >> 6) % S, t = (i >> 6) / S;
        const int o = t * 32 + (l & 31), k = split ? s + (l >> 5) * S : 2 * s + (l >> 5);
        frag[i] = (o < O && k < K) ? W[(size_t)o * K + k] * sc : 0.f;
    }
    if (bias_pad)
        for (int i = threadIdx.x; i < T * 32; i += 1024) bias_pad[i] = (i < O && bias) ? bias[i] : 0.f;
}

// ---- DQN_measurement (IHO/RL.py:29-78): Conv1d stack as implicit GEMMs on f32 MFMA ----------------
// Y[b][co][t] = relu(bias[co] + sum_{ci, j} W[co][ci][j] X[b][ci][S t + j]): M = co (MT tiles of 32),
// N = (env, position) flattened (32 columns per wave), K = ci * KS in pairs (k = ci * KS + j, the
// PyTorch weight order). A = weight fragments (k_actor_prep order), B = the input gathered per lane
// from HBM / L2 (column base X[b] + S t; row offset ci * Tin + j, wave-uniform per k-step half).
// Loads run one batch of kQ k-steps ahead of the MFMAs (two register sets, no copies); every load is
// unconditional (columns past the end read the workgroup's first env, whose results are not stored).
// Output: env-major [b][co][t] (32 consecutive t per store: one 128-B run); conv3's is transposed
// afterwards by k_mtr into fc1's feature-major operand (written directly, every lane's store hit its own
// cache line: 4.6 M partial-line writes per chunk). NT column tiles per wave: every weight fragment
// feeds NT MFMAs, every input value MT. (A polyphase activation layout that turns the stride-S gathers into
// contiguous runs was measured: conv2/conv3 unchanged, conv1's scattered stores +23 %; not kept.)
constexpr int kNTs[3] = {QCART_MCONV_NT};   // (knob defaults: qcart_expt.hpp)
constexpr int kNT1 = kNTs[0], kNT2 = kNTs[1], kNT3 = kNTs[2];
constexpr int kNAs[3] = {QCART_MCONV_NA};
constexpr int kNA1 = kNAs[0], kNA2 = kNAs[1], kNA3 = kNAs[2];
constexpr int kQs[3] = {QCART_MCONV_Q};   // k-steps per load batch
constexpr int kQ1 = kQs[0], kQ2 = kQs[1], kQ3 = kQs[2];
template <int CI, int KS, int S, int MT, int NT, int NA, int kQ>
__global__ __launch_bounds__(256) void k_mconv(const float* __restrict__ X, int Tin, const float* __restrict__ Wf,
                                               const float* __restrict__ bias, float* __restrict__ Y, int Tout,
                                               int64_t n_total) {
    constexpr int K = CI * KS, STEPS = K / 2;
    static_assert(CI % 2 == 0, "split-K pairing: k and k + K/2 are channels ci and ci + CI/2");
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int hi = lane >> 5;
    // buffer descriptor at the workgroup's first env: every lane offset is a small 32-bit VGPR, the
    // k-step's row offset is wave-uniform (SGPR), so a load costs no VALU
    const int64_t b0 = (int64_t)blockIdx.x * 128 * NT / Tout;
    const rsrc_t rx = make_rsrc(X + b0 * CI * Tin, 0xFFFFFFFFu);
    const rsrc_t rw = make_rsrc(Wf, 0xFFFFFFFFu);
    bool col_ok[NT];
    int64_t bb[NT];
    int tt[NT];
    int vx[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
        const int64_t n = (((int64_t)blockIdx.x * 4 + wave) * NT + c) * 32 + (lane & 31);
        col_ok[c] = n < n_total;
        bb[c] = col_ok[c] ? n / Tout : b0;
        tt[c] = col_ok[c] ? (int)(n - bb[c] * Tout) : 0;
        vx[c] = (int)(((bb[c] - b0) * CI * Tin + S * tt[c] + hi * (CI / 2) * Tin) * 4);
    }
    const int vw = lane * 4;
    // NA accumulator sets for alternating k-steps: NA * MT * NT independent MFMA chains (an MFMA that
    // accumulates onto the previous one's result waits for it)
    f32x16 acc[NA][MT][NT];
#pragma unroll
    for (int q = 0; q < NA; ++q)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int c = 0; c < NT; ++c) acc[q][m][c] = f32x16{};
    // k-step s pairs k = s (lanes 0-31) and k = s + K/2 (lanes 32-63); clamped into range (a prefetch
    // past the end reloads the last step, unused)
    auto fetch = [&](int s, float (&x)[kQ][NT], float (&w)[kQ][MT]) {
#pragma unroll
        for (int u = 0; u < kQ; ++u) {
            const int sc = min(s + u, STEPS - 1);
            const int so = ((sc / KS) * Tin + sc % KS) * 4;   // ci * Tin + j
#pragma unroll
            for (int c = 0; c < NT; ++c) x[u][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, vx[c], so, 0));
#pragma unroll
            for (int m = 0; m < MT; ++m)
                w[u][m] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, vw, (m * STEPS + sc) * 256, 0));
        }
    };
    auto mma = [&](int n, const float (&x)[kQ][NT], const float (&w)[kQ][MT]) {
#pragma unroll
        for (int u = 0; u < kQ; ++u)
            if (u < n)
#pragma unroll
                for (int m = 0; m < MT; ++m)
#pragma unroll
                    for (int c = 0; c < NT; ++c)
                        acc[u % NA][m][c] =
                            __builtin_amdgcn_mfma_f32_32x32x2f32(w[u][m], x[u][c], acc[u % NA][m][c], 0, 0, 0);
    };
    float xa[kQ][NT], wa[kQ][MT], xb[kQ][NT], wb[kQ][MT];
    fetch(0, xa, wa);
    int s = 0;
    // the next batch's loads interleaved one by one with this batch's MFMAs (sched_group_barrier:
    // VMEM read 0x020, MFMA 0x008), so the load issue never holds the MFMA stream back
    constexpr int NLD = kQ * (NT + MT), NMF = kQ * MT * NT;
    auto interleave = [&]() {
#pragma unroll
        for (int i = 0; i < (NLD > NMF ? NLD : NMF); ++i) {
            if (i < NLD) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            if (i < NMF) __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        }
    };
    for (; s + 2 * kQ <= STEPS; s += 2 * kQ) {
        fetch(s + kQ, xb, wb);
        mma(kQ, xa, wa);
        interleave();
        __builtin_amdgcn_sched_barrier(0);
        fetch(s + 2 * kQ, xa, wa);
        mma(kQ, xb, wb);
        interleave();
        __builtin_amdgcn_sched_barrier(0);
    }
    if (s + kQ <= STEPS) {   // one full batch (in xa) and a partial one
        fetch(s + kQ, xb, wb);
        mma(kQ, xa, wa);
        mma(STEPS - s - kQ, xb, wb);
    } else {
        mma(STEPS - s, xa, wa);
    }
#pragma unroll
    for (int q = 1; q < NA; ++q)
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int c = 0; c < NT; ++c) acc[0][m][c] += acc[q][m][c];
    float bv[MT][16];   // bias of this lane's output rows, loaded as one batch before the stores
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[m][r] = bias[m * 32 + drow(r, lane)];
    // stores through a descriptor at the workgroup's first env: per-lane offset (env, position, the lane
    // half's 4-row shift) in a VGPR, the output row's (m 32 + (r & 3) + 8 (r >> 2)) Tout wave-uniform
    const rsrc_t ry = make_rsrc(Y + b0 * (MT * 32) * Tout, 0xFFFFFFFFu);
#pragma unroll
    for (int c = 0; c < NT; ++c) {
        if (!col_ok[c]) continue;
        const int vy = (int)((((bb[c] - b0) * (MT * 32) + 4 * hi) * Tout + tt[c]) * 4);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int row = m * 32 + (r & 3) + 8 * (r >> 2);
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaxf(acc[0][m][c][r] + bv[m][r], 0.f)), ry, vy,
                                                      row * Tout * 4, 0);
            }
    }
}

// conv3's env-major chunk output [nb][F] -> fc1's feature-major operand [F][ld] at env column c0: 64x64
// tiles through LDS, coalesced on both sides
__global__ __launch_bounds__(256) void k_mtr(const float* __restrict__ in, float* __restrict__ out, int F,
                                             int64_t nb, int64_t ld, int64_t c0) {
    __shared__ float t[64][65];
    const int64_t b0 = (int64_t)blockIdx.y * 64;
    const int f0 = blockIdx.x * 64, tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
    for (int r = ty; r < 64; r += 4) {
        const int64_t b = b0 + r;
        t[r][tx] = (b < nb && f0 + tx < F) ? in[b * F + f0 + tx] : 0.f;
    }
    __syncthreads();
    for (int r = ty; r < 64; r += 4) {
        const int f = f0 + r;
        if (f < F && b0 + tx < nb) out[(int64_t)f * ld + c0 + b0 + tx] = t[tx][r];
    }
}

// fc1 (nn.Linear K -> 256) + ReLU: B = the feature-major conv output X[k][x_ld] (one coalesced 128-B row
// per k-step half and column tile). A wave computes MT of the 8 output tiles for NT * 32 envs; the 8 / MT
// waves that share an env group sit in one workgroup (their B reads coincide in L1 / L2). Weight
// traffic per env is 8 / (MT * NT) tile streams of K: (MT, NT) = (8, 1) streams the 4.6 MB weight
// matrix once per 32 envs — more than one XCD's L2, so from MALL. Buffer loads with wave-uniform
// k-step offsets, batches of kQF k-steps loaded one batch ahead of the MFMAs.
constexpr int kMfcMT = QCART_MFC_MT, kMfcNT = QCART_MFC_NT, kQF = 4;
template <int MT, int NT>
__global__ __launch_bounds__(256) void k_mfc(const float* __restrict__ X, int64_t x_ld, int K,
                                             const float* __restrict__ Wf, const float* __restrict__ bias,
                                             float* __restrict__ H, int64_t B) {
    constexpr int MP = 8 / MT;   // waves per env group
    static_assert(4 % MP == 0, "the waves of an env group share a workgroup");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // uniform: descriptors stay in SGPRs
    const int mp = wave % MP;
    const int64_t e0 = ((int64_t)blockIdx.x * (4 / MP) + wave / MP) * NT * 32;
    const int steps = K / 2, hi = lane >> 5;   // K = 64 T3 is even
    const rsrc_t rx = make_rsrc(X + e0, 0xFFFFFFFFu);
    const rsrc_t rw = make_rsrc(Wf + (size_t)mp * MT * steps * 64, 0xFFFFFFFFu);
    bool ok[NT];
    int vx[NT];
#pragma unroll
    for (int c = 0; c < NT; ++c) {
        const int64_t e = e0 + c * 32 + (lane & 31);
        ok[c] = e < B;
        vx[c] = (int)(((ok[c] ? c * 32 + (lane & 31) : 0) + (int64_t)hi * x_ld) * 4);   // row k = 2 s + hi
    }
    const int vw = lane * 4;
    f32x16 acc[MT][NT];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int c = 0; c < NT; ++c) acc[m][c] = f32x16{};
    auto fetch = [&](int s, float (&x)[kQF][NT], float (&w)[kQF][MT]) {
#pragma unroll
        for (int u = 0; u < kQF; ++u) {
            const int sc = min(s + u, steps - 1);
            const int xo = (int)((uint32_t)(2 * sc) * (uint32_t)x_ld * 4u);   // < 4 GiB: checked at create
#pragma unroll
            for (int c = 0; c < NT; ++c) x[u][c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, vx[c], xo, 0));
#pragma unroll
            for (int m = 0; m < MT; ++m)
                w[u][m] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, vw, (m * steps + sc) * 256, 0));
        }
    };
    auto mma = [&](const float (&x)[kQF][NT], const float (&w)[kQF][MT]) {
#pragma unroll
        for (int u = 0; u < kQF; ++u)
#pragma unroll
            for (int m = 0; m < MT; ++m)
#pragma unroll
                for (int c = 0; c < NT; ++c)
                    acc[m][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[u][m], x[u][c], acc[m][c], 0, 0, 0);
    };
    float xa[kQF][NT], wa[kQF][MT], xb[kQF][NT], wb[kQF][MT];
    // runtime K (= 64 T3 >= 64, so at least one double batch): whole double batches, then single steps
    const int full = steps / (2 * kQF) * (2 * kQF);
    int s = 0;
    fetch(0, xa, wa);
    do {
        fetch(s + kQF, xb, wb);
        __builtin_amdgcn_sched_barrier(0);
        mma(xa, wa);
        __builtin_amdgcn_sched_barrier(0);
        fetch(s + 2 * kQF, xa, wa);   // past the end: clamped re-reads, unused
        __builtin_amdgcn_sched_barrier(0);
        mma(xb, wb);
        __builtin_amdgcn_sched_barrier(0);
        s += 2 * kQF;
    } while (s < full);
    for (; s < steps; ++s) {
        float x1[NT], w1[MT];
#pragma unroll
        for (int c = 0; c < NT; ++c)
            x1[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rx, vx[c], (int)((uint32_t)(2 * s) * (uint32_t)x_ld * 4u), 0));
#pragma unroll
        for (int m = 0; m < MT; ++m) w1[m] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw, vw, (m * steps + s) * 256, 0));
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int c = 0; c < NT; ++c) acc[m][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(w1[m], x1[c], acc[m][c], 0, 0, 0);
    }
    float bv[MT][16];
#pragma unroll
    for (int m = 0; m < MT; ++m)
#pragma unroll
        for (int r = 0; r < 16; ++r) bv[m][r] = bias[(mp * MT + m) * 32 + drow(r, lane)];
    // feature-major [256][ld] through a descriptor at (row 0, env e0): per-lane offset (column, the
    // lane half's 4-row shift) in a VGPR, the row's offset ((mp MT + m) 32 + (r & 3) + 8 (r >> 2)) x_ld
    // wave-uniform (SGPR)
    const rsrc_t rh = make_rsrc(H + e0, 0xFFFFFFFFu);
#pragma unroll
    for (int c = 0; c < NT; ++c) {
        if (!ok[c]) continue;
        const int vh = (int)((c * 32 + (lane & 31) + (int64_t)4 * hi * x_ld) * 4);
#pragma unroll
        for (int m = 0; m < MT; ++m)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const uint32_t row = (uint32_t)((mp * MT + m) * 32 + (r & 3) + 8 * (r >> 2));
                __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(fmaxf(acc[m][c][r] + bv[m][r], 0.f)), rh, vh,
                                                      (int)(row * (uint32_t)x_ld * 4u), 0);
            }
    }
}

}  // namespace actor
}  // namespace qcart

using namespace qcart::actor;

struct qc_actor {
    qc_dqn_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    int in_pad = 0, noise_len = 0;
    bool loaded = false;
    bool has_s[4] = {false, false, false, false};
    std::string err;
    float* d_w = nullptr;        // all fragments + padded biases
    size_t off_u[4]{}, off_s[4]{}, off_ub[4]{}, off_sb[4]{};
    size_t w_floats = 0;
    float* d_noise = nullptr;    // [noise_len][max_batch]
};

namespace {
std::mutex g_actor_mu;
std::string g_actor_err;

struct Dev {
    int prev = -1;
    explicit Dev(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~Dev() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int hip_fail(qc_actor* a, hipError_t e, const char* what) {
    a->err = std::string(what) + ": " + hipGetErrorString(e);
    return QC_EHIP;
}

constexpr int kLayerO[4] = {kH1, kH2, kH3, 0};
}  // namespace

extern "C" {

int qc_actor_create(const qc_dqn_params* p, int device, qc_actor** out) {
    if (!out || !p) return QC_EINVAL;
    *out = nullptr;
    auto fail = [](const char* m, int rc) {
        std::lock_guard<std::mutex> lk(g_actor_mu);
        g_actor_err = m;
        return rc;
    };
    if (p->data_length < 1 || p->data_length > kMaxIn) return fail("data_length must be in [1, 512]", QC_EINVAL);
    if (p->n_actions < 1 || p->n_actions > 32) return fail("n_actions must be in [1, 32]", QC_EINVAL);
    if (p->max_batch < 1) return fail("max_batch must be >= 1", QC_EINVAL);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0)
        return fail("no HIP device available (the actor has no CPU fallback)", QC_EHIP);
    if (device < 0 || device >= ndev) return fail("device index out of range", QC_EINVAL);
    qc_actor* a = new qc_actor();
    a->p = *p;
    a->device = device;
    a->in_pad = (p->data_length + 1) & ~1;
    a->noise_len = 2 * kH2 + kH3 + p->n_actions;
    const int K[4] = {a->in_pad, kH1, kH2, kH3};
    const int O[4] = {kH1, kH2, kH3, p->n_actions};
    size_t off = 0;
    for (int l = 0; l < 4; ++l) {
        const size_t fr = (size_t)tiles(O[l]) * ksteps(K[l]) * 64, bp = (size_t)tiles(O[l]) * 32;
        a->off_u[l] = off; off += fr;
        a->off_s[l] = off; off += fr;
        a->off_ub[l] = off; off += bp;
        a->off_sb[l] = off; off += bp;
    }
    a->w_floats = off;
    Dev g(device);
    hipError_t e = hipMalloc(&a->d_w, off * sizeof(float));
    if (e == hipSuccess) e = hipMemset(a->d_w, 0, off * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&a->d_noise, (size_t)a->noise_len * (size_t)p->max_batch * sizeof(float));
    if (e != hipSuccess) {
        if (a->d_w) (void)hipFree(a->d_w);
        if (a->d_noise) (void)hipFree(a->d_noise);
        delete a;
        return fail("device allocation failed", QC_ENOMEM);
    }
    if (hipFuncSetAttribute((const void*)k_actor_act, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (2 * kH1 * kE + 16 * 64) * (int)sizeof(float)) != hipSuccess) {
        (void)hipFree(a->d_w);
        (void)hipFree(a->d_noise);
        delete a;
        return fail("cannot enable 140 KiB of LDS for the actor kernel", QC_EHIP);
    }
    *out = a;
    (void)kLayerO;
    return QC_OK;
}

void qc_actor_destroy(qc_actor* a) {
    if (!a) return;
    {
        Dev g(a->device);
        (void)hipDeviceSynchronize();
        if (a->d_w) (void)hipFree(a->d_w);
        if (a->d_noise) (void)hipFree(a->d_noise);
    }
    delete a;
}

const char* qc_actor_last_error(const qc_actor* a) {
    if (a) return a->err.c_str();
    std::lock_guard<std::mutex> lk(g_actor_mu);
    return g_actor_err.c_str();
}

int qc_actor_set_stream(qc_actor* a, void* stream) {
    if (!a) return QC_EINVAL;
    a->stream = (hipStream_t)stream;
    return QC_OK;
}

int qc_actor_noise_len(const qc_actor* a) { return a ? a->noise_len : QC_EINVAL; }

int qc_actor_load(qc_actor* a, const qc_dqn_layer layers[4]) {
    if (!a || !layers) return QC_EINVAL;
    const int K[4] = {a->p.data_length, kH1, kH2, kH3};
    const int Kp[4] = {a->in_pad, kH1, kH2, kH3};
    const int O[4] = {kH1, kH2, kH3, a->p.n_actions};
    for (int l = 0; l < 4; ++l) {
        const qc_dqn_layer& L = layers[l];
        if (!L.weight || !L.bias) { a->err = "layer " + std::to_string(l) + ": weight and bias are required"; return QC_EINVAL; }
        if (l < 2 && (!L.weight_norm || L.sigma_w)) {
            a->err = "fc1 / fc2 are Linear_weight_normalize layers (weight_norm required, no sigma)";
            return QC_EINVAL;
        }
        if ((L.sigma_w == nullptr) != (L.sigma_b == nullptr)) { a->err = "sigma_w and sigma_b go together"; return QC_EINVAL; }
        if (L.sigma_w && L.weight_norm) { a->err = "a noisy layer has no weight_norm"; return QC_EINVAL; }
        if (!L.sigma_w && !L.weight_norm) { a->err = "a deterministic layer needs weight_norm"; return QC_EINVAL; }
    }
    Dev g(a->device);
    float* w = a->d_w;
    for (int l = 0; l < 4; ++l) {
        const qc_dqn_layer& L = layers[l];
        hipLaunchKernelGGL(k_actor_prep, dim3(1), dim3(1024), 0, a->stream, L.weight, L.weight_norm, O[l], K[l], Kp[l],
                           w + a->off_u[l], L.bias, w + a->off_ub[l], 0);
        a->has_s[l] = L.sigma_w != nullptr;
        if (L.sigma_w)
            hipLaunchKernelGGL(k_actor_prep, dim3(1), dim3(1024), 0, a->stream, L.sigma_w, (const float*)nullptr, O[l],
                               K[l], Kp[l], w + a->off_s[l], L.sigma_b, w + a->off_sb[l], 0);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(a, e, "actor weight preparation");
    a->loaded = true;
    return QC_OK;
}

int qc_actor_act(qc_actor* a, int64_t B, int64_t env_offset, const float* obs, int32_t noisy, const float* noise,
                 double eps, uint64_t counter, int32_t* actions, float* q_out, int32_t* random_out) {
    if (!a) return QC_EINVAL;
    if (!a->loaded) { a->err = "qc_actor_load has not been called"; return QC_EINVAL; }
    if (B < 0 || B > a->p.max_batch) { a->err = "B must be in [0, max_batch]"; return QC_EINVAL; }
    if (B == 0) return QC_OK;
    if (!obs || !actions) { a->err = "obs and actions are required"; return QC_EINVAL; }
    Dev g(a->device);
    const bool need_noise = noisy && (a->has_s[2] || a->has_s[3]);
    if (need_noise) {
        if (noise) {
            const int64_t n = B * a->noise_len;
            hipLaunchKernelGGL(k_actor_transpose, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, a->stream, noise,
                               a->d_noise, a->p.max_batch, B, a->noise_len);
        } else {
            hipLaunchKernelGGL(k_actor_noise, dim3((unsigned)((B + 255) / 256), (unsigned)((a->noise_len + 1) / 2)),
                               dim3(256), 0, a->stream, a->d_noise, a->p.max_batch, B, a->noise_len, env_offset,
                               a->p.seed, counter);
        }
    }
    ActArgs k{};
    for (int l = 0; l < 4; ++l) {
        k.L[l].u = a->d_w + a->off_u[l];
        k.L[l].ub = a->d_w + a->off_ub[l];
        k.L[l].s = a->has_s[l] ? a->d_w + a->off_s[l] : nullptr;
        k.L[l].sb = a->has_s[l] ? a->d_w + a->off_sb[l] : nullptr;
    }
    k.in_len = a->p.data_length;
    k.in_pad = a->in_pad;
    k.n_act = a->p.n_actions;
    k.B = B;
    k.env_offset = env_offset;
    k.obs = obs;
    k.noisy = need_noise ? 1 : 0;
    k.noise = a->d_noise;
    k.noise_ld = a->p.max_batch;
    k.eps = (float)eps;
    k.seed = a->p.seed;
    k.counter = counter;
    k.actions = actions;
    k.q_out = q_out;
    k.random_out = random_out;
    hipLaunchKernelGGL(k_actor_act, dim3((unsigned)((B + kE - 1) / kE)), dim3(kThreads),
                       (2 * kH1 * kE + 16 * 64) * sizeof(float), a->stream, k);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(a, e, "actor launch");
    return QC_OK;
}

}  // extern "C"

// ---- the measurement-input actor (DQN_measurement, IHO/RL.py:29-78) --------------------------------
struct qc_mactor {
    qc_mdqn_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    int T1 = 0, T2 = 0, T3 = 0, flat = 0, chunk = 0, noise_len = 0;
    bool loaded = false, has_s21 = false, has_s31 = false;
    float* d_w = nullptr;
    size_t off_w[6]{}, off_b[6]{}, off_s[6]{}, off_sb[6]{};
    float *d_y1 = nullptr, *d_y2 = nullptr, *d_y3e = nullptr, *d_y3 = nullptr, *d_h1 = nullptr, *d_noise = nullptr;
};

namespace {
std::string g_mactor_err;
// layer shapes: conv1 (32, 2, 13, /5), conv2 (64, 32, 11, /4), conv3 (64, 64, 9, /4) (RL.py:36-45)
constexpr int kC1 = 32, kC2 = 64, kC3 = 64;
int conv_out(int n, int k, int s) { return (n - (k - 1) + (s - 1)) / s; }   // calculate_next_layer_dim (RL.py:49-50)
}  // namespace

extern "C" {

int qc_mactor_create(const qc_mdqn_params* p, int device, qc_mactor** out) {
    if (!out || !p) return QC_EINVAL;
    *out = nullptr;
    auto fail = [](const char* m, int rc) {
        std::lock_guard<std::mutex> lk(g_actor_mu);
        g_mactor_err = m;
        return rc;
    };
    if (p->n_actions < 1 || p->n_actions > 32) return fail("n_actions must be in [1, 32]", QC_EINVAL);
    if (p->max_batch < 1) return fail("max_batch must be >= 1", QC_EINVAL);
    qc_mactor* a = new qc_mactor();
    a->p = *p;
    a->device = device;
    a->T1 = conv_out(p->read_length, 13, 5);
    a->T2 = conv_out(a->T1, 11, 4);
    a->T3 = conv_out(a->T2, 9, 4);
    if (p->read_length < 1 || a->T3 < 1) {
        delete a;
        return fail("read_length too short for the three convolutions", QC_EINVAL);
    }
    a->flat = kC3 * a->T3;
    if ((uint64_t)a->flat * (uint64_t)p->max_batch * sizeof(float) >= (1ull << 32)) {   // 32-bit buffer offsets
        delete a;
        return fail("max_batch too large: fc1's operand [64 T3][max_batch] must stay below 4 GiB", QC_EINVAL);
    }
    a->noise_len = 2 * kH2 + kH3 + p->n_actions;
    a->chunk = (int)std::min<int64_t>(p->max_batch, p->chunk > 0 ? p->chunk : 2048);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        delete a;
        return fail("no HIP device available (the actor has no CPU fallback)", QC_EHIP);
    }
    if (device < 0 || device >= ndev) {
        delete a;
        return fail("device index out of range", QC_EINVAL);
    }
    const int O[6] = {kC1, kC2, kC3, kH2, kH3, p->n_actions};
    const int K[6] = {2 * 13, kC1 * 11, kC2 * 9, a->flat, kH2, kH3};
    size_t off = 0;
    for (int l = 0; l < 6; ++l) {
        const size_t fr = (size_t)tiles(O[l]) * ksteps(K[l]) * 64, bp = (size_t)tiles(O[l]) * 32;
        a->off_w[l] = off; off += fr;
        a->off_b[l] = off; off += bp;
        if (l >= 4) {
            a->off_s[l] = off; off += fr;
            a->off_sb[l] = off; off += bp;
        }
    }
    Dev g(device);
    const size_t mb = (size_t)p->max_batch, ch = (size_t)a->chunk;
    hipError_t e = hipMalloc(&a->d_w, off * sizeof(float));
    if (e == hipSuccess) e = hipMemset(a->d_w, 0, off * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&a->d_y1, ch * kC1 * a->T1 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&a->d_y2, ch * kC2 * a->T2 * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&a->d_y3e, (size_t)a->flat * ch * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&a->d_y3, (size_t)a->flat * mb * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&a->d_h1, (size_t)kH2 * mb * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&a->d_noise, (size_t)a->noise_len * mb * sizeof(float));
    if (e == hipSuccess &&
        hipFuncSetAttribute((const void*)k_actor_act, hipFuncAttributeMaxDynamicSharedMemorySize,
                            (2 * kH1 * kE + 16 * 64) * (int)sizeof(float)) != hipSuccess)
        e = hipErrorInvalidValue;
    if (e != hipSuccess) {
        qc_mactor_destroy(a);
        return fail("device allocation failed", QC_ENOMEM);
    }
    *out = a;
    return QC_OK;
}

void qc_mactor_destroy(qc_mactor* a) {
    if (!a) return;
    {
        Dev g(a->device);
        (void)hipDeviceSynchronize();
        for (float* q : {a->d_w, a->d_y1, a->d_y2, a->d_y3e, a->d_y3, a->d_h1, a->d_noise})
            if (q) (void)hipFree(q);
    }
    delete a;
}

const char* qc_mactor_last_error(const qc_mactor* a) {
    if (a) return a->err.c_str();
    std::lock_guard<std::mutex> lk(g_actor_mu);
    return g_mactor_err.c_str();
}

int qc_mactor_set_stream(qc_mactor* a, void* stream) {
    if (!a) return QC_EINVAL;
    a->stream = (hipStream_t)stream;
    return QC_OK;
}

int qc_mactor_noise_len(const qc_mactor* a) { return a ? a->noise_len : QC_EINVAL; }
int qc_mactor_flat_len(const qc_mactor* a) { return a ? a->flat : QC_EINVAL; }

int qc_mactor_load(qc_mactor* a, const qc_dqn_layer layers[6]) {
    if (!a || !layers) return QC_EINVAL;
    const int O[6] = {kC1, kC2, kC3, kH2, kH3, a->p.n_actions};
    const int K[6] = {2 * 13, kC1 * 11, kC2 * 9, a->flat, kH2, kH3};
    for (int l = 0; l < 6; ++l) {
        const qc_dqn_layer& L = layers[l];
        if (!L.weight || !L.bias) { a->err = "layer " + std::to_string(l) + ": weight and bias are required"; return QC_EINVAL; }
        if (l < 4 && (L.sigma_w || L.weight_norm)) {
            a->err = "conv1..3 and fc1 are plain Conv1d / Linear layers (no weight_norm, no sigma)";
            return QC_EINVAL;
        }
        if ((L.sigma_w == nullptr) != (L.sigma_b == nullptr)) { a->err = "sigma_w and sigma_b go together"; return QC_EINVAL; }
        if (l >= 4 && !L.sigma_w && !L.weight_norm) { a->err = "fc21 / fc31: FactorizedNoisy or Linear_weight_normalize"; return QC_EINVAL; }
    }
    Dev g(a->device);
    float* w = a->d_w;
    for (int l = 0; l < 6; ++l) {
        const qc_dqn_layer& L = layers[l];
        const int Kp = (K[l] + 1) & ~1;
        hipLaunchKernelGGL(k_actor_prep, dim3(1), dim3(1024), 0, a->stream, L.weight, L.weight_norm, O[l], K[l], Kp,
                           w + a->off_w[l], L.bias, w + a->off_b[l], l < 3 ? 1 : 0);
        if (l >= 4 && L.sigma_w)
            hipLaunchKernelGGL(k_actor_prep, dim3(1), dim3(1024), 0, a->stream, L.sigma_w, (const float*)nullptr, O[l],
                               K[l], Kp, w + a->off_s[l], L.sigma_b, w + a->off_sb[l], 0);
    }
    a->has_s21 = layers[4].sigma_w != nullptr;
    a->has_s31 = layers[5].sigma_w != nullptr;
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        a->err = std::string("measurement actor weight preparation: ") + hipGetErrorString(e);
        return QC_EHIP;
    }
    a->loaded = true;
    return QC_OK;
}

int qc_mactor_act(qc_mactor* a, int64_t B, int64_t env_offset, const float* obs, int32_t noisy, const float* noise,
                  double eps, uint64_t counter, int32_t* actions, float* q_out, int32_t* random_out) {
    if (!a) return QC_EINVAL;
    if (!a->loaded) { a->err = "qc_mactor_load has not been called"; return QC_EINVAL; }
    if (B < 0 || B > a->p.max_batch) { a->err = "B must be in [0, max_batch]"; return QC_EINVAL; }
    if (B == 0) return QC_OK;
    if (!obs || !actions) { a->err = "obs and actions are required"; return QC_EINVAL; }
    Dev g(a->device);
    const int L = a->p.read_length;
    const float* w = a->d_w;
    const int64_t ld = a->p.max_batch;
    for (int64_t c0 = 0; c0 < B; c0 += a->chunk) {   // conv stack per env chunk (its activations stay in L2 / MALL)
        const int64_t nb = std::min<int64_t>(a->chunk, B - c0);
        const int64_t n1 = nb * a->T1, n2 = nb * a->T2, n3 = nb * a->T3;
        hipLaunchKernelGGL((k_mconv<2, 13, 5, 1, kNT1, kNA1, kQ1>), dim3((unsigned)((n1 + 128 * kNT1 - 1) / (128 * kNT1))),
                           dim3(256), 0, a->stream, obs + c0 * 2 * L, L, w + a->off_w[0], w + a->off_b[0], a->d_y1,
                           a->T1, n1);
        hipLaunchKernelGGL((k_mconv<32, 11, 4, 2, kNT2, kNA2, kQ2>), dim3((unsigned)((n2 + 128 * kNT2 - 1) / (128 * kNT2))),
                           dim3(256), 0, a->stream, a->d_y1, a->T1, w + a->off_w[1], w + a->off_b[1], a->d_y2, a->T2,
                           n2);
        hipLaunchKernelGGL((k_mconv<64, 9, 4, 2, kNT3, kNA3, kQ3>), dim3((unsigned)((n3 + 128 * kNT3 - 1) / (128 * kNT3))),
                           dim3(256), 0, a->stream, a->d_y2, a->T2, w + a->off_w[2], w + a->off_b[2], a->d_y3e, a->T3,
                           n3);
        hipLaunchKernelGGL(k_mtr, dim3((unsigned)((a->flat + 63) / 64), (unsigned)((nb + 63) / 64)), dim3(256), 0,
                           a->stream, a->d_y3e, a->d_y3, a->flat, nb, ld, c0);
    }
    {
        constexpr int envs_per_wg = (4 / (8 / kMfcMT)) * kMfcNT * 32;
        hipLaunchKernelGGL((k_mfc<kMfcMT, kMfcNT>), dim3((unsigned)((B + envs_per_wg - 1) / envs_per_wg)), dim3(256), 0,
                           a->stream, a->d_y3, ld, a->flat, w + a->off_w[3], w + a->off_b[3], a->d_h1, B);
    }
    const bool need_noise = noisy && (a->has_s21 || a->has_s31);
    if (need_noise) {
        if (noise) {
            const int64_t n = B * a->noise_len;
            hipLaunchKernelGGL(k_actor_transpose, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, a->stream, noise,
                               a->d_noise, ld, B, a->noise_len);
        } else {
            hipLaunchKernelGGL(k_actor_noise, dim3((unsigned)((B + 255) / 256), (unsigned)((a->noise_len + 1) / 2)),
                               dim3(256), 0, a->stream, a->d_noise, ld, B, a->noise_len, env_offset, a->p.seed, counter);
        }
    }
    ActArgs k{};
    k.L[2].u = w + a->off_w[4];
    k.L[2].ub = w + a->off_b[4];
    k.L[2].s = a->has_s21 ? w + a->off_s[4] : nullptr;
    k.L[2].sb = a->has_s21 ? w + a->off_sb[4] : nullptr;
    k.L[3].u = w + a->off_w[5];
    k.L[3].ub = w + a->off_b[5];
    k.L[3].s = a->has_s31 ? w + a->off_s[5] : nullptr;
    k.L[3].sb = a->has_s31 ? w + a->off_sb[5] : nullptr;
    k.n_act = a->p.n_actions;
    k.B = B;
    k.env_offset = env_offset;
    k.noisy = need_noise ? 1 : 0;
    k.noise = a->d_noise;
    k.noise_ld = ld;
    k.eps = (float)eps;
    k.seed = a->p.seed;
    k.counter = counter;
    k.actions = actions;
    k.q_out = q_out;
    k.random_out = random_out;
    k.h_in = a->d_h1;
    k.h_ld = ld;
    hipLaunchKernelGGL(k_actor_act, dim3((unsigned)((B + kE - 1) / kE)), dim3(kThreads),
                       (2 * kH1 * kE + 16 * 64) * sizeof(float), a->stream, k);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        a->err = std::string("measurement actor launch: ") + hipGetErrorString(e);
        return QC_EHIP;
    }
    return QC_OK;
}

}  // extern "C"
