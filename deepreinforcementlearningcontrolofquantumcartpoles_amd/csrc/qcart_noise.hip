// qcart_noise.hip — the reference's noise stream on the device: one MT19937 per env with MKL's
// Box–Muller Gaussian transform (set_seed / vdRngGaussian, IHO/simulation_i.cpp:574-579, :435).
//
// The reference draws two N(0,1) per go_one_step from a per-process VSL_BRNG_MT19937 stream created by
// vslNewStream(&stream, VSL_BRNG_MT19937, seed), with VSL_RNG_METHOD_GAUSSIAN_BOXMULLER. What that is,
// measured against the MKL 2021.4 runtime in this image (tests/golden/make_mkl_fixtures.py):
//   * the generator is MT19937 (Matsumoto–Nishimura) initialised by init_by_array({seed}, 1) — the
//     uniform bits equal MKL's viRngUniformBits bit for bit;
//   * each normal consumes two consecutive 32-bit outputs, u = bits * 2^-32:
//     x = sqrt(-2 ln u1) * sin(2 pi u2); draws are a plain sequence (vdRngGaussian(n = 2) per step
//     equals one long call), so step k of an env uses normals 2k, 2k+1 = words 4k .. 4k+3;
//   * MKL evaluates ln / sqrt / sin with its reduced-accuracy vector math by default (ISA-dependent:
//     the AVX-512 and AVX2 paths differ by up to 1e-8, both within 5e-8 of the exact formula); under
//     MKL_CBWR=COMPATIBLE it is the formula above to <= 2 ulp, which this kernel (fp64 ocml log / sin)
//     reproduces.
//   * a first word of 0 (u1 = 0, probability 2^-32 per normal) does not give MKL an infinite normal: its
//     Box–Muller returns sqrt(-2 ln u1) = 3.4244955099270222 for it on every code path (a state with a
//     planted zero word loaded by vslLoadStreamM, tests/golden/mkl_v2.npz "zero/*"), so that radius is used.
// The states live in HBM ([B][kMtWords] uint32: 624 words + the read index) and advance only by the
// words an env actually consumes (2 normals per step it takes), exactly as each reference actor's
// stream does.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qcart_kargs.hpp"
#include "qcart_mt.hpp"

namespace qcart {
namespace {

using mt::kM;
using mt::kN;
using mt::temper;
using mt::twist;

// init_by_array({seed}, 1) of mt19937ar.c (the serial part runs on lane 0 over the wave's LDS copy)
// mask (optional, [B]): only envs with mask[e] != 0 are (re)seeded, the others keep their streams
__global__ __launch_bounds__(256) void k_mt_seed(const uint32_t* seeds, const uint8_t* mask, int64_t B, uint32_t* st) {
    __shared__ uint32_t lds[4][kN];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 4 + w;
    if (e >= B) return;
    if (mask && !mask[e]) return;
    uint32_t* mt = lds[w];
    if (lane == 0) {
        const uint32_t key = seeds[e];
        mt[0] = 19650218u;
        for (int i = 1; i < kN; ++i) mt[i] = 1812433253u * (mt[i - 1] ^ (mt[i - 1] >> 30)) + (uint32_t)i;
        int i = 1;
        for (int k = kN; k; --k) {   // j stays 0 (key_length 1): + key[0] + 0
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1664525u)) + key;
            if (++i >= kN) { mt[0] = mt[kN - 1]; i = 1; }
        }
        for (int k = kN - 1; k; --k) {
            mt[i] = (mt[i] ^ ((mt[i - 1] ^ (mt[i - 1] >> 30)) * 1566083941u)) - (uint32_t)i;
            if (++i >= kN) { mt[0] = mt[kN - 1]; i = 1; }
        }
        mt[0] = 0x80000000u;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    uint32_t* g = st + (size_t)e * kMtWords;
    for (int i = lane; i < kN; i += 64) g[i] = mt[i];
    if (lane == 0) g[kN] = kN;   // read index: the first draw twists
}

// One wave per env: the env's min(n_steps, env_steps[e]) steps need 4 words each; normals go to
// noise[k][e][0..1] (the step kernel's injected-noise layout). Steps past the env's budget are left
// untouched (the step kernel never reads them). With `pre` (optional, [B][2]) an env with has_pre[e] != 0 already
// drew its first step's pair into pre[e] (the step server's prefetch): that pair becomes step 0 and only the
// remaining steps draw from the stream.
__global__ __launch_bounds__(256) void k_mt_normals(uint32_t* st, int64_t B, int32_t n_steps, const int32_t* env_steps,
                                                    double* noise, const double* pre, const uint8_t* has_pre) {
    __shared__ uint32_t lds[4][kN + 1];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t e = (int64_t)blockIdx.x * 4 + w;
    if (e >= B) return;
    int n_my = n_steps;
    if (env_steps) {
        const int b = env_steps[e];
        n_my = b < 0 ? 0 : (b < n_my ? b : n_my);
    }
    if (n_my <= 0) return;
    const int s0 = (pre && has_pre[e]) ? 1 : 0;
    if (s0) {
        if (lane < 2) noise[(size_t)e * 2 + lane] = pre[(size_t)e * 2 + lane];
        if (n_my == 1) return;
    }
    uint32_t* mt = lds[w];
    uint32_t* g = st + (size_t)e * kMtWords;
    for (int i = lane; i < kN; i += 64) mt[i] = g[i];
    int idx = (int)g[kN];   // even: words are only ever consumed in pairs
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const int64_t need = 4 * (int64_t)(n_my - s0);
    int64_t done = 0;
    while (done < need) {
        if (idx >= kN) {
            twist(mt, lane);
            idx = 0;
        }
        const int avail = (int)((need - done) < (int64_t)(kN - idx) ? (need - done) : (int64_t)(kN - idx));
        for (int p = lane; p < avail / 2; p += 64) {
            const double x = qcart::mt::boxmuller(temper(mt[idx + 2 * p]), temper(mt[idx + 2 * p + 1]));
            const int64_t n = done / 2 + p + 2 * s0;   // normal index of the env: step n / 2, component n % 2
            noise[((size_t)(n >> 1) * B + e) * 2 + (n & 1)] = x;
        }
        idx += avail;
        done += avail;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (int i = lane; i < kN; i += 64) g[i] = mt[i];
    if (lane == 0) g[kN] = (uint32_t)idx;
}

__global__ __launch_bounds__(256) void k_fill_u64(uint64_t* p, int64_t n, uint64_t v) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) p[i] = v;
}

}  // namespace

int launch_mt_seed(const uint32_t* seeds, const uint8_t* mask, int64_t B, uint32_t* st, void* stream) {
    if (B <= 0) return 0;
    hipLaunchKernelGGL(k_mt_seed, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream, seeds, mask, B, st);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_mt_normals(uint32_t* st, int64_t B, int32_t n_steps, const int32_t* env_steps, double* noise,
                      void* stream, const double* pre, const uint8_t* has_pre) {
    if (B <= 0 || n_steps <= 0) return 0;
    hipLaunchKernelGGL(k_mt_normals, dim3((unsigned)((B + 3) / 4)), dim3(256), 0, (hipStream_t)stream, st, B, n_steps,
                       env_steps, noise, pre, has_pre);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_fill_u64(uint64_t* p, int64_t n, uint64_t v, void* stream) {
    if (n <= 0) return 0;
    hipLaunchKernelGGL(k_fill_u64, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, p, n, v);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace qcart
