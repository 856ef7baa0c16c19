// qcart_mt.hpp — the reference's noise stream on the device, shared by the MT19937 kernels (qcart_noise.hip) and
// the step server's resident kernel (k_resident, qcart_kernels.hpp): MT19937 (mt19937ar.c) tempering and the
// in-LDS generation twist, and MKL's Box–Muller normal of two words (vdRngGaussian BOXMULLER, the reference's
// IHO/simulation_i.cpp:435, :574-579). What MKL does exactly is pinned in qcart_noise.hip's header.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qcart {
namespace mt {

constexpr int kN = 624, kM = 397;
constexpr double kMklZeroWordRadius = 3.4244955099270222;   // MKL 2021.4 BOXMULLER at u1 = 0

__device__ __forceinline__ uint32_t temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// the generation twist of mt19937ar.c over a wave's LDS state, in 64-lane chunks of increasing k: a
// chunk reads mt[k], mt[k+1], mt[(k+397) % 624] before any lane of it writes, and everything it reads
// is exactly what the serial loop would see (old above the chunk, already-new (k+397) % 624 < k)
__device__ __forceinline__ void twist(uint32_t* mt, int lane) {
    for (int c = 0; c < kN; c += 64) {
        const int k = c + lane;
        uint32_t v = 0;
        if (k < kN) {
            const uint32_t y = (mt[k] & 0x80000000u) | (mt[k + 1 == kN ? 0 : k + 1] & 0x7fffffffu);
            const int m = k + kM < kN ? k + kM : k + kM - kN;
            v = mt[m] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        if (k < kN) mt[k] = v;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// one N(0, 1) from two consecutive tempered words, u = bits * 2^-32: sqrt(-2 ln u1) sin(2 pi u2); a zero first word
// gives MKL's finite radius, not inf (tests/golden/mkl_v2.npz "zero/*")
__device__ __forceinline__ double boxmuller(uint32_t w1, uint32_t w2) {
    // contraction as in qcart_noise.hip whatever the including TU's mode (the grid TU's fast-honor-pragmas)
#pragma clang fp contract(on)
    const double u1 = (double)w1 * 0x1.0p-32;
    const double u2 = (double)w2 * 0x1.0p-32;
    const double rad = w1 ? sqrt(-2.0 * log(u1)) : kMklZeroWordRadius;
    return rad * sin(6.283185307179586 * u2);
}

}  // namespace mt
}  // namespace qcart
