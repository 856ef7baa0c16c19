// qcart_expt.hpp — diagnostic hooks of the step kernel, compiled out of the shipped library.
//
// -DQCART_STAMPS (a diagnostic build only, tools/diag_stamps.py): per-phase cycle shares of the step loop
// (s_memtime at each QC_STAMP(phase) site of qcart_kernels.hpp), summed over all waves into qc_stamps[] and
// read back by qc_debug_stamps. Without it every hook below expands to nothing.
//
// Experiment knobs: compile-time defaults of the shipped build that an experiment build (make expt / expt_actor
// EXPT=-D...) overrides for an A/B. Each default is the measured winner.
#pragma once
#include <hip/hip_runtime.h>

// step kernel: the largest rows-per-lane R (fp64-equivalent) that runs 8-wave workgroups (two waves per SIMD),
// Fock families / grid
#ifndef QCART_W8_MAX_R
#define QCART_W8_MAX_R 8
#endif
#ifndef QCART_W8_MAX_RG
#define QCART_W8_MAX_RG 9
#endif
// grid step kernels up to R = 9: the host-folded step constants of the Fock kernels (HC; round 6, alternating
// same-call pairs: C4 9.09 -> 8.91 ms; C3's R = 17 kernel with them, 150.2 -> 149.0 ms, computed wrong values, k_step
// comment). QCART_GRID_KAR: the per-step kernarg re-read for R = 17 too (A/B knob; with HC: C3's spilled SGPRs
// 260 -> 109, 151.2 vs 149.8 ms against the shipped kernel)
#ifndef QCART_GRID_HC
#define QCART_GRID_HC 1
#endif
#ifndef QCART_GRID_KAR
#define QCART_GRID_KAR 0
#endif
// band solve: the fp32 Fock kernels' whole-wave Kogge-Stone (no row carry) for up to this many kept levels (0: off;
// 3: C5 -1.6 %)
#ifndef QCART_WKS_F32
#define QCART_WKS_F32 3
#endif
// step kernel: the fp32 R = 32 kernel's Y+- means in two reductions (1; C5 46.7 -> 43.2 ms) or one (0)
#ifndef QCART_SPLITM
#define QCART_SPLITM 1
#endif
// step kernel: the 64-step noise refill parked in a 1 KiB per-wave LDS buffer, read back one step at a time (1), or
// held in 4 VGPRs across the step loop (0) — fp64 kernels with LDS tables (MODE >= 1)
#ifndef QCART_NZ_LDS
#define QCART_NZ_LDS 1
#endif
// measurement actor (qcart_actor.hip): conv1..3 column tiles per wave, accumulator sets, k-steps per load batch;
// fc1 output tiles x env tiles per wave
#ifndef QCART_MCONV_NT
#define QCART_MCONV_NT 2, 2, 1
#endif
#ifndef QCART_MCONV_NA
#define QCART_MCONV_NA 2, 1, 2
#endif
#ifndef QCART_MCONV_Q
#define QCART_MCONV_Q 4, 4, 4
#endif
#ifndef QCART_MFC_MT
#define QCART_MFC_MT 2
#endif
#ifndef QCART_MFC_NT
#define QCART_MFC_NT 2
#endif

#ifdef QCART_STAMPS
namespace qcart {
__device__ unsigned long long qc_stamps[20];
}
#define QC_STAMP(ph)                                                                                 \
    do {                                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                                           \
        unsigned long long t_;                                                                       \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                   \
        __builtin_amdgcn_sched_barrier(0);                                                           \
        st_acc[st_ph] += t_ - st_t;                                                                  \
        st_t = t_;                                                                                   \
        st_ph = (ph);                                                                                \
    } while (0)
// the step kernel's stamp state, declared before its loop and flushed after it
#define QC_STAMP_BEGIN()                                                                             \
    unsigned long long st_acc[16] = {0}, st_t = 0;                                                   \
    int st_ph = 9;                                                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t)::"memory");                     \
    const unsigned long long st_loop0 = st_t
// wave entry (k_step) and exit (after the write-back): slots 16 (entry -> loop), 17 (loop end -> exit),
// 18 (wave count)
#define QC_KSTAMP_ENTRY()                                                                            \
    unsigned long long kst_t0;                                                                       \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(kst_t0)::"memory")
#define QC_KSTAMP_EXIT(lane)                                                                         \
    do {                                                                                             \
        unsigned long long t_;                                                                       \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                   \
        if ((lane) == 0) {                                                                           \
            atomicAdd(&qc_stamps[16], st_loop0 - kst_t0);                                            \
            atomicAdd(&qc_stamps[17], t_ - st_t);                                                    \
            atomicAdd(&qc_stamps[18], 1ull);                                                         \
        }                                                                                            \
    } while (0)
#define QC_STAMP_END(lane)                                                                           \
    do {                                                                                             \
        QC_STAMP(9);                                                                                 \
        if ((lane) == 0)                                                                             \
            for (int i_ = 0; i_ < 16; ++i_) atomicAdd(&qc_stamps[i_], st_acc[i_]);                   \
    } while (0)
// the band solve's stamps use the caller's state
#define QC_SOLVE_STAMP_ARGS , unsigned long long (&st_acc)[16], unsigned long long& st_t, int& st_ph
#define QC_SOLVE_STAMP_PASS , st_acc, st_t, st_ph

// read and clear the per-phase cycle sums (weak: an experiment build stamps one family TU)
extern "C" __attribute__((weak)) int qc_debug_stamps(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(qcart::qc_stamps), sizeof(unsigned long long) * 20) != hipSuccess) return -1;
    unsigned long long z[20] = {0};
    return hipMemcpyToSymbol(HIP_SYMBOL(qcart::qc_stamps), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#else
#define QC_STAMP(ph) \
    do {             \
    } while (0)
#define QC_STAMP_BEGIN() \
    do {                 \
    } while (0)
#define QC_STAMP_END(lane) \
    do {                   \
    } while (0)
#define QC_KSTAMP_ENTRY() \
    do {                  \
    } while (0)
#define QC_KSTAMP_EXIT(lane) \
    do {                     \
    } while (0)
#define QC_SOLVE_STAMP_ARGS
#define QC_SOLVE_STAMP_PASS
#endif

// the fp32 R = 32 kernel's mirror bands read in pipelined half-band batches (k_step MPIPE; A/B)
#ifndef QCART_MPIPE
#define QCART_MPIPE 1
#endif
#ifndef QCART_MPIPE_ROWS
#define QCART_MPIPE_ROWS 16
#endif
#ifndef QCART_MPIPE_DEPTH
#define QCART_MPIPE_DEPTH 2
#endif

// -DQCART_RES_STAMPS (a diagnostic build only, tools/probe_resident_lat.py --stamps): the resident kernel sums, per
// slot, the s_memrealtime ticks (10 ns) of its request phases — acquire, the pair, the step, the results + release —
// into the slot's err bytes (unused by the resident path) as 5 uint64: count, then the four sums
#ifndef QCART_RES_STAMPS
#define QCART_RES_STAMPS 0
#endif
