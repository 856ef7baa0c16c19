// qcart_expt.hpp — diagnostic hooks of the step kernel, compiled out of the shipped library.
//
// -DQCART_STAMPS (a diagnostic build only, tools/diag_stamps.py): per-phase cycle shares of the step loop
// (s_memtime at each QC_STAMP(phase) site of qcart_kernels.hpp), summed over all waves into qc_stamps[] and
// read back by qc_debug_stamps. Without it every hook below expands to nothing.
#pragma once
#include <hip/hip_runtime.h>

#ifdef QCART_STAMPS
namespace qcart {
__device__ unsigned long long qc_stamps[16];
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
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_t)::"memory")
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
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(qcart::qc_stamps), sizeof(unsigned long long) * 16) != hipSuccess) return -1;
    unsigned long long z[16] = {0};
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
#define QC_SOLVE_STAMP_ARGS
#define QC_SOLVE_STAMP_PASS
#endif
