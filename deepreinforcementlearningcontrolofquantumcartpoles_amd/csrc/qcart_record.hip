// qcart_record.hip — the measurement-record input mode: the per-env coarse-grained
// measurement history that the reference's 'measurements' input feeds to its network and stores in its
// experience rows (IHO/main_parallel.py:143-151,270-309; HO/main_parallel.py:142-150,259-292).
//
// Per env, in place in HBM (the network input layout np.array([measurements_input[::-1],
// forces_along_measurements_input[::-1]]), float32):
//   hist   [2][L]  channel 0: the last L measurements, newest first; channel 1: force * input_scaling
//                  applied during each of them
//   forces [K+1]   forces_to_store after the control step's append, newest first (K = L / m)
// One control interval of n_steps physics steps adds m = n_steps / coarse_grain measurements, each the
// mean of coarse_grain consecutive q outputs of step() times input_scaling (IHO:284-288). The kernel
// shifts the env's history by m through LDS (one workgroup per env, so the update is in place), and
// optionally writes the experience row [measurements (L + m), forces (K + 1), last_action, reward]
// (IHO:279-283) — the continuous record connecting the two control steps.
#include <hip/hip_runtime.h>

#include "qcart_kargs.hpp"

namespace qcart {

namespace {

constexpr int kRecThreads = 256;

__global__ __launch_bounds__(kRecThreads) void k_record(const RecArgs a) {
    extern __shared__ float lds[];
    const int64_t env = blockIdx.x;
    const int mode = a.mode ? (int)a.mode[env] : 1;
    if (mode == 0) return;   // frozen env: history untouched
    const int L = a.L, m = a.m, K = a.K, cg = a.cg;
    const int tid = threadIdx.x;
    float* hist = a.hist + (size_t)env * 2 * L;
    float* frc = a.forces + (size_t)env * (K + 1);
    float* sh = lds;             // [2][L] previous history
    float* sf = lds + 2 * L;     // [K + 1] previous forces
    const bool fresh = mode == 2;   // a new episode: the reference starts from zero lists (IHO:271-272)
    if (a.vec4) {
        for (int v = tid; v < (2 * L) / 4; v += kRecThreads)
            reinterpret_cast<float4*>(sh)[v] =
                fresh ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<const float4*>(hist)[v];
    } else {
        for (int j = tid; j < 2 * L; j += kRecThreads) sh[j] = fresh ? 0.f : hist[j];
    }
    for (int j = tid; j < K + 1; j += kRecThreads) sf[j] = fresh ? 0.f : frc[j];
    __syncthreads();
    int slot = a.actions ? a.actions[env] : a.default_action;
    // an out-of-range action raises the handle's error word (reported by the next qc_take_errors, like
    // qc_step's) and is clamped so no table is indexed past its end
    if (slot < 0 || slot >= a.n_slots) {
        if (tid == 0 && a.bad) a.bad[0] = 1;
        slot = slot < 0 ? 0 : a.n_slots - 1;
    }
    const double f = a.slot_force[slot];
    const float fs = (float)(f * a.scaling);   // force * args.input_scaling (IHO:266, :288)
    const int64_t B = a.B;
    // channel 0 / 1 element j of the new history
    auto meas = [&](int j) -> float {
        const int t = m - 1 - j;   // t-th measurement of this interval (newest first in the history)
        double s = 0.0;            // sum(measurements_cache) / coarse_grain * input_scaling
        for (int u = 0; u < cg; ++u) s += a.q[(size_t)(t * cg + u) * B + env];
        return (float)(s / cg * a.scaling);
    };
    float* row = a.rows ? a.rows + (size_t)env * a.row_len : nullptr;
    if (a.vec4) {
        for (int v = tid; v < (2 * L) / 4; v += kRecThreads) {
            const int j0 = 4 * v;
            const int c = j0 >= L ? 1 : 0, j = j0 - c * L;
            float4 o;
            if (j >= m) {
                o = reinterpret_cast<const float4*>(sh)[(c * L + j - m) / 4];
            } else {
                o.x = c ? fs : meas(j);
                o.y = c ? fs : meas(j + 1);
                o.z = c ? fs : meas(j + 2);
                o.w = c ? fs : meas(j + 3);
            }
            reinterpret_cast<float4*>(hist)[v] = o;
            if (row && c == 0) {   // rows are L + m + K + 3 floats: not 16-B aligned in general
                row[j0] = o.x;
                row[j0 + 1] = o.y;
                row[j0 + 2] = o.z;
                row[j0 + 3] = o.w;
            }
        }
        if (row)
            for (int j = tid; j < m; j += kRecThreads) row[L + j] = sh[L - m + j];
    } else {
        for (int i = tid; i < 2 * L; i += kRecThreads) {
            const int c = i >= L ? 1 : 0, j = i - c * L;
            const float o = j >= m ? sh[c * L + j - m] : (c ? fs : meas(j));
            hist[i] = o;
            if (row && c == 0) row[j] = o;
        }
        if (row)
            for (int j = tid; j < m; j += kRecThreads) row[L + j] = sh[L - m + j];
    }
    for (int i = tid; i < K + 1; i += kRecThreads) {
        const float o = i == 0 ? fs : sf[i - 1];
        frc[i] = o;
        if (row) row[L + m + i] = o;
    }
    if (row && tid == 0) {
        row[L + m + K + 1] = (float)slot;   // np.array([last_action], dtype=np.float32)
        if (a.reward) row[L + m + K + 2] = a.reward[env];
    }
}

// get_data_wavefunction (IHO/main_parallel.py:133-135: hstack(Re state[:-20], Im state[:-20]); IQO/QO
// main_parallel.py:136-137: state[10:-10]) * input_scaling, in float32 like the reference's
// float32 array times a Python float: out [B][2 * cnt]
template <typename RT>
__global__ __launch_bounds__(256) void k_wavefunction(const RT* psi, int64_t B, int32_t N, int32_t lo, int32_t cnt,
                                                      float scaling, float* out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= B * 2 * (int64_t)cnt) return;
    const int64_t env = i / (2 * cnt);
    const int j = (int)(i - env * 2 * cnt);
    const int c = j >= cnt ? 1 : 0, r = lo + j - c * cnt;
    out[i] = (float)psi[((size_t)env * N + r) * 2 + c] * scaling;
}

}  // namespace

int launch_wavefunction(const void* psi, int precision, int64_t B, int32_t N, int32_t lo, int32_t cnt, double scaling,
                        float* out, void* stream) {
    const int64_t n = B * 2 * (int64_t)cnt;
    if (n <= 0) return 0;
    const dim3 g((unsigned)((n + 255) / 256));
    if (precision == 1)
        hipLaunchKernelGGL(k_wavefunction<float>, g, dim3(256), 0, (hipStream_t)stream, (const float*)psi, B, N, lo, cnt,
                           (float)scaling, out);
    else
        hipLaunchKernelGGL(k_wavefunction<double>, g, dim3(256), 0, (hipStream_t)stream, (const double*)psi, B, N, lo,
                           cnt, (float)scaling, out);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

int launch_record(const RecArgs& a, void* stream) {
    if (a.B <= 0) return 0;
    const size_t lds = sizeof(float) * (size_t)(2 * a.L + a.K + 1);
    static bool attr_set = false;
    if (!attr_set) {
        if (hipFuncSetAttribute((const void*)k_record, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) !=
            hipSuccess)
            return -3;
        attr_set = true;
    }
    hipLaunchKernelGGL(k_record, dim3((unsigned)a.B), dim3(kRecThreads), lds, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace qcart
