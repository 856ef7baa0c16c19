// qcart_env.hip — the batched episode loop's per-control-step bookkeeping (BatchedEnv, reset="deferred") in one
// kernel, so that PyTorch only holds the tensors: the cartpoles' termination, reward and return accounting of
// Control.do_episode (IHO/main_parallel.py:242-268, IQO/main_parallel.py:190-221) for every env of the batch,
// and the append of the finished episodes (return, length) to a device ring in env order (the reference's
// per-actor result queue, IHO/main_parallel.py:300-327) — no host synchronisation.
//
// Per env e, after a step call of one control interval:
//   * pending[e] set: this call was env e's reset interval (|0> / the IQO packet at F = 0, the zero-th step
//     without control, IHO:231-232, :250): its episode time restarts at one interval, its return at 0, no
//     transition is valid; an episode already over at that first control step (Fail or out of bounds) is
//     reported with return 0 and restarts again in the next call (the i != control_interval guard, IHO:250,
//     and the queue puts, IHO:312-313);
//   * otherwise: t += interval dt, done = Fail during the interval (numerical_failure, IHO:243-247) or out of
//     bounds (IHO |<x>| > xth, IHO:246; IQO the outside probability passed 0.5 at some physics step,
//     IQO:199-200); reward = failing_reward when done else 1, every transition valid, return += reward; a done
//     env is reported (return, t) and resets in the next call.
// One workgroup walks the batch in chunks of its 1024 threads, a workgroup scan per chunk placing the finished
// episodes of the chunk after the previous ones (env order, deterministic).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qcart_kargs.hpp"

namespace qcart {
namespace {

constexpr int kTailThreads = 1024;

__global__ __launch_bounds__(kTailThreads) void k_env_tail(const EnvTailArgs a) {
    __shared__ int32_t wsum[kTailThreads / 64];
    __shared__ int64_t base;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    if (t == 0) base = *a.fin_n;
    __syncthreads();
    const double ci_dt = (double)a.interval * a.dt;
    for (int64_t c0 = 0; c0 < a.B; c0 += kTailThreads) {
        const int64_t e = c0 + t;
        int fin = 0;
        double f_ret = 0.0, f_len = 0.0;
        if (e < a.B) {
            const bool pend = a.pending[e] != 0;
            const bool fail = a.fail_step[e] > 0;
            const bool oob = a.kind == 3 ? (a.term_step[e] >= 0) : (fabs(a.obs[(size_t)e * a.n_obs]) > a.xth);
            const bool over = fail || oob;
            if (a.obs32)
                for (int i = 0; i < a.n_obs; ++i)
                    a.obs32[(size_t)e * a.n_obs + i] = (float)a.obs[(size_t)e * a.n_obs + i] * (float)a.input_scaling;
            double tt, ret;
            float rw;
            if (pend) {
                tt = ci_dt;
                ret = 0.0;
                rw = 0.0f;
                a.steps[e] = a.interval;
                a.valid[e] = 0;
            } else {
                tt = a.t[e] + ci_dt;
                rw = over ? (float)a.failing_reward : 1.0f;
                // the return accumulates the float64 reward values, as BatchedEnv's immediate mode does
                ret = a.episode_return[e] + (over ? a.failing_reward : 1.0);
                a.steps[e] += a.interval;
                a.valid[e] = 1;
            }
            a.t[e] = tt;
            a.episode_return[e] = ret;
            a.reward[e] = rw;
            a.done[e] = over ? 1 : 0;
            a.pending[e] = over ? 1 : 0;
            fin = over ? 1 : 0;
            f_ret = ret;
            f_len = tt;
        }
        // workgroup exclusive scan of fin (wave ballot + per-wave counts)
        const uint64_t m = __ballot(fin);
        const int before = __popcll(m & ((1ull << lane) - 1ull));
        if (lane == 63) wsum[w] = __popcll(m);
        __syncthreads();
        int woff = 0, tot = 0;
        for (int i = 0; i < kTailThreads / 64; ++i) {
            const int v = wsum[i];
            woff += i < w ? v : 0;
            tot += v;
        }
        if (fin) {
            const int64_t pos = (base + woff + before) % a.fin_cap;
            a.fin[pos] = f_ret;
            a.fin[a.fin_cap + 1 + pos] = f_len;
        }
        __syncthreads();
        if (t == 0) base += tot;
        __syncthreads();
    }
    if (t == 0) *a.fin_n = base;
}

}  // namespace

int launch_env_tail(const EnvTailArgs& a, void* stream) {
    if (a.B <= 0) return 0;
    hipLaunchKernelGGL(k_env_tail, dim3(1), dim3(kTailThreads), 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace qcart
