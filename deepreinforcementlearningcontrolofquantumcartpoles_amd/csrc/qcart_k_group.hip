// qcart_k_group.hip — groups the envs of a step call by force slot so that each workgroup of
// the step kernel shares one slot's factor tables through LDS. One workgroup: LDS histogram of the
// slots, group offsets padded to whole workgroups, then a scatter of env ids (order inside a group is
// arbitrary and does not affect any result: envs are independent). Unused entries are -1 (idle
// waves). Envs with no step budget this call (env_steps[e] <= 0: the reset intervals of a partly
// finished batch) go to a last bucket of their own, so they never stretch a working workgroup.
// An out-of-range action of an env with a step budget raises the handle's error word (bad): the step kernel
// clamps it, and the host reports it at its next check (qc_take_errors) instead of syncing on every call.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "qcart_kargs.hpp"

namespace qcart {

constexpr int kGroupSlots = 64;
constexpr int kBuckets = kGroupSlots + 1;   // + the no-budget bucket (last)

__global__ __launch_bounds__(1024) void k_group(const int32_t* __restrict__ actions, int32_t default_action,
                                                const int32_t* __restrict__ env_steps, int32_t n_steps, int64_t B,
                                                int n_slots, int g, int32_t* __restrict__ order, int32_t cap,
                                                int32_t* __restrict__ bad) {
    __shared__ int cnt[kBuckets], off[kBuckets], cur[kBuckets];
    __shared__ int total;
    const int t = threadIdx.x;
    if (t < kBuckets) {
        cnt[t] = 0;
        cur[t] = 0;
    }
    __syncthreads();
    auto slot_of = [&](int64_t e) {
        if (env_steps && (env_steps[e] <= 0 || n_steps <= 0)) return kGroupSlots;
        const int s = actions ? actions[e] : default_action;
        return s < 0 ? 0 : (s >= n_slots ? n_slots - 1 : s);
    };
    for (int64_t e = t; e < B; e += blockDim.x) {
        const int s = slot_of(e);
        if (actions && s != kGroupSlots && (actions[e] < 0 || actions[e] >= n_slots)) bad[0] = 1;
        atomicAdd(&cnt[s], 1);
    }
    __syncthreads();
    if (t == 0) {
        int o = 0;
        for (int s = 0; s < kBuckets; ++s) {
            off[s] = o;
            o += (cnt[s] + g - 1) / g * g;
        }
        total = o;
    }
    __syncthreads();
    for (int64_t e = t; e < B; e += blockDim.x) {
        const int s = slot_of(e);
        order[off[s] + atomicAdd(&cur[s], 1)] = (int32_t)e;
    }
    if (t < kBuckets)
        for (int p = cnt[t]; p < (cnt[t] + g - 1) / g * g; ++p) order[off[t] + p] = -1;
    for (int i = total + t; i < cap; i += blockDim.x) order[i] = -1;
}

int launch_group(const int32_t* actions, int32_t default_action, const int32_t* env_steps, int32_t n_steps, int64_t B,
                 int n_slots, int gran, int32_t* order, int32_t cap, int32_t* bad, void* stream) {
    if (n_slots > kGroupSlots || gran < 1 ||
        (int64_t)cap < (B + gran - 1) / gran * gran + (int64_t)(gran - 1) * (n_slots + 1))
        return -1;
    hipLaunchKernelGGL(k_group, dim3(1), dim3(1024), 0, (hipStream_t)stream, actions, default_action, env_steps, n_steps,
                       B, n_slots, gran, order, cap, bad);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace qcart
