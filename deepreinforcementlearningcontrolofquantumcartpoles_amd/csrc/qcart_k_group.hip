// qcart_k_group.hip — groups the envs of a step call by force slot so that each workgroup of
// the step kernel shares one slot's factor tables through LDS. One workgroup: LDS histogram of the
// slots, group offsets, then a scatter of env ids (order inside a group is arbitrary and does not affect
// any result: envs are independent). Unused entries are -1 (idle waves). Without order_mixed every slot's
// group is padded to whole workgroups; with it (step kernels with two-slot blocks, k_step DUAL) the slots
// of >= g envs are packed back to back, so the batch fills ceil(B / g) workgroups plus only the small
// slots' padding, and the few workgroups that straddle two slots run with both slots' tables in LDS. Envs with no step budget this call (env_steps[e] <= 0: the reset intervals of a partly
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
                                                int32_t* __restrict__ bad, int32_t* __restrict__ order_mixed) {
    __shared__ int cnt[kBuckets], off[kBuckets], cur[kBuckets];
    // the packed region (order_mixed given): slots with >= g envs back to back, in slot order
    __shared__ int start[kBuckets];      // first position of a packed slot (-1: padded on its own)
    __shared__ int head_mix[kBuckets];   // two-slot workgroup index of the workgroup holding start[s], or -1
    __shared__ int nmix_le[kBuckets];    // two-slot workgroups whose second slot is <= s
    __shared__ int next_big[kBuckets];   // the next packed slot (-1: none)
    __shared__ int total, packed_end, n_mix, last_big;
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
        // packed slots (>= g envs each): laid out back to back and cut every g envs, so a workgroup holds
        // at most one slot boundary — i.e. at most two slots. A workgroup with a boundary strictly inside
        // is a two-slot workgroup (order_mixed), every other one a single-slot workgroup (order)
        int C = 0, nm = 0, prev = -1;
        for (int s = 0; s < kBuckets; ++s) {
            start[s] = -1;
            head_mix[s] = -1;
            next_big[s] = -1;
        }
        for (int s = 0; s < n_slots; ++s) {
            if (!order_mixed || cnt[s] < g) continue;
            start[s] = C;
            if (prev >= 0) {
                next_big[prev] = s;
                if (C % g != 0) head_mix[s] = nm++;
            }
            nmix_le[s] = nm;
            prev = s;
            C += cnt[s];
        }
        last_big = prev;
        packed_end = C;
        n_mix = nm;
        // single-slot workgroups: the packed region's (its workgroups minus the two-slot ones), then the
        // padded groups of the other slots and of the no-budget bucket
        int o = ((C + g - 1) / g - nm) * g;
        for (int s = 0; s < kBuckets; ++s) {
            if (start[s] >= 0) continue;
            off[s] = o;
            o += (cnt[s] + g - 1) / g * g;
        }
        total = o;
    }
    __syncthreads();
    // position p of the packed region -> its slot in order / order_mixed (s: the slot owning p, or the last
    // packed slot for the padding past the region's end)
    auto packed_dst = [&](int s, int p) -> int32_t* {
        const int G = p / g, s2 = next_big[s];
        if (head_mix[s] >= 0 && G == start[s] / g) return order_mixed + head_mix[s] * g + p % g;
        if (s2 >= 0 && head_mix[s2] >= 0 && G == start[s2] / g) return order_mixed + head_mix[s2] * g + p % g;
        return order + (G - nmix_le[s]) * g + p % g;
    };
    for (int64_t e = t; e < B; e += blockDim.x) {
        const int s = slot_of(e);
        const int k = atomicAdd(&cur[s], 1);
        if (start[s] >= 0) *packed_dst(s, start[s] + k) = (int32_t)e;
        else order[off[s] + k] = (int32_t)e;
    }
    if (t < kBuckets && start[t] < 0)
        for (int p = cnt[t]; p < (cnt[t] + g - 1) / g * g; ++p) order[off[t] + p] = -1;
    if (last_big >= 0)   // the packed region's last, partial workgroup
        for (int p = packed_end + t; p < (packed_end + g - 1) / g * g; p += blockDim.x) *packed_dst(last_big, p) = -1;
    for (int i = total + t; i < cap; i += blockDim.x) order[i] = -1;
    if (order_mixed) {
        for (int i = n_mix * g + t; i < n_slots * g; i += blockDim.x) order_mixed[i] = -1;
        if (t == 0) order_mixed[n_slots * g] = n_mix;   // k_step DUAL: the two-slot blocks come first
    }
}

int launch_group(const int32_t* actions, int32_t default_action, const int32_t* env_steps, int32_t n_steps, int64_t B,
                 int n_slots, int gran, int32_t* order, int32_t cap, int32_t* bad, int32_t* order_mixed, void* stream) {
    if (n_slots > kGroupSlots || gran < 1 ||
        (int64_t)cap < (B + gran - 1) / gran * gran + (int64_t)(gran - 1) * (n_slots + 1))
        return -1;
    hipLaunchKernelGGL(k_group, dim3(1), dim3(1024), 0, (hipStream_t)stream, actions, default_action, env_steps, n_steps,
                       B, n_slots, gran, order, cap, bad, order_mixed);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace qcart
