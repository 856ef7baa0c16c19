// qcart_replay.hip — prioritized experience replay on the device: the reference's
// SumTree + Memory (inverted harmonic oscillator/RL.py:234-475) for a whole batch of transitions per call,
// resident in HBM next to the environments, so the experience rows never leave the GPU.
//
// Layout (the reference's, RL.py:241-257): tree = float64 [n_nodes + capacity], heap-indexed
// (children 2i+1, 2i+2; n_nodes = 1 + 2 + ... over the widths < capacity; leaf of slot d at n_nodes + d);
// data = float32 [capacity][row_len]. Every parent equals left + right exactly, as the reference's
// compiled_update recomputes it (RL.py:303-310), so path updates here and the reference's one-by-one
// updates give the same bits.
// Batched semantics:
//   store  (Memory.store x k, RL.py:417-420 / SumTree.add :273-288): the valid rows in index order;
//          'sequential' adds while passes < 1 (passes += 1 / capacity each), then random positions
//          (random.randrange -> Philox4x32-10); a slot written twice in one call keeps the later row.
//   sample (compiled_sampling :449-469): stratified v = (i + u_i) total / n, tree descent
//          (compiled_get_leaf :334-364), IS weight (p / (total / len))^-beta.
//   update (Memory.batch_update :438-446 / compiled_batch_update :471-475): p = min(e + eps, upper)^alpha
//          in float32 as numpy computes it, eps = 1e-5 max, max <- 0.95 max(max, max clipped);
//          a leaf listed twice keeps the later error.
// Scalars that depend on device data (pointer, length, passes, max) live in device memory; the host
// never synchronises inside store / sample / update.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/qcart.h"
#include "qcart_kernels.hpp"

namespace qcart {
namespace replay {

struct State {
    int64_t ptr;        // SumTree.data_pointer
    int64_t len;        // SumTree.len
    double passes;      // SumTree.passes
    double max;         // Memory.max
    uint64_t rand_ctr;  // Philox counter of the random-policy positions
    uint64_t epoch;     // store-call counter (owner tags)
    double p_new;       // priority of this store call's rows
    int32_t k;          // this call: rows stored
    int32_t n_seq;      // this call: sequential adds
    int32_t n_leaf;     // this call: leaves whose paths need recomputing
    int32_t pad;
};

constexpr int kPlanThreads = 1024;

__device__ __forceinline__ double u53(uint64_t seed, uint64_t ctr, uint32_t i, uint32_t tag) {
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), i, tag};
    philox10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    return (double)(((((uint64_t)c[0]) << 32) | c[1]) >> 11) * 0x1.0p-53;
}

// SumTree.add's `passes += 1./capacity` for up to k sequential adds while passes < 1 (RL.py:274-280),
// bit-exact and without k dependent additions: inside one binade of p (grid spacing u) every addition
// of inc rounds the same way, so p moves by a constant d = fl(p + inc) - p; runs of such adds are
// jumped in closed form (p + m d is exact), and the adds next to a binade edge, a sign change, zero or
// a round-half-even tie (d1 != d2) are done one at a time. Returns the number of adds made.
__device__ int advance_passes(double& p, double inc, int k) {
    int j = 0;
    while (j < k && p < 1.0) {
        const double q1 = p + inc, q2 = q1 + inc;
        const double d1 = q1 - p, d2 = q2 - q1;
        int e0, e1, e2;
        (void)frexp(p, &e0);
        (void)frexp(q1, &e1);
        (void)frexp(q2, &e2);
        if (d1 == 0.0) return k;   // inc below half an ulp: passes never moves again
        const bool uniform = p != 0.0 && q1 != 0.0 && d1 == d2 && e0 == e1 && e1 == e2 && ((p < 0) == (q2 < 0));
        if (!uniform || k - j < 4) {
            p = q1;
            ++j;
            continue;
        }
        const double u = ldexp(1.0, e0 - 53);   // grid spacing of the binade [2^(e0-1), 2^e0)
        // step i (from p + i d1) is uniform while the exact sum stays a grid step inside the binade
        const double lim = p > 0 ? ldexp(1.0, e0) - u - d1 : -ldexp(1.0, e0 - 1) - u - d1;
        double m = floor((lim - p) / d1);
        if (m < 1.0) {
            p = q1;
            ++j;
            continue;
        }
        m = fmin(m, (double)(k - j));
        while (m > 1.0 && p + m * d1 > lim) m -= 1.0;
        p += m * d1;
        j += (int)m;
    }
    return j;
}

struct PlanArgs {
    State* st;
    const uint8_t* valid;   // [n] or null
    int64_t n, cap;
    int32_t* src;           // [n] rank -> source row
    int64_t* dest;          // [n] rank -> slot
    unsigned long long* owner;   // [cap] (epoch << 32 | rank) of the last writer
    int policy_seq;
    double abs_err_upper;
    uint64_t seed;
};

// one workgroup: order-preserving compaction of the valid rows, the policy decisions, the owner tags
__global__ __launch_bounds__(kPlanThreads) void k_plan(const PlanArgs a) {
    __shared__ int wsum[kPlanThreads / 64];
    __shared__ int carry;
    __shared__ State s0;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (int64_t base = 0; base < a.n; base += kPlanThreads) {
        const int64_t j = base + tid;
        const bool f = j < a.n && (!a.valid || a.valid[j]);
        const uint64_t bal = __ballot(f);
        const int below = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wsum[wv] = __popcll(bal);
        __syncthreads();
        int off = carry;
        for (int w = 0; w < wv; ++w) off += wsum[w];
        if (f) a.src[off + below] = (int32_t)j;
        __syncthreads();
        if (tid == 0) {
            int t = 0;
            for (int w = 0; w < kPlanThreads / 64; ++w) t += wsum[w];
            carry += t;
        }
        __syncthreads();
    }
    if (tid == 0) {
        State s = *a.st;
        const int k = carry;
        int n_seq = k;
        if (!a.policy_seq)   // SumTree.add: sequential while passes < 1, passes += 1 / capacity per add
            n_seq = advance_passes(s.passes, 1.0 / (double)a.cap, k);
        s.p_new = s.max == 0.0 ? a.abs_err_upper : s.max;   // Memory.store (RL.py:418-420)
        s.k = k;
        s.n_seq = n_seq;
        s.n_leaf = k;
        s.epoch += 1;
        s0 = s;   // ptr / len / rand_ctr as before this call
        State e = s;
        e.ptr = (s.ptr + n_seq) % a.cap;
        e.len = std::min<int64_t>(s.len + n_seq, a.cap);
        e.rand_ctr = s.rand_ctr + (uint64_t)(k - n_seq);
        *a.st = e;
    }
    __syncthreads();
    const State s = s0;
    for (int r = tid; r < s.k; r += kPlanThreads) {
        int64_t d;
        if (r < s.n_seq) d = (s.ptr + r) % a.cap;
        else d = (int64_t)(u53(a.seed, s.rand_ctr + (uint64_t)(r - s.n_seq), 0u, 0x200u) * (double)a.cap);
        if (d >= a.cap) d = a.cap - 1;
        a.dest[r] = d;
        atomicMax(&a.owner[d], (unsigned long long)(s.epoch << 32) | (unsigned long long)r);
    }
}

struct CopyArgs {
    const State* st;
    const int32_t* src;
    const int64_t* dest;
    const unsigned long long* owner;
    float* data;
    double* tree;
    int64_t n_nodes;
    int32_t row_len;
    // row source: rows [n][row_len], or the 'xp' parts [last_obs (d), obs (d), action, reward]
    const float* rows;
    const float* last_obs;
    const float* obs;
    const int32_t* action;
    const float* reward;
    int32_t d;
    int64_t n;
};

// one workgroup per stored row (grid = n; ranks >= k exit): the row copy and its leaf priority
__global__ __launch_bounds__(256) void k_copy(const CopyArgs a) {
    const int r = blockIdx.x;
    const State& s = *a.st;
    if (r >= s.k) return;
    const int64_t d = a.dest[r];
    if (a.owner[d] != ((unsigned long long)(s.epoch << 32) | (unsigned long long)r)) return;   // overwritten later
    const int64_t j = a.src[r];
    float* out = a.data + d * (int64_t)a.row_len;
    if (a.rows) {
        const float* in = a.rows + j * (int64_t)a.row_len;
        for (int c = threadIdx.x; c < a.row_len; c += 256) out[c] = in[c];
    } else {
        const int dd = a.d;
        for (int c = threadIdx.x; c < a.row_len; c += 256) {
            float v;
            if (c < dd) v = a.last_obs[j * dd + c];
            else if (c < 2 * dd) v = a.obs[j * dd + c - dd];
            else if (c == 2 * dd) v = (float)a.action[j];
            else v = a.reward[j];
            out[c] = v;
        }
    }
    if (threadIdx.x == 0) a.tree[a.n_nodes + d] = s.p_new;
}

// one tree level of the path updates: the ancestor `up` levels above each listed leaf becomes
// left + right (children beyond the array count 0, as in recalculate_structure, RL.py:320-331)
__global__ __launch_bounds__(256) void k_level(const State* st, const int64_t* leaf_slot, int64_t n_nodes,
                                               int64_t tree_size, double* tree, int up, int64_t n) {
    const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (r >= n || r >= st->n_leaf || leaf_slot[r] < 0) return;   // < 0: a rejected update index
    int64_t node = n_nodes + leaf_slot[r];
    for (int u = 0; u < up; ++u) node = (node - 1) / 2;
    const int64_t cl = 2 * node + 1, cr = cl + 1;
    const double left = cl < tree_size ? tree[cl] : 0.0, right = cr < tree_size ? tree[cr] : 0.0;
    tree[node] = left + right;
}

// full rebuild (Memory.clean / recalculate_structure, RL.py:312-331): one level of parents
__global__ __launch_bounds__(256) void k_rebuild_level(double* tree, int64_t lo, int64_t hi, int64_t tree_size) {
    const int64_t node = lo + (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (node >= hi) return;
    const int64_t cl = 2 * node + 1, cr = cl + 1;
    tree[node] = (cl < tree_size ? tree[cl] : 0.0) + (cr < tree_size ? tree[cr] : 0.0);
}

struct SampleArgs {
    const State* st;
    const double* tree;
    int64_t n_nodes, tree_size, cap;
    int32_t n;
    const double* u;   // [n] injected or null
    uint64_t seed, ctr;
    double beta;
    int32_t* tree_idx;
    int64_t* data_idx;
    float* isw;
};

__device__ __forceinline__ int64_t get_leaf(const double* tree, int64_t tree_size, double v) {
    int64_t parent = 0;
    for (;;) {   // compiled_get_leaf (RL.py:347-359)
        const int64_t cl = 2 * parent + 1, cr = cl + 1;
        if (cl >= tree_size) return parent;
        if (v <= tree[cl]) {
            parent = cl;
        } else {
            v -= tree[cl];
            parent = cr;
        }
    }
}

__global__ __launch_bounds__(256) void k_sample(const SampleArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const double total = a.tree[0];
    const double seg = total / a.n;
    const double u = a.u ? a.u[i] : u53(a.seed, a.ctr, (uint32_t)i, 0x300u);
    double v = (i + u) * seg;
    int64_t idx = get_leaf(a.tree, a.tree_size, v);
    double p = a.tree[idx];
    // "sometimes it errors": resample inside the segment until p != 0 (RL.py:457-463); the tree here is
    // always consistent, so this only triggers on zero-priority leaves at a segment edge
    for (int t = 0; p == 0.0 && t < 64; ++t) {
        const double lo = seg * i, hi = seg * (i + 1);
        v = (hi - lo) * u53(a.seed, a.ctr, (uint32_t)i, 0x301u + (uint32_t)t) + lo;
        idx = get_leaf(a.tree, a.tree_size, v);
        p = a.tree[idx];
    }
    int64_t di = idx - a.n_nodes;   // data_idx = leaf_idx - (len(tree) - capacity)
    if (di >= a.cap) di = a.cap - 1;
    if (di < 0) di += a.cap;        // Python negative index
    const double avg = total / (double)a.st->len;
    a.isw[i] = (float)pow(p / avg, -a.beta);
    a.tree_idx[i] = (int32_t)idx;
    a.data_idx[i] = di;
}

__global__ __launch_bounds__(256) void k_gather(const float* data, const int64_t* data_idx, int32_t row_len,
                                                float* out, int32_t n) {
    const int i = blockIdx.x;
    if (i >= n) return;
    const float* in = data + data_idx[i] * (int64_t)row_len;
    for (int c = threadIdx.x; c < row_len; c += 256) out[(int64_t)i * row_len + c] = in[c];
}

constexpr int kUpdThreads = 1024;

struct UpdateArgs {
    State* st;
    const int32_t* tree_idx;
    const float* err;
    int32_t n;
    double* tree;
    int64_t n_nodes, cap;
    int64_t* leaf_slot;   // out: the leaves to recompute (as slots; -1 = index rejected)
    float alpha, upper;
    double eps_scale;
};

// one workgroup: priorities of the sampled leaves, the later duplicate wins, Memory.max
__global__ __launch_bounds__(kUpdThreads) void k_update(const UpdateArgs a) {
    __shared__ float cmax[kUpdThreads];
    const int tid = threadIdx.x;
    const double mx = a.st->max;
    const float eps = (float)(a.eps_scale * mx);   // abs_errors += 0.00001 * max in float32 (RL.py:442-443)
    float cm = 0.0f;
    for (int i = tid; i < a.n; i += kUpdThreads) {
        const float c = fminf(a.err[i] + eps, a.upper);   // np.minimum(abs_errors, abs_err_upper)
        const int32_t ti = a.tree_idx[i];
        // only leaf indices [n_nodes, n_nodes + capacity) are updates: anything else (an internal node, a
        // stale or corrupt index) is skipped, so the tree and the device memory beyond it stay intact
        const bool leaf = (int64_t)ti >= a.n_nodes && (int64_t)ti < a.n_nodes + a.cap;
        if (leaf) cm = fmaxf(cm, c);
        bool last = true;
        for (int j = i + 1; j < a.n; ++j) last = last && a.tree_idx[j] != ti;
        if (leaf && last) a.tree[ti] = (double)powf(c, a.alpha);   // np.power(clipped, alpha) in float32
        a.leaf_slot[i] = leaf ? (int64_t)ti - a.n_nodes : -1;
    }
    cmax[tid] = cm;
    __syncthreads();
    for (int s = kUpdThreads / 2; s > 0; s >>= 1) {
        if (tid < s) cmax[tid] = fmaxf(cmax[tid], cmax[tid + s]);
        __syncthreads();
    }
    if (tid == 0) {
        a.st->max = 0.95 * fmax(mx, (double)cmax[0]);   // self.max = 0.95 * max(self.max, max(clipped))
        a.st->n_leaf = a.n;
    }
}

}  // namespace replay
}  // namespace qcart

using namespace qcart::replay;

struct qc_replay {
    qc_replay_params p{};
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    int64_t n_nodes = 0, tree_size = 0;
    int depth = 0;             // tree levels above the leaves
    double beta = 0.2;         // Memory.beta (host: depends only on the number of samples)
    uint64_t sample_ctr = 0;
    State* st = nullptr;
    double* tree = nullptr;
    float* data = nullptr;
    unsigned long long* owner = nullptr;
    int32_t* src = nullptr;
    int64_t* dest = nullptr;
    int64_t cap_n = 0;         // allocated length of src / dest
    int64_t* data_idx = nullptr;
    int64_t* leaf_slot = nullptr;
    int64_t cap_s = 0;         // allocated length of data_idx / leaf_slot
};

namespace {

int rfail(qc_replay* r, int code, const std::string& msg) {
    r->err = msg;
    return code;
}

struct Dev {
    int prev = -1;
    explicit Dev(int d) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~Dev() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

std::string g_replay_err;

int grow(qc_replay* r, int64_t n) {
    if (n <= r->cap_n) return QC_OK;
    if (r->src) (void)hipFree(r->src);
    if (r->dest) (void)hipFree(r->dest);
    r->src = nullptr;
    r->dest = nullptr;
    r->cap_n = 0;
    if (hipMalloc((void**)&r->src, n * sizeof(int32_t)) != hipSuccess ||
        hipMalloc((void**)&r->dest, n * sizeof(int64_t)) != hipSuccess)
        return rfail(r, QC_ENOMEM, "hipMalloc (store staging)");
    r->cap_n = n;
    return QC_OK;
}

int grow_s(qc_replay* r, int64_t n) {
    if (n <= r->cap_s) return QC_OK;
    if (r->data_idx) (void)hipFree(r->data_idx);
    if (r->leaf_slot) (void)hipFree(r->leaf_slot);
    r->data_idx = nullptr;
    r->leaf_slot = nullptr;
    r->cap_s = 0;
    if (hipMalloc((void**)&r->data_idx, n * sizeof(int64_t)) != hipSuccess ||
        hipMalloc((void**)&r->leaf_slot, n * sizeof(int64_t)) != hipSuccess)
        return rfail(r, QC_ENOMEM, "hipMalloc (sample staging)");
    r->cap_s = n;
    return QC_OK;
}

// ancestors of the listed leaves, bottom-up, one launch per level
void path_levels(qc_replay* r, const int64_t* leaf_slot, int64_t n) {
    const unsigned g = (unsigned)((n + 255) / 256);
    for (int up = 1; up <= r->depth; ++up)
        hipLaunchKernelGGL(k_level, dim3(g), dim3(256), 0, r->stream, r->st, leaf_slot, r->n_nodes, r->tree_size,
                           r->tree, up, n);
}

int store_common(qc_replay* r, int64_t n, const uint8_t* valid, CopyArgs ca) {
    if (n < 0) return rfail(r, QC_EINVAL, "n must be >= 0");
    if (n == 0) return QC_OK;
    if (n > (int64_t)1 << 30) return rfail(r, QC_EINVAL, "n too large");
    Dev g(r->device);
    int rc = grow(r, n);
    if (rc) return rc;
    PlanArgs pa{};
    pa.st = r->st;
    pa.valid = valid;
    pa.n = n;
    pa.cap = r->p.capacity;
    pa.src = r->src;
    pa.dest = r->dest;
    pa.owner = r->owner;
    pa.policy_seq = r->p.policy == 0;
    pa.abs_err_upper = r->p.abs_err_upper;
    pa.seed = r->p.seed;
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(kPlanThreads), 0, r->stream, pa);
    ca.st = r->st;
    ca.src = r->src;
    ca.dest = r->dest;
    ca.owner = r->owner;
    ca.data = r->data;
    ca.tree = r->tree;
    ca.n_nodes = r->n_nodes;
    ca.row_len = r->p.row_len;
    ca.n = n;
    hipLaunchKernelGGL(k_copy, dim3((unsigned)n), dim3(256), 0, r->stream, ca);
    path_levels(r, r->dest, n);
    return hipGetLastError() == hipSuccess ? QC_OK : rfail(r, QC_EHIP, "replay store launch failed");
}

}  // namespace

extern "C" {

int qc_replay_create(const qc_replay_params* p, int device, qc_replay** out) {
    if (!out) return QC_EINVAL;
    *out = nullptr;
    if (!p || p->capacity < 1 || p->capacity > ((int64_t)1 << 30) || p->row_len < 1) {
        g_replay_err = "capacity must be in [1, 2^30] and row_len >= 1";
        return QC_EINVAL;
    }
    if (p->policy != 0 && p->policy != 1) {
        g_replay_err = "policy must be 0 (sequential) or 1 (random)";
        return QC_EINVAL;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        g_replay_err = "no HIP device available (libqcart has no CPU fallback)";
        return QC_EHIP;
    }
    if (device < 0 || device >= ndev) {
        g_replay_err = "device index out of range";
        return QC_EINVAL;
    }
    qc_replay* r = new qc_replay();
    r->p = *p;
    r->device = device;
    r->beta = p->beta;
    int64_t width = 1, nodes = 0;
    int depth = 0;
    while (width < p->capacity) {   // SumTree.__init__ (RL.py:245-248)
        nodes += width;
        width *= 2;
        ++depth;
    }
    r->n_nodes = nodes;
    r->tree_size = nodes + p->capacity;
    r->depth = depth;
    Dev g(device);
    const size_t data_bytes = (size_t)p->capacity * (size_t)p->row_len * sizeof(float);
    if (hipMalloc((void**)&r->st, sizeof(State)) != hipSuccess ||
        hipMalloc((void**)&r->tree, (size_t)r->tree_size * sizeof(double)) != hipSuccess ||
        hipMalloc((void**)&r->data, data_bytes) != hipSuccess ||
        hipMalloc((void**)&r->owner, (size_t)p->capacity * sizeof(unsigned long long)) != hipSuccess) {
        g_replay_err = "hipMalloc failed (capacity x row_len too large?)";
        qc_replay_destroy(r);
        return QC_ENOMEM;
    }
    State s{};
    s.passes = -p->passes_before_random;   // SumTree.passes = -passes_before_random (RL.py:260)
    (void)hipMemcpy(r->st, &s, sizeof(State), hipMemcpyHostToDevice);
    (void)hipMemset(r->tree, 0, (size_t)r->tree_size * sizeof(double));
    (void)hipMemset(r->data, 0, data_bytes);
    (void)hipMemset(r->owner, 0, (size_t)p->capacity * sizeof(unsigned long long));
    if (hipDeviceSynchronize() != hipSuccess) {
        g_replay_err = "device initialisation failed";
        qc_replay_destroy(r);
        return QC_EHIP;
    }
    *out = r;
    return QC_OK;
}

void qc_replay_destroy(qc_replay* r) {
    if (!r) return;
    {
        Dev g(r->device);
        (void)hipDeviceSynchronize();
        for (void* q : {(void*)r->st, (void*)r->tree, (void*)r->data, (void*)r->owner, (void*)r->src, (void*)r->dest,
                        (void*)r->data_idx, (void*)r->leaf_slot})
            if (q) (void)hipFree(q);
    }
    delete r;
}

const char* qc_replay_last_error(const qc_replay* r) { return r ? r->err.c_str() : g_replay_err.c_str(); }

int qc_replay_set_stream(qc_replay* r, void* stream) {
    if (!r) return QC_EINVAL;
    r->stream = (hipStream_t)stream;
    return QC_OK;
}

int qc_replay_store(qc_replay* r, int64_t n, const uint8_t* valid, const float* rows) {
    if (!r || (n > 0 && !rows)) return QC_EINVAL;
    CopyArgs ca{};
    ca.rows = rows;
    return store_common(r, n, valid, ca);
}

int qc_replay_store_xp(qc_replay* r, int64_t n, const uint8_t* valid, const float* last_obs, const float* obs,
                       int32_t obs_len, const int32_t* action, const float* reward) {
    if (!r) return QC_EINVAL;
    if (obs_len < 1 || 2 * obs_len + 2 != r->p.row_len)
        return rfail(r, QC_EINVAL, "row_len must be 2 * obs_len + 2 for the 'xp' row layout");
    if (n > 0 && (!last_obs || !obs || !action || !reward)) return rfail(r, QC_EINVAL, "null row part");
    CopyArgs ca{};
    ca.last_obs = last_obs;
    ca.obs = obs;
    ca.action = action;
    ca.reward = reward;
    ca.d = obs_len;
    return store_common(r, n, valid, ca);
}

int qc_replay_sample(qc_replay* r, int32_t n, const double* u, float* transitions, int32_t* tree_idx,
                     float* is_weights) {
    if (!r || n < 1 || !tree_idx || !is_weights) return QC_EINVAL;
    Dev g(r->device);
    int rc = grow_s(r, n);
    if (rc) return rc;
    r->beta = std::min(1.0, r->beta + r->p.beta_increment);   // Memory.obtain_sample (RL.py:430)
    SampleArgs sa{};
    sa.st = r->st;
    sa.tree = r->tree;
    sa.n_nodes = r->n_nodes;
    sa.tree_size = r->tree_size;
    sa.cap = r->p.capacity;
    sa.n = n;
    sa.u = u;
    sa.seed = r->p.seed;
    sa.ctr = r->sample_ctr++;
    sa.beta = r->beta;
    sa.tree_idx = tree_idx;
    sa.data_idx = r->data_idx;
    sa.isw = is_weights;
    hipLaunchKernelGGL(k_sample, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, r->stream, sa);
    if (transitions)
        hipLaunchKernelGGL(k_gather, dim3((unsigned)n), dim3(256), 0, r->stream, r->data, r->data_idx, r->p.row_len,
                           transitions, n);
    return hipGetLastError() == hipSuccess ? QC_OK : rfail(r, QC_EHIP, "replay sample launch failed");
}

int qc_replay_update(qc_replay* r, int32_t n, const int32_t* tree_idx, const float* abs_errors) {
    if (!r || n < 0 || (n > 0 && (!tree_idx || !abs_errors))) return QC_EINVAL;
    if (n == 0) return QC_OK;
    Dev g(r->device);
    int rc = grow_s(r, n);
    if (rc) return rc;
    UpdateArgs ua{};
    ua.st = r->st;
    ua.tree_idx = tree_idx;
    ua.err = abs_errors;
    ua.n = n;
    ua.tree = r->tree;
    ua.n_nodes = r->n_nodes;
    ua.cap = r->p.capacity;
    ua.leaf_slot = r->leaf_slot;
    ua.alpha = (float)r->p.alpha;
    ua.upper = (float)r->p.abs_err_upper;
    ua.eps_scale = r->p.epsilon_scale;
    hipLaunchKernelGGL(k_update, dim3(1), dim3(kUpdThreads), 0, r->stream, ua);
    path_levels(r, r->leaf_slot, n);
    return hipGetLastError() == hipSuccess ? QC_OK : rfail(r, QC_EHIP, "replay update launch failed");
}

int qc_replay_rebuild(qc_replay* r) {
    if (!r) return QC_EINVAL;
    Dev g(r->device);
    // levels of internal nodes bottom-up: level l holds nodes [2^l - 1, 2^(l+1) - 1)
    for (int l = r->depth - 1; l >= 0; --l) {
        const int64_t lo = ((int64_t)1 << l) - 1, hi = ((int64_t)1 << (l + 1)) - 1;
        hipLaunchKernelGGL(k_rebuild_level, dim3((unsigned)((hi - lo + 255) / 256)), dim3(256), 0, r->stream, r->tree,
                           lo, hi, r->tree_size);
    }
    return hipGetLastError() == hipSuccess ? QC_OK : rfail(r, QC_EHIP, "replay rebuild launch failed");
}

int qc_replay_stats(qc_replay* r, qc_replay_stats_t* out) {
    if (!r || !out) return QC_EINVAL;
    Dev g(r->device);
    State s{};
    double total = 0.0;
    if (hipStreamSynchronize(r->stream) != hipSuccess ||
        hipMemcpy(&s, r->st, sizeof(State), hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&total, r->tree, sizeof(double), hipMemcpyDeviceToHost) != hipSuccess)
        return rfail(r, QC_EHIP, "stats copy failed");
    out->len = s.len;
    out->data_pointer = s.ptr;
    out->passes = s.passes;
    out->max = s.max;
    out->beta = r->beta;
    out->total_p = total;
    out->n_nodes = r->n_nodes;
    out->tree_size = r->tree_size;
    return QC_OK;
}

int qc_replay_buffers(const qc_replay* r, const double** tree, const float** data) {
    if (!r) return QC_EINVAL;
    if (tree) *tree = r->tree;
    if (data) *data = r->data;
    return QC_OK;
}

}  // extern "C"
