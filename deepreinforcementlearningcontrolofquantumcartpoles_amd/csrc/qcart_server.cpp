// qcart_server.cpp — the step server: the reference's process model (P actor processes, each with its own
// `simulation` module stepping ONE env per call, IHO/main_parallel.py:345-359, :264) served by one process that
// owns the GPU. Clients (qcart_client.c, libqcart_client.so, no HIP) post their state into a shared-memory slot
// (qcart_shm.h); every tick the server steps all pending envs in ONE batched launch of its handle (env e = slot
// e): the per-process H2D copy + two launches + D2H copy + sync of the plain drop-in, serialised over P HIP
// contexts, becomes one set of launches per tick for all of them.
//
// The resident path (QCART_SERVER_RESIDENT=0 turns it off): for the Fock modules the server keeps k_resident on the
// GPU while it runs — one wave per slot polling the slot's rreq word in the device-mapped object — and a client sends
// its step(state, dt, force, gamma) there directly (on the action grid, at the kernel's dt and gamma): the GPU steps
// the row in place and publishes rdone; the server thread only keeps the heartbeat and serves everything else by
// ticks. Table changes (a new dt, an off-grid force slot) stop the kernel first and relaunch it after the tick.
//
// A tick: wait until every owned slot has a pending request or batch_wait_us has passed since the first one;
// copy the pending states into the server's pinned, device-mapped work rows (the kernels read and write them
// in place: no hipMemcpy); per-env MT19937 reseeds (masked), the step envs grouped by physics-step count and
// (dt, gamma) — each group one qc_step with a per-env step budget (env_steps: the others stay frozen) — then
// x_expectation / moments over the batch; one stream synchronisation; results back into the slots; done = req.
#include <hip/hip_runtime.h>
#include <errno.h>
#include <fcntl.h>
#include <signal.h>
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/qcart.h"
#include "qcart_shm.h"

namespace qcart {
void set_global_error(const std::string& m);   // qcart_api.cpp: what qc_last_error(NULL) returns
bool resident_available(const qc_handle* h);
int resident_launch(qc_handle* h, void* psi, void* slots, double* obs, const uint32_t* ctl, double beat_s,
                    double lease_s, uint32_t gen, void* stream);
}

namespace {

int futex_wait(uint32_t* addr, uint32_t val, long timeout_ns) {
    struct timespec ts = {timeout_ns / 1000000000L, timeout_ns % 1000000000L};
    return (int)syscall(SYS_futex, addr, FUTEX_WAIT, val, &ts, nullptr, 0);
}
void futex_wake(uint32_t* addr, int n) { syscall(SYS_futex, addr, FUTEX_WAKE, n, nullptr, nullptr, 0); }

inline uint32_t ld_acq(const uint32_t* p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline void cpu_relax() { __builtin_ia32_pause(); }

size_t round_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

template <typename T>
int host_alloc(T** h, T** d, size_t n) {
    if (hipHostMalloc((void**)h, n * sizeof(T), hipHostMallocMapped) != hipSuccess) return QC_ENOMEM;
    std::memset(*h, 0, n * sizeof(T));
    if (hipHostGetDevicePointer((void**)d, *h, 0) != hipSuccess) return QC_EHIP;
    return QC_OK;
}

}  // namespace

struct qc_server {
    qc_params p{};
    int device = 0;
    int P = 0, N = 0, n_obs = 0;
    double wait_us = 40.0;
    std::string name, err;
    qc_handle* h = nullptr;
    hipStream_t stream = nullptr;
    // the tick's completion: an event polled by this (already busy) server thread — hipStreamSynchronize's
    // blocking wait adds its wake-up latency to every tick; QCART_SERVER_SYNC=block restores it (A/B)
    hipEvent_t done = nullptr;
    bool spin_sync = true;
    // shared memory
    int fd = -1;
    size_t shm_bytes = 0;
    uint8_t* shm = nullptr;
    qcs_header* hdr = nullptr;
    qcs_slot* slots = nullptr;
    double* spsi = nullptr;   // [P][2N] the clients' rows
    double* sobs = nullptr;   // [P][QCS_MAX_OBS]
    // pinned, device-mapped work buffers (host pointer, device pointer)
    double *psi = nullptr, *d_psi = nullptr;         // [P][2N]
    int32_t *act = nullptr, *d_act = nullptr;        // [P]
    int32_t *st1 = nullptr, *d_st1 = nullptr;        // [P] step budgets of the 1-step group
    int32_t *st10 = nullptr, *d_st10 = nullptr;      // [P] ... of the 10-step group
    uint32_t *seeds = nullptr, *d_seeds = nullptr;   // [P]
    uint8_t *mask = nullptr, *d_mask = nullptr;      // [P]
    double *q1 = nullptr, *d_q1 = nullptr, *xm1 = nullptr, *d_xm1 = nullptr;     // [1][P]
    double *q10 = nullptr, *d_q10 = nullptr, *xm10 = nullptr, *d_xm10 = nullptr; // [10][P]
    int32_t *fs1 = nullptr, *d_fs1 = nullptr, *fb10 = nullptr, *d_fb10 = nullptr; // [P]
    double *xe = nullptr, *d_xe = nullptr;           // [P]
    double *hp = nullptr, *d_hp = nullptr;           // [P][2N] Hamiltonian_dot_psi rows (the op writes every row of
                                                     // its buffer: never the clients' own rows, nor the step buffer)
    double *obs = nullptr, *d_obs = nullptr;         // [P][n_obs]
    // the clients' state rows registered with HIP (device-mapped): the kernels step them in place, no copy in or out
    // (QCART_SERVER_INPLACE=0, or a failed registration: copies through `psi`)
    double* d_spsi = nullptr;
    bool inplace = false;
    // the resident path: the whole object registered (d_shm), k_resident on its own stream while run() serves
    bool resident = false, r_running = false, r_lost = false;   // r_lost: a launch failed, the path is off
    uint8_t* d_shm = nullptr;
    hipStream_t rstream = nullptr;
    hipEvent_t r_exit = nullptr;   // recorded after the resident launch: complete once every wave has exited
    uint32_t beat = 0;
    double t_beat = 0;
    // a launch's lease (QCART_RESIDENT_LEASE_MS, default 20 ms): its waves exit at their first idle poll after it and
    // the loop relaunches at once, so a device-wide synchronisation in this process never waits longer
    double lease_us = 20000.0, t_lease = 0;
    int64_t launches = 0;
    uint32_t r_gen = 0;   // + 1 per dynamics change (dt, gamma): requests checked against older ones bounce
    // MT19937 prefetch (QCART_SERVER_PREFETCH=0 turns it off): after a tick, every owned env that has no drawn pair
    // draws its next step's pair into d_pre (has_pre = 1) while the clients turn round; a 1-step call then steps on
    // it directly and a 10-step call takes it as its step 0 — the normals kernel leaves the tick's critical path.
    // The streams advance exactly as without it (the same words in the same order).
    bool prefetch = true;
    double* d_pre = nullptr;                         // device [P][2]
    double* d_n10 = nullptr;                         // device [10][P][2]
    std::vector<uint8_t> pre_ok;                     // [P] env e has a drawn pair in d_pre (host bookkeeping)
    uint8_t *has_pre = nullptr, *d_has_pre = nullptr;   // [P] pre_ok as the 10-step draw reads it (written before
                                                        // the launch: a kernel reads mapped memory when it runs)
    int32_t *gen = nullptr, *d_gen = nullptr;        // [P] draw budgets of the tick's 1-step envs without a pair
    int32_t *pf = nullptr, *d_pf = nullptr;          // [P] draw budgets of the prefetch
    std::vector<uint32_t> served;                    // last served req per slot
    std::map<double, int> custom;                    // off-grid force -> slot
    double cur_dt = 0, cur_gamma = 0;
    std::atomic<int> stop{0};
    int64_t ticks = 0, calls = 0;
    // per-tick phase sums (us): batching wait, host launches, GPU until the stream sync returned, publishing
    double t_wait = 0, t_launch = 0, t_gpu = 0, t_publish = 0;
};

namespace {

int sfail(qc_server* s, int code, const std::string& msg) {
    if (s) s->err = msg;
    return code;
}

void resident_stop(qc_server* s);

// force -> action slot, as the drop-in (simulation.py _slot): the 21-level grid, else a cached custom slot
int slot_of(qc_server* s, double force, int& slot) {
    const int half = s->p.n_actions / 2;
    const double spacing = s->p.f_max / half;
    const double a = std::nearbyint(force / spacing);
    if (a >= -half && a <= half && a * spacing == force) {
        slot = (int)a + half;
        return QC_OK;
    }
    auto it = s->custom.find(force);
    if (it != s->custom.end()) {
        slot = it->second;
        return QC_OK;
    }
    resident_stop(s);   // the slot tables are rebuilt
    const int rc = qc_add_force(s->h, force);
    if (rc < 0) return rc;
    s->custom[force] = rc;
    slot = rc;
    return QC_OK;
}

// the resident kernel (no-ops without the resident path): stopped before anything changes the slot tables or the
// handle's dynamics, and when run() returns; (re)launched by the serving loop
void resident_stop(qc_server* s) {
    if (!s->r_running) return;
    __atomic_store_n(&s->hdr->r_quit, 1u, __ATOMIC_SEQ_CST);
    (void)hipStreamSynchronize(s->rstream);   // every wave reaches the quit word within a poll
    __atomic_store_n(&s->hdr->r_quit, 0u, __ATOMIC_SEQ_CST);
    s->r_running = false;
}
void resident_start(qc_server* s) {
    if (!s->resident || s->r_running) return;
    if (s->r_exit && hipEventQuery(s->r_exit) == hipErrorNotReady) return;   // (a previous launch still draining)
    qcs_header* H = s->hdr;
    H->r_dt = s->cur_dt;
    H->r_gamma = s->cur_gamma;
    __atomic_store_n(&H->r_gen, s->r_gen, __ATOMIC_SEQ_CST);
    __atomic_store_n(&H->r_quit, 0u, __ATOMIC_SEQ_CST);
    const size_t ctl = offsetof(qcs_header, r_quit);
    const int rc = qcart::resident_launch(s->h, s->d_spsi, s->d_shm + H->slot_off, (double*)(s->d_shm + H->obs_off),
                                          (const uint32_t*)(s->d_shm + ctl), 1.0, s->lease_us * 1e-6, s->r_gen,
                                          s->rstream);
    if (rc != QC_OK || hipEventRecord(s->r_exit, s->rstream) != hipSuccess) {
        // no resident kernel: every request goes through the ticks (clients bounce off r_on = 0; a request posted
        // before they saw it is bounced by resident_tend)
        __atomic_store_n(&H->r_on, 0u, __ATOMIC_SEQ_CST);
        s->resident = false;
        s->r_lost = true;
        return;
    }
    s->r_running = true;
    s->t_lease = now_us() + s->lease_us;
    s->launches++;
}
// the server loop's heartbeat (every 100 us at most) and the kernel's state: exited on its own (a heartbeat gap
// longer than its limit) -> relaunched
void resident_tend(qc_server* s, double now) {
    if (s->r_lost) {   // the path was turned off while clients may still post resident requests: they take the ticks
        for (int e = 0; e < s->P; ++e) {
            qcs_slot& sl = s->slots[e];
            const uint32_t rr = __atomic_load_n(&sl.rreq, __ATOMIC_ACQUIRE);
            if (rr != __atomic_load_n(&sl.rdone, __ATOMIC_ACQUIRE)) {
                sl.rstatus = QCS_EBOUNCE;
                __atomic_store_n(&sl.rdone, rr, __ATOMIC_RELEASE);
            }
        }
    }
    if (!s->resident) return;
    if (now - s->t_beat > 100.0) {
        __atomic_store_n(&s->hdr->r_beat, ++s->beat, __ATOMIC_RELAXED);
        s->t_beat = now;
    }
    if (s->r_running && hipEventQuery(s->r_exit) == hipSuccess) s->r_running = false;
    if (!s->r_running) resident_start(s);
}

void free_server(qc_server* s) {
    resident_stop(s);
    if (s->h) qc_destroy(s->h);
    void* hb[] = {s->psi, s->act, s->st1, s->st10, s->seeds, s->mask, s->q1, s->xm1, s->q10, s->xm10, s->fs1, s->fb10,
                  s->xe, s->obs, s->has_pre, s->gen, s->pf, s->hp};
    for (void* b : hb)
        if (b) (void)hipHostFree(b);
    if (s->d_pre) (void)hipFree(s->d_pre);
    if (s->d_n10) (void)hipFree(s->d_n10);
    if (s->inplace && s->shm) (void)hipHostUnregister(s->d_shm ? s->shm : s->shm + s->hdr->psi_off);
    if (s->r_exit) (void)hipEventDestroy(s->r_exit);
    if (s->rstream) (void)hipStreamDestroy(s->rstream);
    if (s->done) (void)hipEventDestroy(s->done);
    if (s->stream) (void)hipStreamDestroy(s->stream);
    if (s->shm) {
        if (s->hdr) __atomic_store_n(&s->hdr->alive, 0u, __ATOMIC_SEQ_CST);
        munmap(s->shm, s->shm_bytes);
    }
    if (s->fd >= 0) close(s->fd);
    if (!s->name.empty()) shm_unlink(s->name.c_str());
}

// one tick over the pending slots `pend`
void serve_tick(qc_server* s, const std::vector<int>& pend) {
    const double t_start = now_us();
    const int P = s->P, N = s->N;
    struct Req { int op, n; uint32_t seed; double dt, force, gamma; };
    std::vector<Req> rq(P);
    bool any_seed = false, any_x = false, any_obs = false, any_h = false;
    std::vector<int> g1, g10;   // step groups
    for (int e : pend) {
        qcs_slot& sl = s->slots[e];
        Req r{sl.op, sl.n, sl.seed, sl.dt, sl.force, sl.gamma};
        rq[e] = r;
        sl.status = QC_OK;
        sl.err[0] = 0;
        if (r.op == QCS_OP_SET_SEED) {
            s->seeds[e] = r.seed;
            s->mask[e] = 1;
            s->pre_ok[e] = 0;   // a drawn pair belongs to the old stream
            any_seed = true;
            continue;
        }
        if (r.op == QCS_OP_HDOT) {
            if (!s->hp) {   // (grid modules have no Hamiltonian_dot_psi)
                sl.status = QC_EINVAL;
                std::snprintf(sl.err, sizeof(sl.err), "Hamiltonian_dot_psi is a Fock-module function");
                continue;
            }
            std::memcpy(s->hp + (size_t)e * 2 * N, s->spsi + (size_t)e * 2 * N, sizeof(double) * 2 * N);
            any_h = true;
            continue;
        }
        if (!s->inplace) std::memcpy(s->psi + (size_t)e * 2 * N, s->spsi + (size_t)e * 2 * N, sizeof(double) * 2 * N);
        if (r.op == QCS_OP_STEP) (r.n == 10 ? g10 : g1).push_back(e);
        else if (r.op == QCS_OP_X_EXPECT) any_x = true;
        else any_obs = true;
    }
    auto err_all = [&](const std::vector<int>& es, int rc) {
        const char* m = qc_last_error(s->h);
        for (int e : es) {
            s->slots[e].status = rc;
            std::snprintf(s->slots[e].err, sizeof(s->slots[e].err), "%s", m ? m : "");
        }
    };
    if (any_seed) {
        std::vector<int> es;
        for (int e : pend) if (rq[e].op == QCS_OP_SET_SEED) es.push_back(e);
        const int rc = qc_set_seed_mt19937_envs(s->h, s->d_seeds, s->d_mask);
        if (rc) err_all(es, rc);
    }
    // step groups: by step count, then by (dt, gamma) (one set of tables per handle: the drivers pass the same
    // dt and gamma on every call; a change rebuilds them, as the reference's reset_ab on a dt change)
    for (int grp = 0; grp < 2; ++grp) {
        const std::vector<int>& G = grp == 0 ? g1 : g10;
        std::vector<int> rest = G;
        while (!rest.empty()) {
            const double dt = rq[rest[0]].dt, gamma = rq[rest[0]].gamma;
            std::vector<int> now, later;
            for (int e : rest) ((rq[e].dt == dt && rq[e].gamma == gamma) ? now : later).push_back(e);
            rest = later;
            int rc = QC_OK;
            if (dt != s->cur_dt || gamma != s->cur_gamma) {
                resident_stop(s);
                (void)hipStreamSynchronize(s->stream);
                rc = qc_set_dynamics(s->h, dt, gamma);
                if (rc == QC_OK) { s->cur_dt = dt; s->cur_gamma = gamma; s->r_gen++; }
            }
            int32_t* stb = grp == 0 ? s->st1 : s->st10;
            if (!later.empty()) (void)hipStreamSynchronize(s->stream);   // the budget array is read by the kernels
            std::memset(stb, 0, sizeof(int32_t) * P);
            std::vector<int> ok;
            for (int e : now) {
                int sl = 0;
                const int r2 = rc ? rc : slot_of(s, rq[e].force, sl);
                if (r2) { err_all({e}, r2); continue; }
                s->act[e] = sl;
                stb[e] = grp == 0 ? 1 : 10;
                ok.push_back(e);
            }
            if (ok.empty()) continue;
            const int n = grp == 0 ? 1 : 10;
            const double* noise = nullptr;   // nullptr: qc_step draws from the streams itself
            if (s->prefetch) {
                if (grp == 0) {
                    // the pairs of the group's envs that have none yet (after a reseed or a 10-step call)
                    bool any = false;
                    for (int e = 0; e < P; ++e) s->gen[e] = 0;
                    for (int e : ok)
                        if (!s->pre_ok[e]) { s->gen[e] = 1; any = true; }
                    if (any) rc = qc_mt19937_normals(s->h, 1, s->d_gen, nullptr, nullptr, s->d_pre);
                    noise = s->d_pre;
                } else {
                    for (int e = 0; e < P; ++e) s->has_pre[e] = s->pre_ok[e];
                    rc = qc_mt19937_normals(s->h, 10, s->d_st10, s->d_pre, s->d_has_pre, s->d_n10);
                    noise = s->d_n10;
                }
                if (rc) { err_all(ok, rc); continue; }
            }
            rc = qc_step(s->h, s->inplace ? s->d_spsi : s->d_psi, s->d_act, s->p.n_actions / 2, n,
                         grp == 0 ? s->d_st1 : s->d_st10, noise, grp == 0 ? s->d_q1 : s->d_q10,
                         grp == 0 ? s->d_xm1 : s->d_xm10, grp == 0 ? s->d_fs1 : nullptr, nullptr, nullptr);
            // the pairs consumed (a 10-step draw took them already)
            if (s->prefetch && (grp == 1 || rc == QC_OK))
                for (int e : ok) s->pre_ok[e] = 0;
            // simulate_10_steps' Fail is the boundary test of the final state (IHO/simulation_i.cpp:391-421)
            if (rc == QC_OK && grp == 1) rc = qc_boundary_fail(s->h, s->inplace ? s->d_spsi : s->d_psi, s->d_fb10);
            if (rc) err_all(ok, rc);
        }
    }
    if (any_x) {
        const int rc = qc_x_expectation(s->h, s->inplace ? s->d_spsi : s->d_psi, s->d_xe);
        if (rc) { std::vector<int> es; for (int e : pend) if (rq[e].op == QCS_OP_X_EXPECT) es.push_back(e); err_all(es, rc); }
    }
    if (any_h) {
        const int rc = qc_hamiltonian_dot_psi(s->h, s->d_hp);
        if (rc) { std::vector<int> es; for (int e : pend) if (rq[e].op == QCS_OP_HDOT) es.push_back(e); err_all(es, rc); }
    }
    if (any_obs) {
        const int rc = qc_moments(s->h, s->inplace ? s->d_spsi : s->d_psi, s->d_obs);
        if (rc) { std::vector<int> es; for (int e : pend) if (rq[e].op == QCS_OP_MOMENTS || rq[e].op == QCS_OP_FOCK_OBS) es.push_back(e); err_all(es, rc); }
    }
    const double t_l = now_us();
    hipError_t e = hipSuccess;
    if (s->spin_sync && hipEventRecord(s->done, s->stream) == hipSuccess) {
        while ((e = hipEventQuery(s->done)) == hipErrorNotReady) cpu_relax();
    } else {
        e = hipStreamSynchronize(s->stream);
    }
    if (e != hipSuccess) {
        qc_sync(s->h);
        err_all(pend, QC_EHIP);
    }
    if (qc_take_errors(s->h) != 0) err_all(pend, QC_EINVAL);
    const double t_g = now_us();
    s->t_launch += t_l - t_start;
    s->t_gpu += t_g - t_l;
    for (int e : pend) {
        qcs_slot& sl = s->slots[e];
        const Req& r = rq[e];
        if (sl.status == QC_OK) {
            if (r.op == QCS_OP_STEP) {
                if (!s->inplace) std::memcpy(s->spsi + (size_t)e * 2 * N, s->psi + (size_t)e * 2 * N, sizeof(double) * 2 * N);
                if (r.n == 10) {
                    sl.q = s->q10[(size_t)9 * P + e];
                    sl.xmean = s->xm10[(size_t)9 * P + e];
                    sl.fail = s->fb10[e] ? 1 : 0;
                } else {
                    sl.q = s->q1[e];
                    sl.xmean = s->xm1[e];
                    sl.fail = s->fs1[e] > 0 ? 1 : 0;
                }
            } else if (r.op == QCS_OP_X_EXPECT) {
                sl.value = s->xe[e];
            } else if (r.op == QCS_OP_HDOT) {
                std::memcpy(s->spsi + (size_t)e * 2 * N, s->hp + (size_t)e * 2 * N, sizeof(double) * 2 * N);
            } else if (r.op == QCS_OP_MOMENTS || r.op == QCS_OP_FOCK_OBS) {
                std::memcpy(s->sobs + (size_t)e * QCS_MAX_OBS, s->obs + (size_t)e * s->n_obs, sizeof(double) * s->n_obs);
            }
        }
        s->mask[e] = 0;
        s->served[e] = __atomic_load_n(&sl.req, __ATOMIC_RELAXED);
        __atomic_store_n(&sl.done, s->served[e], __ATOMIC_SEQ_CST);
    }
    s->t_publish += now_us() - t_g;
    if (s->prefetch) {
        // every owned env without a drawn pair draws its next one now, while the clients turn round (the next tick's
        // launches queue behind it on the stream; pf is rewritten only after the next tick's completion)
        bool any = false;
        for (int e = 0; e < P; ++e) {
            s->pf[e] = 0;
            if (ld_acq(&s->slots[e].owner) && !s->pre_ok[e]) { s->pf[e] = 1; s->pre_ok[e] = 1; any = true; }
        }
        if (any && qc_mt19937_normals(s->h, 1, s->d_pf, nullptr, nullptr, s->d_pre) != QC_OK) {
            for (int e = 0; e < P; ++e) if (s->pf[e]) s->pre_ok[e] = 0;
            s->prefetch = false;   // (a launch failure: draw in qc_step from now on)
        }
    }
    s->ticks++;
    s->calls += (int64_t)pend.size();
    s->hdr->ticks = (uint64_t)s->ticks;
    s->hdr->calls = (uint64_t)s->calls;
    __atomic_add_fetch(&s->hdr->tick, 1u, __ATOMIC_SEQ_CST);
    bool wake = false;
    for (int e : pend) wake = wake || __atomic_load_n(&s->slots[e].waiting, __ATOMIC_SEQ_CST);
    if (wake) futex_wake(&s->hdr->tick, 1 << 30);
}

// slots whose client process has exited without qcc_close (killed actor): released, so that the batching wait
// does not hold every tick for a request that never comes (a pending one is dropped)
void reap_dead_clients(qc_server* s) {
    for (int e = 0; e < s->P; ++e) {
        qcs_slot& sl = s->slots[e];
        const int32_t pid = __atomic_load_n(&sl.pid, __ATOMIC_ACQUIRE);
        if (!ld_acq(&sl.owner) || pid <= 0) continue;
        if (kill(pid, 0) == 0 || errno != ESRCH) continue;
        const uint32_t rr = __atomic_load_n(&sl.rreq, __ATOMIC_ACQUIRE);
        if (rr != __atomic_load_n(&sl.rdone, __ATOMIC_ACQUIRE)) {
            if (s->r_running) continue;   // the resident wave serves it first (the slot is released afterwards)
            sl.rstatus = QCS_EDROPPED;
            __atomic_store_n(&sl.rdone, rr, __ATOMIC_RELEASE);
        }
        // a pending request is published as dropped, never as served (its state row and results were not written)
        sl.status = QCS_EDROPPED;
        std::snprintf(sl.err, sizeof(sl.err), "request dropped: client process %d exited", (int)pid);
        s->served[e] = __atomic_load_n(&sl.req, __ATOMIC_ACQUIRE);
        __atomic_store_n(&sl.done, s->served[e], __ATOMIC_RELEASE);
        __atomic_store_n(&sl.pid, 0, __ATOMIC_RELAXED);
        __atomic_sub_fetch(&s->hdr->n_clients, 1u, __ATOMIC_SEQ_CST);
        __atomic_store_n(&sl.owner, 0u, __ATOMIC_RELEASE);
    }
}

// an existing step-server object whose server is gone: it stopped (alive 0) or its process no longer exists in this
// PID namespace. Anything else (a live server, another program's object, one from another namespace) is kept.
bool stale_object(const char* name) {
    const int fd = shm_open(name, O_RDONLY, 0);
    if (fd < 0) return false;
    qcs_header h{};
    const bool got = pread(fd, &h, sizeof(h), 0) == (ssize_t)sizeof(h);
    close(fd);
    if (!got || h.magic != QCS_MAGIC || h.version != QCS_VERSION || h.pid_ns != qcs_pid_ns()) return false;
    if (!__atomic_load_n(&h.alive, __ATOMIC_RELAXED)) return true;
    return h.server_pid > 0 && kill(h.server_pid, 0) != 0 && errno == ESRCH;
}

void scan(qc_server* s, std::vector<int>& pend, int& owned) {
    pend.clear();
    owned = 0;
    for (int e = 0; e < s->P; ++e) {
        if (!ld_acq(&s->slots[e].owner)) continue;
        ++owned;
        if (ld_acq(&s->slots[e].req) != s->served[e]) pend.push_back(e);
    }
}

}  // namespace

extern "C" {

int qc_server_create(const qc_params* p, int device, int32_t max_clients, const char* name, double batch_wait_us,
                     qc_server** out) {
    if (!out || !p || !name || !*name || name[0] != '/' || max_clients < 1 || max_clients > 4096) return QC_EINVAL;
    *out = nullptr;
    if (p->precision != QC_FP64) return QC_EINVAL;   // the drop-in computes in fp64 like the reference
    qc_server* s = new qc_server();
    s->p = *p;
    s->p.batch = max_clients;
    s->p.env_offset = 0;
    s->device = device;
    s->P = max_clients;
    s->wait_us = batch_wait_us > 0 ? batch_wait_us : 40.0;
    int rc = qc_create(&s->p, device, &s->h);
    if (rc) { delete s; return rc; }
    s->N = qc_dim(s->h);
    s->n_obs = qc_n_obs(s->h);
    s->cur_dt = p->dt;
    s->cur_gamma = p->gamma;
    const int P = s->P, N = s->N;
    // (the message also goes to qc_last_error(NULL): the caller has no server handle to ask)
    auto bail = [&](int code, const std::string& m) {
        s->err = m;
        qcart::set_global_error(m);
        free_server(s);
        delete s;
        return code;
    };
    if (s->n_obs > QCS_MAX_OBS)   // the shared object's observation rows (grid moment orders <= 9)
        return bail(QC_EINVAL, "the step server serves moment_order <= 9 (its observation rows hold 64 values)");
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(QC_EHIP, "hipStreamCreate failed");
    if (hipEventCreateWithFlags(&s->done, hipEventDisableTiming) != hipSuccess)
        return bail(QC_EHIP, "hipEventCreate failed");
    {
        const char* m = std::getenv("QCART_SERVER_SYNC");
        s->spin_sync = !(m && std::strcmp(m, "block") == 0);
    }
    qc_set_stream(s->h, s->stream);
    if (host_alloc(&s->psi, &s->d_psi, (size_t)P * 2 * N) || host_alloc(&s->act, &s->d_act, P) ||
        host_alloc(&s->st1, &s->d_st1, P) || host_alloc(&s->st10, &s->d_st10, P) || host_alloc(&s->seeds, &s->d_seeds, P) ||
        host_alloc(&s->mask, &s->d_mask, P) || host_alloc(&s->q1, &s->d_q1, P) || host_alloc(&s->xm1, &s->d_xm1, P) ||
        host_alloc(&s->q10, &s->d_q10, (size_t)10 * P) || host_alloc(&s->xm10, &s->d_xm10, (size_t)10 * P) ||
        host_alloc(&s->fs1, &s->d_fs1, P) || host_alloc(&s->fb10, &s->d_fb10, P) || host_alloc(&s->xe, &s->d_xe, P) ||
        host_alloc(&s->obs, &s->d_obs, (size_t)P * (s->n_obs > 0 ? s->n_obs : 1)) ||
        host_alloc(&s->has_pre, &s->d_has_pre, P) || host_alloc(&s->gen, &s->d_gen, P) || host_alloc(&s->pf, &s->d_pf, P) ||
        (p->family <= 1 && host_alloc(&s->hp, &s->d_hp, (size_t)P * 2 * N)))
        return bail(QC_ENOMEM, "pinned host buffers");
    {
        const char* m = std::getenv("QCART_SERVER_PREFETCH");
        s->prefetch = !(m && std::atoi(m) == 0);
    }
    if (hipMalloc((void**)&s->d_pre, sizeof(double) * 2 * P) != hipSuccess ||
        hipMalloc((void**)&s->d_n10, sizeof(double) * 20 * P) != hipSuccess)
        return bail(QC_ENOMEM, "device noise buffers");
    // every env starts on seed 0's MT19937 stream (the plain drop-in's state before the first set_seed)
    rc = qc_set_seed_mt19937(s->h, s->d_seeds);
    if (rc == QC_OK) rc = qc_sync(s->h);
    if (rc) return bail(rc, "initial MT19937 seeding failed");
    // the shared-memory object
    const size_t slot_off = round_up(sizeof(qcs_header), 4096);
    const size_t psi_off = round_up(slot_off + sizeof(qcs_slot) * P, 4096);
    const size_t obs_off = round_up(psi_off + sizeof(double) * 2 * N * P, 4096);
    const size_t total = round_up(obs_off + sizeof(double) * QCS_MAX_OBS * P, 4096);
    s->fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (s->fd < 0 && errno == EEXIST && stale_object(name)) {
        // left behind by a server that died without qc_server_destroy: replaced
        shm_unlink(name);
        s->fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    }
    if (s->fd < 0) return bail(QC_EINVAL, std::string("shm_open(") + name + "): " + strerror(errno));
    s->name = name;
    if (ftruncate(s->fd, (off_t)total) != 0) return bail(QC_ENOMEM, "ftruncate");
    void* m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, s->fd, 0);
    if (m == MAP_FAILED) return bail(QC_ENOMEM, "mmap");
    s->shm = (uint8_t*)m;
    s->shm_bytes = total;
    std::memset(s->shm, 0, total);
    s->hdr = (qcs_header*)s->shm;
    s->slots = (qcs_slot*)(s->shm + slot_off);
    s->spsi = (double*)(s->shm + psi_off);
    s->sobs = (double*)(s->shm + obs_off);
    {
        // the state rows (page-aligned, whole pages) registered and device-mapped: stepped in place
        // in place needs the short-call step kernel (qc_step's MODE 0 for n <= 10 on a batch <= 4096), which leaves a
        // frozen env's row unread and unwritten: the rows of clients not in the tick are theirs to write meanwhile
        const char* m = std::getenv("QCART_SERVER_INPLACE");
        const char* m0 = std::getenv("QCART_SHORT_MODE0");
        const char* mr = std::getenv("QCART_SERVER_RESIDENT");
        if (const char* ml = std::getenv("QCART_RESIDENT_LEASE_MS")) s->lease_us = std::max(0.05, std::atof(ml)) * 1e3;
        const bool inpl = !(m && std::atoi(m) == 0) && !(m0 && std::atoi(m0) == 0) && P <= 4096;
        // the resident path: the whole object (header, slots, rows) registered, the kernel's stream and exit event
        if (inpl && !(mr && std::atoi(mr) == 0) && qcart::resident_available(s->h) &&
            hipStreamCreateWithFlags(&s->rstream, hipStreamNonBlocking) == hipSuccess &&
            hipEventCreateWithFlags(&s->r_exit, hipEventDisableTiming) == hipSuccess &&
            hipHostRegister(s->shm, total, hipHostRegisterMapped) == hipSuccess) {
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, s->shm, 0) == hipSuccess) {
                s->d_shm = (uint8_t*)d;
                s->d_spsi = (double*)(s->d_shm + psi_off);
                s->inplace = true;
                s->resident = true;
                s->prefetch = false;   // the resident wave draws each step's pair itself: no pair drawn ahead
            } else {
                (void)hipHostUnregister(s->shm);
            }
        } else if (inpl &&
            hipHostRegister(s->shm + psi_off, obs_off - psi_off, hipHostRegisterMapped) == hipSuccess) {
            void* d = nullptr;
            if (hipHostGetDevicePointer(&d, s->shm + psi_off, 0) == hipSuccess) {
                s->d_spsi = (double*)d;
                s->inplace = true;
            } else {
                (void)hipHostUnregister(s->shm + psi_off);
            }
        }
        (void)hipGetLastError();
    }
    qcs_header* H = s->hdr;
    H->magic = QCS_MAGIC;
    H->version = QCS_VERSION;
    H->max_clients = P;
    H->N = N;
    H->n_obs = s->n_obs;
    H->family = p->family;
    H->slot_off = slot_off;
    H->psi_off = psi_off;
    H->obs_off = obs_off;
    H->total_bytes = total;
    H->n_max = p->n_max;
    H->moment_order = p->moment_order;
    H->omega = p->omega;
    H->x_max = p->x_max;
    H->grid_size = p->grid_size;
    H->lambda_ = p->lambda_;
    H->mass = p->mass;
    H->f_max = p->f_max;
    H->n_actions = p->n_actions;
    H->server_pid = (int32_t)getpid();
    H->pid_ns = qcs_pid_ns();
    H->r_on = s->resident ? 1u : 0u;
    H->r_dt = s->cur_dt;
    H->r_gamma = s->cur_gamma;
    s->served.assign(P, 0u);
    s->pre_ok.assign(P, 0);
    __atomic_store_n(&H->alive, 1u, __ATOMIC_SEQ_CST);
    *out = s;
    return QC_OK;
}

int qc_server_run(qc_server* s, double seconds) {
    if (!s) return QC_EINVAL;
    if (hipSetDevice(s->device) != hipSuccess) return sfail(s, QC_EHIP, "hipSetDevice");
    const double t_end = seconds > 0 ? now_us() + seconds * 1e6 : 1e300;
    std::vector<int> pend;
    int owned = 0;
    double idle_since = now_us(), last_reap = now_us();
    resident_tend(s, now_us());
    while (!s->stop.load(std::memory_order_relaxed) && now_us() < t_end) {
        resident_tend(s, now_us());
        if (now_us() - last_reap > 100000.0) {   // every 0.1 s
            reap_dead_clients(s);
            last_reap = now_us();
        }
        scan(s, pend, owned);
        if (pend.empty()) {
            if (now_us() - idle_since < 200.0) {   // short spin: the next request is usually microseconds away
                for (int i = 0; i < 64; ++i) cpu_relax();
                continue;
            }
            // asleep until a client kicks (or 2 ms; with a resident kernel until its lease is up, then in 20 us steps
            // until it has drained): a client posting while server_sleeping is set wakes us
            const uint32_t k = __atomic_load_n(&s->hdr->kick, __ATOMIC_SEQ_CST);
            __atomic_store_n(&s->hdr->server_sleeping, 1u, __ATOMIC_SEQ_CST);
            scan(s, pend, owned);
            long ns = 2000000L;
            if (s->r_running) ns = std::min(ns, std::max(20000L, (long)((s->t_lease - now_us()) * 1e3)));
            if (pend.empty()) futex_wait(&s->hdr->kick, k, ns);
            __atomic_store_n(&s->hdr->server_sleeping, 0u, __ATOMIC_SEQ_CST);
            continue;
        }
        // batch: wait (briefly) for the other owned slots' requests of this tick (with the resident path the ticks
        // carry only the rare calls — set_seed, x_expectation, ... — which do not come together: no wait)
        const double t0 = now_us();
        while (!s->resident && (int)pend.size() < owned && now_us() - t0 < s->wait_us) {
            for (int i = 0; i < 32; ++i) cpu_relax();
            scan(s, pend, owned);
        }
        s->t_wait += now_us() - t0;
        serve_tick(s, pend);
        idle_since = now_us();
    }
    resident_stop(s);
    return QC_OK;
}

int qc_server_stop(qc_server* s) {
    if (!s) return QC_EINVAL;
    s->stop.store(1);
    if (s->hdr) futex_wake(&s->hdr->kick, 1);
    return QC_OK;
}

int qc_server_stats(const qc_server* s, int64_t* ticks, int64_t* calls) {
    if (!s) return QC_EINVAL;
    if (ticks) *ticks = s->ticks;
    if (calls) *calls = s->calls;
    return QC_OK;
}

int qc_server_timing(const qc_server* s, double* out) {
    if (!s || !out) return QC_EINVAL;
    out[0] = s->t_wait;
    out[1] = s->t_launch;
    out[2] = s->t_gpu;
    out[3] = s->t_publish;
    return QC_OK;
}

int qc_server_resident(const qc_server* s, int64_t* calls, int64_t* launches) {
    if (!s) return QC_EINVAL;
    int64_t n = 0;
    for (int e = 0; e < s->P; ++e) n += __atomic_load_n(&s->slots[e].rcount, __ATOMIC_ACQUIRE);
    if (calls) *calls = n;
    if (launches) *launches = s->launches;
    return s->resident ? 1 : 0;
}

const char* qc_server_last_error(const qc_server* s) { return s ? s->err.c_str() : ""; }

void qc_server_destroy(qc_server* s) {
    if (!s) return;
    free_server(s);
    delete s;
}

}  // extern "C"
