/*
 * qcart_client.c — libqcart_client.so: the actor-process side of the step server (qcart_server.cpp).
 * Plain C over POSIX shared memory and futexes: no HIP, no GPU context in the client process (the reference's
 * actors each own a CPU-only `simulation` module; here they own one slot of the server's batch).
 * Protocol and layout: qcart_shm.h. A call copies the state into the slot's row, publishes req + 1, and waits
 * (a short spin, then a futex on the header's tick word) until the server has published done = req.
 * step(state, dt, force, gamma) on the action grid goes to the server's resident kernel when it has one (r_on): the
 * same row, rreq + 1, and a poll of rdone that the GPU writes (no futex: the GPU cannot wake one; past the usable
 * CPUs the poll yields its CPU). A request the kernel does not take (QCS_EBOUNCE) is sent through the ticks.
 */
#define _GNU_SOURCE
#include <errno.h>
#include <math.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include "../../include/qcart_client.h"
#include "qcart_shm.h"

struct qcc {
    int fd;
    size_t bytes;
    unsigned char* shm;
    qcs_header* hdr;
    qcs_slot* slot;
    double* psi;   /* this slot's state row [2N] */
    double* obs;   /* this slot's observation row [QCS_MAX_OBS] */
    int index;
    double spin_s;   /* how long a call polls its done word before sleeping on the tick word (< 0: adaptive) */
    int cpus;        /* usable host CPUs (affinity mask, capped by the cgroup CPU quota) */
    int row_kept;    /* the slot's row is the one the resident wave returned last (no call since wrote it) */
    uint32_t last_rep;   /* the stream epoch this client's last resident step carried */
    char err[160];
};

static char g_err[160];

static int rcall(qcc* c, int op, int act, uint32_t gen, int keep);

static void set_err(qcc* c, const char* m) {
    snprintf(c ? c->err : g_err, sizeof(g_err), "%s", m);
}

/* usable CPUs: the affinity mask, capped by a cgroup v2 CPU quota (cpu.max "quota period") */
static int usable_cpus(void) {
    cpu_set_t set;
    int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set) : 1;
    FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r");
    if (f) {
        char q[32] = {0};
        long period = 0;
        if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
            const long lim = (atol(q) + period - 1) / period;
            if (lim > 0 && lim < n) n = (int)lim;
        }
        fclose(f);
    }
    return n < 1 ? 1 : n;
}

/* the server is gone: it cleared `alive` (qc_server_destroy), or its process no longer exists (killed, aborted on
 * a GPU fault: `alive` is never cleared then) */
static int server_gone(const qcs_header* h) {
    if (!__atomic_load_n(&h->alive, __ATOMIC_ACQUIRE)) return 1;
    const int32_t pid = h->server_pid;
    return pid > 0 && kill(pid, 0) != 0 && errno == ESRCH;
}

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

int qcc_open(const char* name, qcc** out) {
    if (!out || !name) return QCC_EINVAL;
    *out = NULL;
    int fd = shm_open(name, O_RDWR, 0);
    if (fd < 0) {
        snprintf(g_err, sizeof(g_err), "no step server at %s (shm_open: %s)", name, strerror(errno));
        return QCC_ENOSERVER;
    }
    struct stat sb;
    if (fstat(fd, &sb) != 0 || (size_t)sb.st_size < sizeof(qcs_header)) {
        close(fd);
        snprintf(g_err, sizeof(g_err), "%s is not a step-server object", name);
        return QCC_ENOSERVER;
    }
    unsigned char* m = (unsigned char*)mmap(NULL, (size_t)sb.st_size, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) {
        close(fd);
        snprintf(g_err, sizeof(g_err), "mmap: %s", strerror(errno));
        return QCC_ENOSERVER;
    }
    qcs_header* h = (qcs_header*)m;
    if (h->magic != QCS_MAGIC || h->version != QCS_VERSION || h->total_bytes != (uint64_t)sb.st_size ||
        server_gone(h)) {
        munmap(m, (size_t)sb.st_size);
        close(fd);
        snprintf(g_err, sizeof(g_err), "%s: no live step server (version / state mismatch, or its process exited)",
                 name);
        return QCC_ENOSERVER;
    }
    if (h->pid_ns != qcs_pid_ns()) {
        /* pids (the server's liveness check of its clients, and ours of it) mean nothing across PID namespaces */
        munmap(m, (size_t)sb.st_size);
        close(fd);
        snprintf(g_err, sizeof(g_err), "%s: the step server runs in another PID namespace", name);
        return QCC_ENOSERVER;
    }
    qcs_slot* slots = (qcs_slot*)(m + h->slot_off);
    int idx = -1;
    for (int e = 0; e < h->max_clients && idx < 0; ++e) {
        uint32_t z = 0;
        if (__atomic_compare_exchange_n(&slots[e].owner, &z, 1u, 0, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED)) idx = e;
    }
    if (idx < 0) {
        snprintf(g_err, sizeof(g_err), "%s: all %d client slots are taken", name, h->max_clients);
        munmap(m, (size_t)sb.st_size);
        close(fd);
        return QCC_EFULL;
    }
    qcc* c = (qcc*)calloc(1, sizeof(qcc));
    c->fd = fd;
    c->bytes = (size_t)sb.st_size;
    c->shm = m;
    c->hdr = h;
    c->slot = &slots[idx];
    c->index = idx;
    {
        /* QCC_SPIN_US: a tick is tens of microseconds, a futex wake-up adds its own; the default polls for 150 us */
        const char* v = getenv("QCC_SPIN_US");
        c->spin_s = v && *v ? atof(v) * 1e-6 : -1.0;
        c->cpus = usable_cpus();
    }
    c->psi = (double*)(m + h->psi_off) + (size_t)idx * 2 * (size_t)h->N;
    c->obs = (double*)(m + h->obs_off) + (size_t)idx * QCS_MAX_OBS;
    c->slot->pid = (int32_t)getpid();
    __atomic_add_fetch(&h->n_clients, 1u, __ATOMIC_SEQ_CST);
    c->last_rep = c->slot->repoch;
    if (__atomic_load_n(&h->r_on, __ATOMIC_ACQUIRE)) {
        /* what the resident wave holds for this slot (a pair drawn ahead, a kept row) is the previous owner's */
        const int rc = rcall(c, QCS_ROP_RESET, 0, 0u, 0);
        if (rc && rc != QCS_EBOUNCE) {   /* (the grid kernels answer every non-step op with a bounce) */
            snprintf(g_err, sizeof(g_err), "%s", c->err);
            qcc_close(c);
            return rc;
        }
    }
    /* the env starts on seed 0's stream, whatever an earlier owner of the slot left (the plain drop-in's state
     * before the first set_seed) */
    const int rc = qcc_set_seed(c, 0u);
    if (rc) {
        snprintf(g_err, sizeof(g_err), "%s", c->err);
        qcc_close(c);
        return rc;
    }
    *out = c;
    return QCC_OK;
}

void qcc_close(qcc* c) {
    if (!c) return;
    /* a request still pending is completed first (its slot must not be re-claimed mid-tick), unless the server is
     * gone; bounded, so a close (also from a destructor) never hangs on a server that stopped answering */
    const double t0 = now_s();
    while ((__atomic_load_n(&c->slot->done, __ATOMIC_ACQUIRE) != __atomic_load_n(&c->slot->req, __ATOMIC_RELAXED) ||
            __atomic_load_n(&c->slot->rdone, __ATOMIC_ACQUIRE) != __atomic_load_n(&c->slot->rreq, __ATOMIC_RELAXED)) &&
           !server_gone(c->hdr) && now_s() - t0 < 60.0)
        usleep(100);
    c->slot->pid = 0;
    __atomic_sub_fetch(&c->hdr->n_clients, 1u, __ATOMIC_SEQ_CST);
    __atomic_store_n(&c->slot->owner, 0u, __ATOMIC_RELEASE);
    munmap(c->shm, c->bytes);
    close(c->fd);
    free(c);
}

const char* qcc_last_error(const qcc* c) { return c ? c->err : g_err; }
int qcc_dim(const qcc* c) { return c ? c->hdr->N : QCC_EINVAL; }
int qcc_n_obs(const qcc* c) { return c ? c->hdr->n_obs : QCC_EINVAL; }
int qcc_family(const qcc* c) { return c ? c->hdr->family : QCC_EINVAL; }
int qcc_slot(const qcc* c) { return c ? c->index : QCC_EINVAL; }

int qcc_settings(const qcc* c, double* out) {
    if (!c || !out) return QCC_EINVAL;
    const qcs_header* h = c->hdr;
    out[0] = h->n_max;
    out[1] = h->omega;
    out[2] = h->x_max;
    out[3] = h->grid_size;
    out[4] = h->lambda_;
    out[5] = h->mass;
    out[6] = h->moment_order;
    out[7] = h->f_max;
    out[8] = h->n_actions;
    return QCC_OK;
}

/* the force's index on the server's action grid (its slot_of), or -1: off the grid (a custom slot, the ticks) */
static int grid_action(const qcs_header* h, double force) {
    const int half = h->n_actions / 2;
    if (half <= 0) return -1;
    const double spacing = h->f_max / half;
    const double a = nearbyint(force / spacing);
    if (a >= -half && a <= half && a * spacing == force) return (int)a + half;
    return -1;
}

/* post a resident request (the whole request in the rreq word, qcart_shm.h QCS_RQ) and poll for its results */
static int rcall(qcc* c, int op, int act, uint32_t gen, int keep) {
    qcs_slot* s = c->slot;
    qcs_header* h = c->hdr;
    const uint32_t prev = __atomic_load_n(&s->rreq, __ATOMIC_RELAXED);
    if (op == QCS_ROP_STEP && s->repoch != c->last_rep && ((s->repoch - c->last_rep) & QCS_RQ_EP_MASK) == 0)
        s->repoch++;   /* tick-path draws since the last resident step must show in the word's 15 epoch bits */
    const uint32_t r = QCS_RQ((prev & 3u) + 1u, op, act, gen, s->repoch, keep);
    __atomic_store_n(&s->rreq, r, __ATOMIC_SEQ_CST);
    /* more clients than usable CPUs: a polling client gives its CPU to the others (sched_yield) */
    const int yield = (int)__atomic_load_n(&h->n_clients, __ATOMIC_RELAXED) > c->cpus;
    double t0 = 0.0, tl = 0.0;
    for (uint32_t i = 0;; ++i) {
        if (__atomic_load_n(&s->rdone, __ATOMIC_ACQUIRE) == r) {
            const int st = s->rstatus;
            if (st == QCS_EDROPPED) set_err(c, "request dropped by the step server");
            return st;
        }
        if (yield) sched_yield();
        else __builtin_ia32_pause();
        if ((i & 255u) == 255u) {
            const double t = now_s();
            if (t0 == 0.0) t0 = tl = t;
            if (t - tl > 0.02) {   /* the server's liveness, as in call() */
                tl = t;
                if (server_gone(h)) {
                    set_err(c, __atomic_load_n(&h->alive, __ATOMIC_ACQUIRE) ? "the step server's process exited"
                                                                            : "the step server stopped");
                    return QCC_ENOSERVER;
                }
            }
            if (t - t0 > 600.0) {
                set_err(c, "no answer from the step server's resident kernel in 600 s");
                return QCC_ENOSERVER;
            }
        }
    }
}

/* post the slot's filled request and wait for its results */
static int call(qcc* c) {
    qcs_slot* s = c->slot;
    qcs_header* h = c->hdr;
    const uint32_t r = __atomic_load_n(&s->req, __ATOMIC_RELAXED) + 1u;
    __atomic_store_n(&s->req, r, __ATOMIC_SEQ_CST);
    if (__atomic_load_n(&h->server_sleeping, __ATOMIC_SEQ_CST)) {
        __atomic_add_fetch(&h->kick, 1u, __ATOMIC_SEQ_CST);
        syscall(SYS_futex, &h->kick, FUTEX_WAKE, 1, NULL, NULL, 0);
    }
    /* a short spin (a tick takes tens of microseconds), then sleep on the tick word. Adaptive (no QCC_SPIN_US):
     * 150 us while every attached client has a CPU of its own (P = 16 at n_max = 180: 4.9e5 step calls/s against
     * 3.5e5 with 20 us), none once they outnumber the usable CPUs — the reference's 30-40 actors on a 16-CPU share,
     * where a polling client takes the CPU from the ones whose tick has completed (P = 40 at n_max = 180: 6.0e5 with
     * no poll, 5.5e5 with 20 us, 4.2e5 with 50 us; round 5: 150 us 3.2e5) */
    double spin = c->spin_s;
    if (spin < 0) spin = (int)__atomic_load_n(&h->n_clients, __ATOMIC_RELAXED) <= c->cpus ? 150e-6 : 0.0;
    const double t0 = now_s();
    for (int i = 0;; ++i) {
        if (__atomic_load_n(&s->done, __ATOMIC_ACQUIRE) == r) {
            if (s->status) set_err(c, s->err);
            return s->status;
        }
        __builtin_ia32_pause();
        if ((i & 31) == 31 && now_s() - t0 > spin) break;
    }
    for (;;) {
        __atomic_store_n(&s->waiting, 1u, __ATOMIC_SEQ_CST);
        const uint32_t t = __atomic_load_n(&h->tick, __ATOMIC_SEQ_CST);
        if (__atomic_load_n(&s->done, __ATOMIC_SEQ_CST) == r) break;
        struct timespec ts = {0, 20000000L};   /* 20 ms: re-check the server's liveness */
        syscall(SYS_futex, &h->tick, FUTEX_WAIT, t, &ts, NULL, 0);
        if (__atomic_load_n(&s->done, __ATOMIC_ACQUIRE) == r) break;
        if (server_gone(h)) {
            __atomic_store_n(&s->waiting, 0u, __ATOMIC_RELAXED);
            set_err(c, __atomic_load_n(&h->alive, __ATOMIC_ACQUIRE) ? "the step server's process exited"
                                                                    : "the step server stopped");
            return QCC_ENOSERVER;
        }
        if (now_s() - t0 > 600.0) {
            __atomic_store_n(&s->waiting, 0u, __ATOMIC_RELAXED);
            set_err(c, "no answer from the step server in 600 s");
            return QCC_ENOSERVER;
        }
    }
    __atomic_store_n(&s->waiting, 0u, __ATOMIC_RELAXED);
    if (s->status) set_err(c, s->err);
    return s->status;
}

int qcc_step(qcc* c, double* psi, int32_t n, double dt, double force, double gamma, double* q, double* xmean,
             int32_t* fail) {
    if (!c || !psi || (n != 1 && n != 10)) return QCC_EINVAL;
    const size_t bytes = sizeof(double) * 2 * (size_t)c->hdr->N;
    /* keep: the previous call was a resident step and the state still equals the row it returned (the resident wave
     * then takes its LDS copy of that row instead of reading ours over PCIe) */
    const int keep = c->row_kept && memcmp(c->psi, psi, bytes) == 0;
    if (!keep) memcpy(c->psi, psi, bytes);
    c->row_kept = 0;
    qcs_slot* s = c->slot;
    s->op = QCS_OP_STEP;
    s->n = n;
    s->dt = dt;
    s->force = force;
    s->gamma = gamma;
    int rc = QCS_EBOUNCE;
    const qcs_header* h = c->hdr;
    if (n == 1 && __atomic_load_n(&h->r_on, __ATOMIC_ACQUIRE)) {
        /* dt and gamma as the server's under generation gen: the request carries gen, and a resident kernel of
         * another generation bounces it */
        const uint32_t gen = __atomic_load_n(&h->r_gen, __ATOMIC_ACQUIRE);
        const int act = grid_action(h, force);
        if (act >= 0 && dt == h->r_dt && gamma == h->r_gamma) {
            rc = rcall(c, QCS_ROP_STEP, act, gen, keep);
            if (rc == QCC_OK) {
                c->row_kept = 1;
                c->last_rep = s->repoch;
            }
        }
    }
    if (rc == QCS_EBOUNCE) {   /* the ticks (a bounced request left the row untouched); they take stream words */
        s->repoch++;
        rc = call(c);
    }
    if (rc) return rc;
    memcpy(psi, c->psi, bytes);
    if (q) *q = s->q;
    if (xmean) *xmean = s->xmean;
    if (fail) *fail = s->fail;
    return QCC_OK;
}

int qcc_set_seed(qcc* c, uint32_t seed) {
    if (!c) return QCC_EINVAL;
    c->row_kept = 0;
    c->slot->op = QCS_OP_SET_SEED;
    c->slot->seed = seed;
    c->slot->repoch++;   /* a pair the resident wave drew ahead belongs to the old stream */
    return call(c);
}

/* x_expectation / the observation vector: on the resident kernel when the server has one (the stream and the row the
 * wave keeps stay as they are: a kept row stays kept), else in a tick */
static int obs_call(qcc* c, const double* psi, int rop, int op) {
    const size_t bytes = sizeof(double) * 2 * (size_t)c->hdr->N;
    const int keep = c->row_kept && memcmp(c->psi, psi, bytes) == 0;
    if (!keep) memcpy(c->psi, psi, bytes);
    c->row_kept = keep;
    /* (the grid's resident kernel bounces them: its moments stay in the ticks) */
    if (__atomic_load_n(&c->hdr->r_on, __ATOMIC_ACQUIRE) && c->hdr->family <= 1) {
        const int rc = rcall(c, rop, 0, 0u, keep);
        if (rc != QCS_EBOUNCE) return rc;
    }
    c->row_kept = 0;
    c->slot->op = op;
    return call(c);
}

int qcc_x_expectation(qcc* c, const double* psi, double* out) {
    if (!c || !psi || !out) return QCC_EINVAL;
    const int rc = obs_call(c, psi, QCS_ROP_X_EXPECT, QCS_OP_X_EXPECT);
    if (rc == QCC_OK) *out = c->slot->value;
    return rc;
}

int qcc_moments(qcc* c, const double* psi, double* out) {
    if (!c || !psi || !out) return QCC_EINVAL;
    const int rc = obs_call(c, psi, QCS_ROP_OBS, c->hdr->family >= 2 ? QCS_OP_MOMENTS : QCS_OP_FOCK_OBS);
    if (rc == QCC_OK) memcpy(out, c->obs, sizeof(double) * (size_t)c->hdr->n_obs);
    return rc;
}

int qcc_hamiltonian_dot_psi(qcc* c, double* psi) {
    if (!c || !psi) return QCC_EINVAL;
    if (c->hdr->family >= 2) {
        set_err(c, "Hamiltonian_dot_psi is a Fock-module function");
        return QCC_EINVAL;
    }
    const size_t bytes = sizeof(double) * 2 * (size_t)c->hdr->N;
    c->row_kept = 0;
    memcpy(c->psi, psi, bytes);
    c->slot->op = QCS_OP_HDOT;
    const int rc = call(c);
    if (rc == QCC_OK) memcpy(psi, c->psi, bytes);
    return rc;
}
