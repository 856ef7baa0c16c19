/*
 * qcart_shm.h — the shared-memory protocol between the step server (qcart_server.cpp, inside libqcart.so, the
 * one process that owns the GPU) and its actor-process clients (qcart_client.c, libqcart_client.so: plain C, no
 * HIP). It reproduces the reference's process model — 30-40 actor processes, each calling its own `simulation`
 * module on one env (IHO/main_parallel.py:345-359, :264) — with every pending env of a tick stepped in ONE
 * batched launch on the server's handle (env e = client slot e).
 *
 * One POSIX shared-memory object /dev/shm/<name>:
 *   [qcs_header][qcs_slot x max_clients][psi: max_clients x N complex128][obs: max_clients x kQcsMaxObs fp64]
 * A client owns its slot's request fields, its psi row and obs row between calls; the server reads them only
 * while the slot has a pending request (req != done) and writes the results before publishing done = req.
 * Synchronisation: GCC __atomic builtins (C and C++ alike) on 32-bit words; sleeping sides wait on futexes of
 * the shared mapping (clients on header.tick, the server on header.kick).
 */
#ifndef QCART_SHM_H
#define QCART_SHM_H

#include <stdint.h>
#include <sys/stat.h>

#define QCS_MAGIC 0x56534351u /* "QCSV" */
#define QCS_VERSION 3u
#define QCS_MAX_OBS 64        /* >= the largest n_obs ((2+9+1)*9/2 = 54 grid moments) */

/* request operations (the reference module's functions, IHO/simulation_i.cpp:618-631, QO/simulation_quart.cpp:656-668) */
enum qcs_op {
    QCS_OP_STEP = 1,       /* step(state, dt, force, gamma): n = 1; simulate_10_steps: n = 10 (Fail of the final state) */
    QCS_OP_SET_SEED = 2,   /* set_seed(seed): the env's MT19937 stream restarts */
    QCS_OP_X_EXPECT = 3,   /* x_expectation(state) */
    QCS_OP_MOMENTS = 4,    /* get_moments(state, data) (grid) */
    QCS_OP_FOCK_OBS = 5,   /* the Fock 'xp' 5-vector (IHO/main_parallel.py:129-131) */
    QCS_OP_HDOT = 6        /* Hamiltonian_dot_psi(state): the row <- H row (Fock; IHO/simulation_i.cpp:585-601) */
};

#define QCS_EDROPPED (-100)   /* a slot status: the server released the slot without serving the request */
#define QCS_EBOUNCE (-101)    /* a resident-path status: not served there (dt / gamma / action not the resident
                                 kernel's); the client sends the request through the tick path instead */

typedef struct qcs_header {
    uint32_t magic, version;
    int32_t max_clients, N, n_obs, family;
    uint32_t alive;          /* 1 while the server serves; 0 after it stopped (clients fail their calls) */
    uint32_t tick;           /* incremented (and futex-woken) after every served tick */
    uint32_t kick;           /* incremented (and futex-woken) by a client whose request finds the server asleep */
    uint32_t server_sleeping;
    uint32_t n_clients;      /* slots currently owned */
    int32_t server_pid;      /* the serving process: a client whose server died without clearing `alive` (killed,
                                aborted on a GPU fault) sees kill(server_pid, 0) fail with ESRCH */
    uint64_t slot_off, psi_off, obs_off, total_bytes;
    /* the module's compiled parameters (check_settings) */
    int32_t n_max, moment_order;
    double omega, x_max, grid_size, lambda_, mass, f_max;
    int32_t n_actions, pad1;
    uint64_t ticks, calls;   /* served ticks / requests (statistics, server-written) */
    uint64_t pid_ns;         /* inode of the server's PID namespace (/proc/self/ns/pid): pids are compared only
                                inside one namespace, so clients from another are refused */
    /* the resident path (qcart_server.cpp, k_resident): one wave per slot polls the slot's rreq word in this
     * device-mapped object and steps the env in place — no launch, no server thread in the call. r_on: the server
     * has a resident kernel for its module; a client sends step(state, dt, force, gamma) there when dt and gamma
     * are r_dt / r_gamma (read under the generation r_gen, which the request carries) and the force is on the action
     * grid (anything else: the tick path) */
    uint32_t r_on, r_gen;
    double r_dt, r_gamma;
    uint64_t r_pad1[8];      /* r_quit / r_beat on a line of their own: the GPU polls it, the clients never read it */
    uint32_t r_quit;         /* set by the server: every resident wave exits */
    uint32_t r_beat;         /* the server loop's heartbeat: the waves exit after ~1 s without a change */
    uint64_t r_pad2[7];
} qcs_header;

typedef struct qcs_slot {
    uint32_t owner;          /* 0 free, 1 owned (claimed by CAS in qcc_open) */
    int32_t pid;
    uint32_t req;            /* the client's request sequence number (incremented to post a request) */
    uint32_t done;           /* = req once the server has written the results */
    uint32_t waiting;        /* the client sleeps on header.tick */
    int32_t op, n;
    uint32_t seed;
    double dt, force, gamma;
    int32_t status;          /* 0 ok, < 0 a qc_status code (QCS_EDROPPED: the request was dropped unserved) */
    int32_t fail;            /* step: Fail */
    double q, xmean;         /* step: the last step's q and x_mean */
    double value;            /* x_expectation */
    char err[96];
    uint32_t rreq;           /* the resident request word QCS_RQ(seq, op, action, gen, epoch, keep) (client): the whole
                                request in the one word the wave polls */
    uint32_t rdone;          /* = rreq once the resident wave has written the results (device) */
    uint32_t repoch;         /* the env's stream epoch: + 1 by the client for every call that takes MT19937 words (or
                                reseeds) through the ticks, so the wave drops a pair it drew ahead */
    int32_t rstatus;         /* 0, or QCS_EBOUNCE / QCS_EDROPPED */
    uint32_t rcount;         /* requests the resident waves have answered for this slot (device; statistics) */
    uint8_t pad[12];
} qcs_slot;

/* the resident request word: a sequence (2 bits, + 1 per request: a word only has to differ from the one served
 * before it), the op (2 bits: QCS_ROP_*), the action slot (6 bits, < 64), the generation of the server's dynamics the
 * client checked (6 bits of r_gen), the env's stream epoch (15 bits of repoch; the client never lets two of its resident
 * steps carry equal epochs across tick-path draws, and a new owner of the slot first sends QCS_ROP_RESET) and `keep`:
 * the row is the one the wave returned last (the client's previous call was a resident step and its state array still
 * equals that row), so the wave may take it from its LDS copy instead of reading it over PCIe */
enum qcs_rop {
    QCS_ROP_STEP = 0,        /* step(state, dt, force, gamma) */
    QCS_ROP_X_EXPECT = 1,    /* x_expectation(state) -> value */
    QCS_ROP_OBS = 2,         /* get_moments (grid) / the Fock 'xp' 5-vector -> the slot's obs row */
    QCS_ROP_RESET = 3        /* a new owner: the wave drops the pair it drew ahead and the row it kept */
};
#define QCS_RQ(seq, op, act, gen, ep, keep) \
    (((uint32_t)(seq) & 3u) | (((uint32_t)(op) & 3u) << 2) | (((uint32_t)(act) & 63u) << 4) | \
     (((uint32_t)(gen) & 63u) << 10) | (((uint32_t)(ep) & 0x7fffu) << 16) | ((uint32_t)((keep) ? 1u : 0u) << 31))
#define QCS_RQ_EP_MASK 0x7fffu
#define QCS_RQ_OP(w) (((w) >> 2) & 3u)
#define QCS_RQ_ACT(w) (((w) >> 4) & 63u)
#define QCS_RQ_GEN(w) (((w) >> 10) & 63u)
#define QCS_RQ_EP(w) (((w) >> 16) & QCS_RQ_EP_MASK)
#define QCS_RQ_KEEP(w) ((w) >> 31)

/* inode of this process's PID namespace (0 if /proc is unavailable) */
static inline uint64_t qcs_pid_ns(void) {
    struct stat st;
    return stat("/proc/self/ns/pid", &st) == 0 ? (uint64_t)st.st_ino : 0u;
}

#endif
