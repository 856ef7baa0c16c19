/*
 * qcart_client.h — C ABI of libqcart_client.so, the actor-process side of the step server.
 *
 * The reference runs 30-40 actor processes, each importing its own `simulation` extension and calling
 * step(state, dt, force, gamma) on ONE env per call (IHO/main_parallel.py:345-359, :264; the module's method
 * table IHO/simulation_i.cpp:618-631, QO/simulation_quart.cpp:656-668). Under the step server (qc_server_*,
 * include/qcart.h) one process owns the GPU and these calls become requests in a shared-memory slot: every
 * pending env of a tick is stepped in one batched launch. This library is plain C (POSIX shared memory +
 * futexes): a client process never creates a HIP context.
 *
 * All state pointers are HOST pointers: psi = one env's complex128 state, [N] interleaved (re, im), mutated in
 * place like the reference's numpy `state`. Return value 0 on success, < 0 on error; qcc_last_error explains.
 *
 * A call copies the state into the slot's row, publishes the request and polls its done word before sleeping on
 * the server's tick futex: QCC_SPIN_US microseconds (environment variable read at qcc_open), by default 150 while
 * the attached clients have a usable CPU each (affinity mask capped by the cgroup CPU quota) and 20 once they
 * outnumber them (spinning clients would take the CPU from those whose tick has completed).
 */
#ifndef QCART_CLIENT_H
#define QCART_CLIENT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum qcc_status {
    QCC_OK = 0,
    QCC_EINVAL = -1,      /* bad argument (reference: ValueError) */
    QCC_ENOSERVER = -7,   /* no live server object of that name, or the server stopped */
    QCC_EFULL = -8        /* every client slot of the server is owned */
};

typedef struct qcc qcc;

/* `import simulation` in an actor (IHO/main_parallel.py:174): attach to the server object `name` (a POSIX
 * shared-memory name, "/..."), claiming one free client slot (= one env of the server's batch). The env
 * starts on seed 0's MT19937 stream until qcc_set_seed. */
int qcc_open(const char* name, qcc** out);
void qcc_close(qcc* c);
const char* qcc_last_error(const qcc* c);   /* c may be NULL: the last qcc_open failure */

/* check_settings() (IHO/simulation_i.cpp:581-583, QO/simulation_quart.cpp:652-654): out[9] = n_max, omega,
 * x_max, grid_size, lambda, mass, moment_order, f_max, n_actions of the server's module */
int qcc_settings(const qcc* c, double* out);
int qcc_dim(const qcc* c);      /* N */
int qcc_n_obs(const qcc* c);    /* 5 (Fock 'xp') or (2+m+1)m/2 (grid get_moments) */
int qcc_family(const qcc* c);   /* enum qc_family */
int qcc_slot(const qcc* c);     /* this client's env index in the server's batch */

/* step(state, dt, force, gamma) (n = 1; IHO/simulation_i.cpp:358-389, QO/simulation_quart.cpp:493-525) and
 * simulate_10_steps (n = 10, Fail of the final state; IHO:391-421, QO:526-558): psi advanced in place; the
 * last step's q and x_mean and Fail written to *q, *xmean, *fail (each may be NULL). */
int qcc_step(qcc* c, double* psi, int32_t n, double dt, double force, double gamma, double* q, double* xmean,
             int32_t* fail);
/* set_seed(seed) (IHO/simulation_i.cpp:574-579): this env's MT19937 stream restarts at vslNewStream(seed) */
int qcc_set_seed(qcc* c, uint32_t seed);
/* x_expectation(state) (IHO/simulation_i.cpp:204-215, QO/simulation_quart.cpp:244-258) */
int qcc_x_expectation(qcc* c, const double* psi, double* out);
/* get_moments(state, data) (grid: QO/simulation_quart.cpp:326-388, n_obs values) or the Fock 'xp' 5-vector
 * (IHO/main_parallel.py:129-131) */
int qcc_moments(qcc* c, const double* psi, double* out);
/* Hamiltonian_dot_psi(state) (Fock modules; IHO/simulation_i.cpp:585-601, HO/simulation.cpp:566-582): psi <- H psi
 * in place with the force-free Hamiltonian */
int qcc_hamiltonian_dot_psi(qcc* c, double* psi);

#ifdef __cplusplus
}
#endif

#endif
