/*
 * qcart_oracle.h — TEST INFRASTRUCTURE ONLY (the parity checker; never shipped, never on the product path).
 *
 * A CPU fp64 restatement of the reference quantum-cartpole stepper
 * (Z-T-WANG/DeepReinforcementLearningControlOfQuantumCartpoles, "implementation codes/"):
 *   HO  = harmonic oscillator/simulation.cpp
 *   IHO = inverted harmonic oscillator/simulation_i.cpp
 *   QO  = quartic oscillator/simulation_quart.cpp (byte-identical to the IQO copy)
 * plus the Python-side observation / termination / reset helpers of each family main_parallel.py.
 *
 * PARITY STATUS: pinned at the reference's MKL boundary; the reference binary itself never ran.
 * Compiling or running the reference extension was denied in this environment and
 * the reference ships no golden vectors or tests. The MKL 2021.4 runtime the reference
 * links is driven through ctypes in the reference's call order and descriptors (tests/golden/mklref.py,
 * make_mkl_fixtures.py -> mkl_v1.npz): this restatement equals it (tests/test_mkl_fixtures.py: MT19937
 * words bit for bit, Box-Muller <= 2 ulp, zgbtrf pivots / zgbtrs solves, the HERMITIAN-descriptor term7,
 * the DIAG_UNIT p relative, 1000-step MKL-ordered trajectories to 1e-9). Also pinned by physics
 * known-answer tests (tests/test_oracle_kat.py: dense-numpy operators built from the reference's
 * own Python operator definitions, unitary expm propagation, Gaussian moments, norm, pivot-free LU)
 * and guarded against drift by the committed fixtures it generated (tests/golden/golden_v1.npz).
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 */
#ifndef QCART_ORACLE_H
#define QCART_ORACLE_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { QO_HO = 0, QO_IHO = 1, QO_QO = 2, QO_IQO = 3 };

typedef struct qo_params {
    int32_t family;        /* QO_HO / QO_IHO (Fock basis), QO_QO / QO_IQO (8th-order FD grid)   */
    int32_t n_max;         /* Fock: N = n_max + 1                                               */
    double omega;          /* Fock: omega (the drivers pass pi)                                 */
    double x_max, grid_size, lambda_, mass;  /* grid: x_n = 2*int(x_max/h + 0.5) + 1           */
    int32_t moment_order;  /* grid moments order (reference MOMENT macro, default 5)            */
    int32_t a_mode;        /* 0: reference sparse-descriptor semantics (App. C H1), 1: exact A  */
} qo_params;

typedef struct qo_sys qo_sys;
typedef struct qo_tab qo_tab;

qo_sys* qo_create(const qo_params* p);
void qo_destroy(qo_sys* s);
int qo_dim(const qo_sys* s);          /* N (Fock) or x_n (grid) */
int qo_n_obs(const qo_sys* s);        /* 5 (Fock 'xp') or (2+m+1)*m/2 (grid) */

/* reset_ab(): LU of ab = I + i dt/2 (H - c F X) (LAPACK zgbtrf semantics, partial pivoting) and the
 * dt^3..dt^6 correction factor A. Returns NULL on failure. n_swaps receives the pivot count. */
qo_tab* qo_make_tab(const qo_sys* s, double dt, double force, int* n_swaps);
void qo_free_tab(qo_tab* t);

/* go_one_step() + check_boundary_error(); r = the two N(0,1) draws of the step. */
void qo_step(const qo_sys* s, const qo_tab* t, double* psi, double dt, double force, double gamma,
             const double r[2], double* q, double* x_mean, int* fail);

double qo_x_expectation(const qo_sys* s, const double* psi);
void qo_moments(const qo_sys* s, const double* psi, double* out);           /* fp64 obs vector */
double qo_outside_prob(const qo_sys* s, const double* psi, double xth);     /* IQO termination */
int qo_boundary_fail(const qo_sys* s, const double* psi);
double qo_energy(const qo_sys* s, const double* psi);                       /* Re<H>*w (F=0) */
double qo_phonon(const qo_sys* s, const double* psi);                       /* Fock <n> */

/* dense operator export for KAT tests: out[N*N] real */
void qo_dense_h(const qo_sys* s, double* out);
void qo_dense_x(const qo_sys* s, double* out);
/* complex band-LU pieces of a table: ab_lu (column-major LAPACK AB, ldab x N, complex) */
int qo_tab_ldab(const qo_tab* t);
void qo_tab_export(const qo_tab* t, double* ab_lu, int32_t* ipiv, double* a_band);

/* MKL-boundary pieces (tests/test_mkl_fixtures.py): term7 = A . v under the a_mode semantics (IHO:551),
 * the band solve in place (zgbtrs, IHO:487), the grid (p_hat - pbar I) v of compute_statistics (QO:337) */
void qo_term7(const qo_sys* s, const qo_tab* t, const double* v, double* y);
void qo_tab_solve(const qo_tab* t, double* b);
void qo_grid_p_apply(const qo_sys* s, const double* v, double pbar, double* out);

/* counter-based noise shared with the product: Philox4x32-10 */
void qo_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
void qo_normals(uint64_t seed, uint64_t env_id, uint64_t step, double r[2]);
/* the reference's stream: MT19937 init_by_array({seed}) + MKL Box-Muller; st uint32 [625] */
void qo_mt_seed(uint32_t seed, uint32_t* st);
uint32_t qo_mt_next(uint32_t* st);
void qo_mt_normals(uint32_t* st, int64_t n, double* out);
void qo_fock_random_state(const qo_sys* s, uint64_t seed, uint64_t env_id, int levels, double* psi);
void qo_gaussian_packet(const qo_sys* s, double wavenumber, double mean, double stdv, double* psi);

/* batched CPU driver (the cpu_baseline): B envs, env e uses action act[e] -> force (a-10)*F_max/10,
 * noise qo_normals(seed, env_offset+e, step0+k). OpenMP over envs when built with -fopenmp.
 * fail_step[e] = first 1-based step with Fail, 0 otherwise. q_out/xm_out [n_steps][B] may be NULL. */
int qo_run_batch(const qo_sys* s, double* psi, int64_t B, const int32_t* act, double f_max,
                 int n_steps, double dt, double gamma, uint64_t seed, int64_t env_offset,
                 uint64_t step0, int32_t* fail_step, double* q_out, double* xm_out, int n_threads);
/* same but with injected noise: noise[k][e][2] */
int qo_run_batch_noise(const qo_sys* s, double* psi, int64_t B, const int32_t* act, double f_max,
                       int n_steps, double dt, double gamma, const double* noise,
                       int32_t* fail_step, double* q_out, double* xm_out, int n_threads);

#ifdef __cplusplus
}
#endif
#endif
