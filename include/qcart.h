/*
 * qcart.h — C ABI of libqcart.so, the MI355X-native quantum-cartpole env.step() hot path.
 *
 * Drop-in boundary for the reference CPython extension `simulation` (one module per physical
 * system, compiled by each directory setupC.py with -D macros). Each entry point below names the reference
 * function it replaces (file:line; aliases as in SURVEY.md: HO/ IHO/ QO/ IQO/ =
 * "implementation codes/{harmonic, inverted harmonic, quartic, inverted quartic} oscillator/").
 *
 * Conventions
 *  - Plain C types only. Every psi / output pointer is a DEVICE pointer (hipMalloc'd or a torch
 *    tensor's data_ptr()) on the handle's device unless stated otherwise.
 *  - psi layout: [B][N] complex fp64, interleaved (re, im) — the numpy complex128 layout the
 *    reference takes (IHO/simulation_i.cpp:374-376), batched env-major.
 *  - All launches are asynchronous on the handle's stream (qc_set_stream; default: the null
 *    stream); qc_sync() fences.
 *  - Return value: 0 on success, < 0 on error (never aborts); qc_last_error() explains.
 *    Reference counterpart: Python exceptions (TypeError/ValueError/RuntimeError,
 *    IHO/simulation_i.cpp:340-372, QO/simulation_quart.cpp:288-323, :517).
 */
#ifndef QCART_H
#define QCART_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QC_ABI_VERSION 1

/* physical systems (one reference directory each) */
enum qc_family {
    QC_HO = 0,   /* harmonic cooling, Fock basis, H = omega (n + 1/2)       HO/simulation.cpp        */
    QC_IHO = 1,  /* inverted harmonic cartpole, H = -omega/2 (a+^2 + a^2)   IHO/simulation_i.cpp     */
    QC_QO = 2,   /* quartic cooling, 8th-order FD grid, lambda > 0          QO/simulation_quart.cpp  */
    QC_IQO = 3   /* inverted quartic cartpole, lambda < 0                   IQO/simulation_quart.cpp */
};

/* semantics of the dt^3..dt^6 correction product term7 = A . D1 */
enum qc_a_mode {
    QC_A_REFERENCE = 0, /* the reference's MKL descriptor: IHO HERMITIAN/UPPER mirror, others exact */
    QC_A_EXACT = 1      /* the intended complex-symmetric A                                          */
};

enum qc_status {
    QC_OK = 0,
    QC_EINVAL = -1,     /* bad argument / shape (reference: ValueError)                 */
    QC_ENOMEM = -2,
    QC_EHIP = -3,       /* HIP runtime error                                            */
    QC_EPIVOT = -4,     /* band LU would need row interchanges       */
    QC_ESINGULAR = -5,
    QC_ENOTBUILT = -6   /* no kernel instantiated for this (family, N)                  */
};

/* Runtime replacement of setupC.py's compile-time macros (HO/setupC.py:49, QO/setupC.py:55)
 * plus the per-call step() arguments dt / gamma that are fixed for a batch. */
/* working precision of the step (psi storage and arithmetic) */
enum qc_precision { QC_FP64 = 0, QC_FP32 = 1 };

typedef struct qc_params {
    int32_t family;        /* enum qc_family                                                     */
    int32_t n_max;         /* Fock: N = n_max + 1  (N_MAX macro)                                 */
    double omega;          /* Fock: OMEGA macro (the drivers pass pi)                           */
    double x_max;          /* grid: X_MAX;  x_n = 2*int(x_max/grid_size + 0.5) + 1              */
    double grid_size;      /* grid: GRID_SIZE (h)                                                */
    double lambda_;        /* grid: LAMBDA (already multiplied by pi, IQO/main_parallel.py:29)  */
    double mass;           /* grid: MASS (already divided by pi)                                 */
    int32_t moment_order;  /* grid: MOMENT macro (default 5 -> 20 observables); 1..16: up to 9 */
                           /* one observable per lane of the env's 64-lane wave, above that   */
                           /* up to 3 per lane ((2+m+1)m/2 <= 152) (QO/setupC.py:16,38        */
                           /* compiles any m >= 1; m >= 17 is refused, QC_EINVAL; the step    */
                           /* server serves m <= 9)                                           */
    int32_t a_mode;        /* enum qc_a_mode                                                     */
    double gamma;          /* measurement strength (step() argument; the drivers pass args.gamma*pi) */
    double dt;             /* time step (step() argument; 1/time_steps)                         */
    double f_max;          /* action -> force map F = (a - 10) * f_max / 10 (IHO/RL.py:107-111)  */
    int32_t n_actions;     /* 21 (2*10 + 1, IHO/RL.py:81,94)                                     */
    int32_t precision;     /* enum qc_precision: 0 fp64 (default, the reference's), 1 fp32 (config C5;
                              Fock families; psi buffers are then complex64)                     */
    int64_t batch;         /* B envs held by this handle (this rank's shard)                   */
    int64_t env_offset;    /* global id of env 0 (multi-GPU sharding keeps noise invariant)    */
    uint64_t seed;         /* Philox key (QC_NOISE_PHILOX; MT19937: qc_set_seed_mt19937)       */
    double xth;            /* IQO per-step outside-probability window half-width (0 = off)      */
} qc_params;

typedef struct qc_handle qc_handle;

/* Module init: Set_World ctor + PyInit (IHO/simulation_i.cpp:26-151, :643-653;
 * QO/simulation_quart.cpp:28-209). Builds the operator bands and the per-action factor tables
 * (reset_ab, IHO:227-277 / QO:394-432) for all n_actions forces on `device`. */
int qc_create(const qc_params* p, int device, qc_handle** out);
void qc_destroy(qc_handle* h);
const char* qc_last_error(const qc_handle* h);   /* h may be NULL: last qc_create failure */
int qc_abi_version(void);

/* check_settings() (IHO/simulation_i.cpp:581-583, QO/simulation_quart.cpp:652-654) */
int qc_get_params(const qc_handle* h, qc_params* out);
int qc_dim(const qc_handle* h);                  /* N = n_max+1 or x_n */
int qc_n_obs(const qc_handle* h);                /* 5 (Fock 'xp') or (2+m+1)*m/2 (grid) */

/* Stream binding (a hipStream_t passed as void*; NULL = default stream). */
int qc_set_stream(qc_handle* h, void* stream);
int qc_sync(qc_handle* h);

/* Noise of the stochastic step (the two N(0,1) draws per go_one_step, IHO/simulation_i.cpp:435).
 * Two sources, per handle:
 *   QC_NOISE_PHILOX   (default) counter-based Philox4x32-10 keyed by (seed, env_offset + e); env e's
 *                     counter is its own: it starts at 0 and advances by the steps env e takes, so an
 *                     env's trajectory never depends on the other envs of the handle or on sharding.
 *   QC_NOISE_MT19937  the reference's stream: set_seed(seed) = vslNewStream(VSL_BRNG_MT19937, seed) +
 *                     vdRngGaussian(VSL_RNG_METHOD_GAUSSIAN_BOXMULLER) (IHO/simulation_i.cpp:574-579,
 *                     :435), one stream per env (the reference runs one env per process with its own
 *                     seed, IHO/main_parallel.py:173-178,358): init_by_array({seed}), two words per
 *                     normal, x = sqrt(-2 ln u1) sin(2 pi u2), u = word * 2^-32 — MKL's uniform bits
 *                     exactly and its Gaussians to <= 1 ulp of the MKL_CBWR=COMPATIBLE path
 *                     (tests/golden/mkl_*.npz; MKL's default vector-math path differs by <= 5e-8).
 * An injected `noise` array in qc_step overrides both and advances neither stream. */
enum qc_noise_mode { QC_NOISE_PHILOX = 0, QC_NOISE_MT19937 = 1 };

/* set_seed(int) (IHO/simulation_i.cpp:574-579), Philox mode: re-keys the counter-based noise and resets
 * every env's counter to 0. */
int qc_set_seed(qc_handle* h, uint64_t seed);
/* set every env's Philox counter to `step` / read env 0's counter (synchronises) */
int qc_set_step_counter(qc_handle* h, uint64_t step);
uint64_t qc_get_step_counter(const qc_handle* h);
/* per-env Philox counters (device uint64 [B]): copied to `out` and/or replaced from `in` (either may be
 * NULL; checkpoint / resume of a batch) */
int qc_env_counters(qc_handle* h, uint64_t* out, const uint64_t* in);
/* set_seed for every env in MT19937 mode: seeds device uint32 [B], env e's stream
 * vslNewStream(VSL_BRNG_MT19937, seeds[e]) */
int qc_set_seed_mt19937(qc_handle* h, const uint32_t* seeds);
/* set_seed for the envs with mask[e] != 0 only (mask: device uint8 [B]); the others keep their streams — one
 * actor process's set_seed under the step server (qc_server_*). Needs the handle in MT19937 mode. */
int qc_set_seed_mt19937_envs(qc_handle* h, const uint32_t* seeds, const uint8_t* mask);
int qc_noise_mode(const qc_handle* h);
/* the next normals of every env's MT19937 stream (the reference's vdRngGaussian draws, IHO/simulation_i.cpp:435)
 * into `noise` (device double [n_steps][B][2], qc_step's injected layout): min(n_steps, env_steps[e]) steps for env e (env_steps NULL: n_steps each), the stream advancing by the
 * words drawn — what qc_step draws itself when it is given no noise. With pre / has_pre (device double [B][2], uint8
 * [B]; both or neither) an env with has_pre[e] != 0 has already drawn its next step's pair into pre[e] (an earlier
 * call with n_steps = 1): it becomes step 0 and only the remaining steps are drawn. The step server prefetches each
 * env's next pair this way after a tick, off the next tick's critical path. */
int qc_mt19937_normals(qc_handle* h, int32_t n_steps, const int32_t* env_steps, const double* pre,
                       const uint8_t* has_pre, double* noise);
/* per-env MT19937 states (device uint32 [B][qc_mt19937_words()]: 624 state words, read index, pad):
 * copied to `out` and/or replaced from `in` */
int qc_mt19937_state(qc_handle* h, uint32_t* out, const uint32_t* in);
int qc_mt19937_words(void);

/* Change dt / gamma (step()'s per-call arguments; reset_ab on dt change, IHO:377-383). */
int qc_set_dynamics(qc_handle* h, double dt, double gamma);

/* Register an arbitrary force (step(state, dt, force, gamma) with a force off the 21-level grid,
 * e.g. the reference's analytic controllers before rounding). Returns a slot >= n_actions usable
 * as an action index, or < 0. Slots are cached by force value. */
int qc_add_force(qc_handle* h, double force);

/*
 * step() / simulate_10_steps() (IHO/simulation_i.cpp:358-421, HO/simulation.cpp:339-402,
 * QO/simulation_quart.cpp:493-558), batched and fused over n_steps physics steps:
 *   psi       [B][N] complex128, advanced in place (the reference mutates `state` in place).
 *   actions   [B] int32 action index per env (0..n_actions-1 or a qc_add_force slot);
 *             NULL -> every env uses `default_action`.
 *   env_steps [B] int32 per-env step budget: env e advances min(n_steps, env_steps[e]) steps (0 =
 *             frozen, e.g. a finished episode awaiting reset); NULL -> n_steps for every env.
 *   noise     [n_steps][B][2] fp64 N(0,1) draws to inject (parity tests), or NULL for the handle's
 *             stream (qc_noise_mode: in-kernel Philox keyed by (seed, env_offset + e, env e's counter),
 *             or env e's MT19937); only the first min(n_steps, env_steps[e]) steps of env e are read.
 *   q_out, xmean_out  [n_steps][B] per-step (q, x_mean) outputs of step(), or NULL.
 *   fail_step [B]: 1-based index of the first step after which Fail (check_boundary_error) held,
 *             0 if none; NULL to skip.
 *   term_step [B]: IQO outside-probability criterion (IQO/main_parallel.py:78-81,199-200) on the
 *             states before each step and after the last: first k in [0, n_steps] with
 *             P_out > 0.5, -1 if none; requires params.xth > 0; NULL to skip.
 *   obs_out   [B][n_obs] fp64 observation of the final state (same as qc_moments), or NULL.
 * Env e's noise stream advances by the min(n_steps, env_steps[e]) steps it takes.
 */
int qc_step(qc_handle* h, void* psi, const int32_t* actions, int32_t default_action, int32_t n_steps,
            const int32_t* env_steps, const double* noise, double* q_out, double* xmean_out, int32_t* fail_step,
            int32_t* term_step, double* obs_out);

/* Step-kernel timing (measurement, bench.py): with timing on, every qc_step records a HIP event pair on the
 * handle's stream around its k_step launch only (not the grouping or noise kernels); qc_step_kernel_time
 * synchronises the stream and returns the summed kernel time and the number of launches since the last
 * call (then restarts the count). */
int qc_set_timing(qc_handle* h, int on);
int qc_step_kernel_time(qc_handle* h, double* total_ms, int64_t* launches);

/* get_moments(state, out) (QO/simulation_quart.cpp:363-388) for grids; the Fock 'xp' vector
 * get_data_xp (IHO/main_parallel.py:129-131) for HO/IHO. out [B][n_obs] fp64. */
int qc_moments(qc_handle* h, const void* psi, double* out);

/* x_expectation(state) (IHO/simulation_i.cpp:204-215, QO/simulation_quart.cpp:244-258): out [B] */
int qc_x_expectation(qc_handle* h, const void* psi, double* out);

/* calculate_outside_probability(state, xth) (IQO/main_parallel.py:78-81): out [B] */
int qc_outside_prob(qc_handle* h, const void* psi, double xth, double* out);

/* check_boundary_error (IHO/simulation_i.cpp:422-426, QO/simulation_quart.cpp:559-565): out [B] */
int qc_boundary_fail(qc_handle* h, const void* psi, int32_t* out);

/* cal_energy(state, Hamil) (QO/main_parallel.py:52-53, quartic reward) = Re<psi|H|psi> w with the
 * force-free H: out [B] */
int qc_energy(qc_handle* h, const void* psi, double* out);

/* Hamiltonian_dot_psi(state) (IHO/simulation_i.cpp:585-601, HO/simulation.cpp:566-582): psi <- H psi in place for
 * every env, H the force-free Hamiltonian (mkl_sparse_z_mv of harmonic_Hamil; grid families: their kinetic +
 * potential H, which the reference's grid modules do not export) */
int qc_hamiltonian_dot_psi(qc_handle* h, void* psi);

/* phonon_number(state) (HO/main_parallel.py:88-89, harmonic-cooling reward) = sum n |psi_n|^2: out [B] */
int qc_phonon_number(qc_handle* h, const void* psi, double* out);

/* get_data_wavefunction (args.input == 'wavefunction'): hstack(Re, Im) of state[:-10] (HO,
 * HO/main_parallel.py:132-134), state[:-20] (IHO, IHO/main_parallel.py:133-135) or state[10:-10] (grid,
 * QO/main_parallel.py:132-133, IQO/main_parallel.py:136-137), cast to float32 and
 * times input_scaling in float32 (IHO:241,247): out [B][qc_wavefunction_len()] float32 (device) */
int qc_wavefunction_len(const qc_handle* h);
int qc_wavefunction_obs(qc_handle* h, const void* psi, double input_scaling, float* out);

/* Episode reset of psi for envs with mask[e] != 0 (mask NULL = all; device uint8 [B]):
 *   QC_RESET_GROUND   Fock |0> (IHO/main_parallel.py:231-232, HO/main_parallel.py:226-227)
 *   QC_RESET_RANDOM   Fock: normalised complex Gaussian amplitudes on levels < arg0 (synthetic
 *                     benchmark input), Philox stream tag 1 keyed by global env id
 *   QC_RESET_GAUSSIAN grid: Gaussian_packet(wavelength=1/k, mean, std) (IQO/main_parallel.py:75-76,
 *                     182-183) with per-env k/mean/std (device fp64 [B] arrays, may be NULL ->
 *                     arg0/arg1/arg2 scalars) */
enum qc_reset_kind { QC_RESET_GROUND = 0, QC_RESET_RANDOM = 1, QC_RESET_GAUSSIAN = 2 };
int qc_reset(qc_handle* h, void* psi, int32_t kind, const uint8_t* mask, double arg0, double arg1,
             double arg2, const double* k_arr, const double* mean_arr, const double* std_arr);

/* Analytic baseline controllers, one action per env from the current state:
 *   QC_CTL_LQG           Fock: the actor's args.LQG branch of call_force (IHO/main_parallel.py:194-206,
 *                        HO/main_parallel.py:192-203) on the network input data = float32 get_data_xp(state)
 *                        * input_scaling (pass 1.0 for the unscaled get_data_xp of a non-'xp' input,
 *                        IHO/main_parallel.py:261-262); control_time = 1 / n_con.
 *                        grid: controllers.LinearQuadratic(state, k = lambda_ * con_parameter)
 *                        (QO/controllers.py:16-20, QO/main_parallel.py:168)
 *   QC_CTL_DAMPING       grid: controllers.steepest_descent(state, damping = con_parameter) (:7-14)
 *   QC_CTL_SEMICLASSICAL grid: controllers.Gaussian_approx(state) (:22-29)
 * Grid forces use the drivers' space_def operators (full Delta_1 p_hat) and control_time =
 * 1 / controls_per_unit_time; force = F / pi (Fock: F / omega) is clipped to +-F_max and rounded to the
 * action grid with Python round() semantics (analytic_controls, QO/main_parallel.py:170-181).
 * actions [B] int32 (device) receive round(force / spacing) + n_actions/2; force_out [B] fp64 (optional)
 * the rounded force passed to step(). A NaN force (Gaussian_approx with a negative root argument,
 * where the reference raises a math domain error) yields action -1 and force NaN. */
enum qc_control_strategy { QC_CTL_LQG = 0, QC_CTL_DAMPING = 1, QC_CTL_SEMICLASSICAL = 2 };
int qc_control(qc_handle* h, const void* psi, int32_t strategy, double con_parameter, double control_time,
               double input_scaling, int32_t* actions, double* force_out);

/* Measurement-record input mode: args.input == 'measurements' of the Fock drivers
 * (IHO/main_parallel.py:143-151,270-309; HO/main_parallel.py:142-150,259-292), for B envs in place on
 * the device. Per env (device float32):
 *   hist   [B][2][read_length]  the network input np.array([measurements_input[::-1],
 *                               forces_along_measurements_input[::-1]]): measurements newest first, and
 *                               force * input_scaling applied during each
 *   forces [B][K + 1]           forces_to_store after the control step's append, newest first,
 *                               K = read_length / m, m = n_steps / coarse_grain
 * One call closes one control interval of n_steps physics steps: q [n_steps][B] fp64 are the q outputs of
 * qc_step for it (q_out), actions [B] (or default_action) the actions applied during it. Each group of
 * coarse_grain steps adds sum(q) / coarse_grain * input_scaling; the histories shift by m.
 * mode [B] (device uint8, NULL = all 1): 0 leaves the env untouched, 1 records, 2 records into a fresh
 * (zero) history (a new episode, IHO:271-272). rows [B][qc_record_row_len()] (optional) receive the
 * experience row hstack(measurements_input[::-1] (read_length + m), forces_to_store[::-1] (K + 1),
 * last_action, reward) (IHO:279-283, TrainDQN reads it at RL.py:180-192); the reward column is written
 * only when reward [B] is given. The drivers' values: read_length = round(n_periods * 2 * 1440) with
 * n_periods 2 (IHO, 5760) or 1.5 (HO, 4320), coarse_grain = time_steps / 1440. An out-of-range action
 * is clamped on the device and raises the handle's error word: the next qc_take_errors reports it (as for
 * qc_step). */
int qc_record_row_len(int32_t read_length, int32_t interval, int32_t coarse_grain);
int qc_record(qc_handle* h, int32_t read_length, int32_t coarse_grain, double input_scaling, const double* q,
              int32_t n_steps, const int32_t* actions, int32_t default_action, const uint8_t* mode, float* hist,
              float* forces, const float* reward, float* rows);

/* Host-side introspection of the factor tables (tests): number of Kogge-Stone levels kept for
 * action a (forward, backward), and the truncation bound used. */
int qc_scan_levels(const qc_handle* h, int32_t action, int32_t* fwd, int32_t* bwd);

/* Deferred input errors: qc_step does not synchronise to validate its actions; an action outside
 * [0, n_slots) of an env with a step budget raises a device error word (the kernels clamp it). This call
 * synchronises the handle's stream, returns QC_EINVAL (message via qc_last_error) if any qc_step since the
 * last call saw such an action, and clears the word; QC_OK otherwise. */
int qc_take_errors(qc_handle* h);

/* Introspection (tests, diagnostics): the workgroup layout of the last grouped qc_step call (k_group).
 * Copies up to order_len entries of the single-slot workgroup list and up to mixed_len of the two-slot list
 * (workgroups of qc_step_group_size() envs each, -1 = idle wave) into host buffers (either may be NULL) and
 * returns the number of two-slot workgroup slots (0 when the handle does not use them). Synchronises. */
int qc_step_group_size(const qc_handle* h);
int qc_group_layout(qc_handle* h, int32_t* order, int64_t order_len, int32_t* mixed, int64_t mixed_len);

/* ---------------------------------------------------------------------------------------------
 * Batched DQN actor: the reference's direct_DQN action selection
 * (inverted harmonic oscillator/RL.py:80-111 + layers.py FactorizedNoisy / Linear_weight_normalize),
 * evaluated for B envs at once on the device, with the actor's epsilon-greedy choice
 * (IHO/main_parallel.py:208-219), replacing the per-actor pipe to the inference process
 * (IHO/main_parallel.py:414-440). Layers: fc1 (in -> 512), fc2 (512 -> 256), fc31 (256 -> 256),
 * fc41 (256 -> n_actions), ReLU between; actions = argmax of fc41 (the mean branch fc32/fc42 does not
 * enter the action). fp32 throughout (the reference net's dtype), f32-input MFMA. */
typedef struct qc_actor qc_actor;

typedef struct qc_dqn_params {
    int32_t data_length;   /* network input length (5 for the 'xp' input, IHO/main_parallel.py:137-138) */
    int32_t n_actions;     /* 21 */
    int64_t max_batch;     /* largest B passed to qc_actor_act */
    uint64_t seed;         /* Philox key of the NoisyNet noise and the epsilon-greedy draws */
} qc_dqn_params;

/* One layer's parameters (device fp32 pointers, the reference state_dict tensors):
 * Linear_weight_normalize: weight [out][in], bias [out], weight_norm (scalar g; effective weight
 *   W g / ||W||_F, layers.py:97-103); sigma_w = sigma_b = NULL.
 * FactorizedNoisy: weight = u_w [out][in], bias = u_b, sigma_w [out][in], sigma_b [out],
 *   weight_norm = NULL (layers.py:7-79). */
typedef struct qc_dqn_layer {
    const float* weight;
    const float* bias;
    const float* weight_norm;
    const float* sigma_w;
    const float* sigma_b;
} qc_dqn_layer;

int qc_actor_create(const qc_dqn_params* p, int device, qc_actor** out);
void qc_actor_destroy(qc_actor* a);
const char* qc_actor_last_error(const qc_actor* a);
int qc_actor_set_stream(qc_actor* a, void* stream);
/* (re)load fc1, fc2, fc31, fc41 (the trainer's periodic state_dict push, IHO/main_parallel.py:400-405):
 * computes the effective weights and stores them in the kernels' fragment order on the device */
int qc_actor_load(qc_actor* a, const qc_dqn_layer layers[4]);

/* Noise of the factorised noisy layers per env: eps_in(fc31)[256], eps_out(fc31)[256],
 * eps_in(fc41)[256], eps_out(fc41)[n_actions], each f(z) = sign(z) sqrt|z| of a standard normal z
 * (layers.py:77-79): qc_actor_noise_len() floats per env. */
int qc_actor_noise_len(const qc_actor* a);

/* One action per env: obs [B][data_length] fp32 (device): the network input exactly as the actor hands it
 * over (get_data(state) * input_scaling in float32, IHO/main_parallel.py:131,241,247; BatchedEnv.obs),
 * actions [B] int32 (device). noisy = 0 evaluates the mean weights
 * (layers.py:41-43); noise NULL draws the NoisyNet noise in-kernel (Philox keyed by seed and
 * env_offset + e, counter `counter`), else injected [B][noise_len] fp32. With probability eps an env
 * takes a uniform random action instead (random_out[e] = 1). q_out [B][n_actions] fp32 and
 * random_out [B] int32 are optional. */
int qc_actor_act(qc_actor* a, int64_t B, int64_t env_offset, const float* obs, int32_t noisy,
                 const float* noise, double eps, uint64_t counter, int32_t* actions, float* q_out,
                 int32_t* random_out);

/* The measurement-input actor (SURVEY §8f rank 1 for args.input == 'measurements'): DQN_measurement
 * (inverted harmonic oscillator/RL.py:29-78) for B envs: conv1 Conv1d(2, 32, 13, stride 5), conv2
 * Conv1d(32, 64, 11, 4), conv3 Conv1d(64, 64, 9, 4) with ReLU, flatten, fc1 Linear(64 T3, 256) + ReLU,
 * fc21 FactorizedNoisy(256, 256) + ReLU, fc31 FactorizedNoisy(256, n_actions) -> argmax, epsilon-greedy.
 * The convolutions run as implicit GEMMs on f32 MFMA over env chunks; the noise layout and the
 * epsilon-greedy draw are qc_actor's (noise_len = 789 at 21 actions). */
typedef struct qc_mdqn_params {
    int32_t read_length;   /* network input length per channel (5760 IHO, 4320 HO; MeasurementRecord) */
    int32_t n_actions;     /* 21 */
    int64_t max_batch;
    uint64_t seed;
    int32_t chunk;         /* envs per convolution chunk (0: 2048) */
} qc_mdqn_params;
typedef struct qc_mactor qc_mactor;
int qc_mactor_create(const qc_mdqn_params* p, int device, qc_mactor** out);
void qc_mactor_destroy(qc_mactor* a);
const char* qc_mactor_last_error(const qc_mactor* a);
int qc_mactor_set_stream(qc_mactor* a, void* stream);
int qc_mactor_noise_len(const qc_mactor* a);
int qc_mactor_flat_len(const qc_mactor* a);   /* 64 * T3, fc1's input length */
/* layers[6] = conv1, conv2, conv3, fc1 (weight [out][in(*kernel)], bias; weight_norm = sigma = NULL),
 * fc21, fc31 (FactorizedNoisy u_w/u_b/sigma_w/sigma_b, or Linear_weight_normalize) — the state_dict */
int qc_mactor_load(qc_mactor* a, const qc_dqn_layer layers[6]);
/* obs [B][2][read_length] fp32 (device): the network input (MeasurementRecord.hist); the rest as
 * qc_actor_act */
int qc_mactor_act(qc_mactor* a, int64_t B, int64_t env_offset, const float* obs, int32_t noisy,
                  const float* noise, double eps, uint64_t counter, int32_t* actions, float* q_out,
                  int32_t* random_out);

/* ---------------------------------------------------------------------------------------------
 * Prioritized experience replay on the device: the reference's SumTree + Memory
 * (inverted harmonic oscillator/RL.py:234-475), fed by BatchedEnv without leaving HBM.
 * Layout as the reference: tree float64 [n_nodes + capacity] heap-indexed, leaf of slot d at n_nodes + d;
 * data float32 [capacity][row_len]. All pointers below are device pointers; calls are asynchronous on
 * the memory's stream (qc_replay_stats synchronises). */
typedef struct qc_replay qc_replay;

typedef struct qc_replay_params {
    int64_t capacity;             /* round(size_of_replay_memory * n_con * 100) (IHO/main_parallel.py:595) */
    int32_t row_len;              /* data_size of one row: 2 * obs_len + 2 ('xp'), qc_record_row_len ('measurements') */
    int32_t policy;               /* 0 'sequential', 1 'random' (the drivers: 'random', main_parallel.py:598) */
    double passes_before_random;  /* 0.2 (main_parallel.py:598); SumTree.passes starts at minus this */
    double alpha;                 /* 0.2  Memory.alpha (RL.py:372)                    */
    double beta;                  /* 0.2  Memory.beta, initial (RL.py:373)            */
    double beta_increment;        /* 0.001 per sample (RL.py:374)                     */
    double abs_err_upper;         /* 1.0 (RL.py:375)                                  */
    double epsilon_scale;         /* 1e-5: epsilon = 1e-5 * max (RL.py:442)           */
    uint64_t seed;                /* Philox key: random-policy positions, sampling uniforms */
} qc_replay_params;

typedef struct qc_replay_stats_t {
    int64_t len;                  /* len(memory) (RL.py:415-416)  */
    int64_t data_pointer;
    double passes;
    double max;                   /* Memory.max                    */
    double beta;                  /* Memory.beta after the last sample */
    double total_p;               /* SumTree.total_p = tree[0]     */
    int64_t n_nodes, tree_size;
} qc_replay_stats_t;

int qc_replay_create(const qc_replay_params* p, int device, qc_replay** out);
void qc_replay_destroy(qc_replay* r);
const char* qc_replay_last_error(const qc_replay* r);   /* r may be NULL: last create failure */
int qc_replay_set_stream(qc_replay* r, void* stream);
/* Memory.store for each row e < n with valid[e] != 0 (valid NULL = all), in index order (RL.py:417-420,
 * SumTree.add :273-288): priority max (or abs_err_upper while max == 0); 'sequential' slots while
 * passes < 1, then random slots (Philox); a slot hit twice in one call keeps the later row. */
int qc_replay_store(qc_replay* r, int64_t n, const uint8_t* valid, const float* rows /*[n][row_len]*/);
/* the same, assembling the 'xp' experience row np.hstack((last_data, data, [last_action], [reward]))
 * (IHO/main_parallel.py:250-257) from its parts: last_obs/obs [n][obs_len] fp32, action [n] int32,
 * reward [n] fp32; row_len must be 2 * obs_len + 2 */
int qc_replay_store_xp(qc_replay* r, int64_t n, const uint8_t* valid, const float* last_obs, const float* obs,
                       int32_t obs_len, const int32_t* action, const float* reward);
/* Memory.obtain_sample(n) / compiled_sampling (RL.py:423-432, :449-469): beta += increment (max 1),
 * stratified v_i = (i + u_i) * total / n with u [n] injected (NULL: Philox), tree_idx [n] int32 leaf
 * indices, is_weights [n] fp32 = (p / (total / len))^-beta, transitions [n][row_len] fp32 (NULL: skip the
 * gather). Requires len >= 1 (the reference returns nothing while len < n). */
int qc_replay_sample(qc_replay* r, int32_t n, const double* u, float* transitions, int32_t* tree_idx,
                     float* is_weights);
/* Memory.batch_update (RL.py:438-446, :471-475): abs_errors [n] fp32 (the per-sample losses); a tree_idx
 * outside the leaves [n_nodes, n_nodes + capacity) is skipped (no write, no ancestor update) */
int qc_replay_update(qc_replay* r, int32_t n, const int32_t* tree_idx, const float* abs_errors);
/* Memory.clean / recalculate_structure (RL.py:312-331, :421-422): every parent recomputed */
int qc_replay_rebuild(qc_replay* r);
int qc_replay_stats(qc_replay* r, qc_replay_stats_t* out);
/* device pointers of the tree and the row storage (introspection, tests) */
int qc_replay_buffers(const qc_replay* r, const double** tree, const float** data);

/* ---- batched episode loop: the per-control-step bookkeeping of Control.do_episode --------------------------
 * (IHO/main_parallel.py:242-268, IQO/main_parallel.py:190-221; the cartpoles, 'xp' input) for every env after a
 * step call of one control interval, on the device (BatchedEnv reset="deferred"): pending[e] (in) marks the envs
 * whose call was their reset interval (the zero-th step without control): their time restarts at one interval,
 * return at 0, no valid transition; an episode over at that first control step is reported with return 0 (the
 * i != control_interval guard, IHO:250). Other envs: t += interval dt, done = Fail in the interval or out of
 * bounds (IHO |<x>| > xth: |obs[e][0]| > xth; IQO: term_step[e] >= 0), reward failing_reward / 1, valid,
 * return += reward. Done envs: (return, t) appended to the ring fin [2][fin_cap + 1] at *fin_n (env order; the
 * reference's result queue, IHO:300-327) and pending[e] (out) = 1: they reset in the next call. All device
 * pointers; obs32 [B][n_obs] = float(obs) * input_scaling (NULL: skip). No host synchronisation. */
typedef struct qc_env_tail_args {
    int64_t B;
    int32_t kind;             /* enum qc_family of the cartpole: QC_IHO or QC_IQO */
    int32_t n_obs, interval;  /* observables per env; physics steps per control interval */
    int32_t pad;
    double dt, xth, input_scaling, failing_reward;
    const int32_t* fail_step; /* [B] qc_step's fail_step */
    const int32_t* term_step; /* [B] qc_step's term_step (IQO) or NULL */
    const double* obs;        /* [B][n_obs] qc_step's obs_out */
    uint8_t* pending;         /* [B] in: reset interval in this call; out: resets in the next call */
    double* t;                /* [B] episode time */
    int64_t* steps;           /* [B] physics steps of the episode */
    double* episode_return;   /* [B] */
    float* obs32;             /* [B][n_obs] or NULL */
    float* reward;            /* [B] the reference's reward-row value */
    uint8_t* done;            /* [B] */
    uint8_t* valid;           /* [B] transitions the reference stores */
    double* fin;              /* [2][fin_cap + 1] finished (return, length) */
    int64_t fin_cap;
    int64_t* fin_n;           /* [1] episodes appended so far */
} qc_env_tail_args;
int qc_env_tail(qc_handle* h, const qc_env_tail_args* a);

/* ---- step server: the reference's process model on one GPU ------------------------------------------------
 * The drivers run 30-40 actor processes, each with its own `simulation` module stepping ONE env per call
 * (IHO/main_parallel.py:345-359, :264). A step server owns one handle of batch max_clients (env e = client slot
 * e, MT19937 noise per env) and a POSIX shared-memory object `name` ("/..."); actor processes attach with
 * libqcart_client.so (include/qcart_client.h, no HIP) and post step / simulate_10_steps / set_seed /
 * x_expectation / get_moments requests. Each tick steps every pending env in one batched launch (per-env step
 * budgets keep the others frozen); the tick waits up to batch_wait_us (<= 0: 40 us) after its first request for
 * the other owned slots' requests. Results equal the plain drop-in's (the same kernels, the same per-env
 * MT19937 stream). Fock modules: while qc_server_run serves, a resident kernel (one wave per slot) answers the
 * clients' step(state, dt, force, gamma) calls on the action grid directly from the shared object, without a
 * launch or a tick (qcart_shm.h); the ticks carry the other calls. */
typedef struct qc_server qc_server;
int qc_server_create(const qc_params* p, int device, int32_t max_clients, const char* name, double batch_wait_us,
                     qc_server** out);
/* serve on the calling thread until qc_server_stop (another thread) or `seconds` (> 0) have passed */
int qc_server_run(qc_server* s, double seconds);
int qc_server_stop(qc_server* s);
int qc_server_stats(const qc_server* s, int64_t* ticks, int64_t* calls);
/* out[4]: microseconds summed over the ticks — batching wait, host launches, GPU (until the stream sync
 * returned), publishing the results */
int qc_server_timing(const qc_server* s, double* out);
/* 1 when the server serves one-step calls on its resident kernel (fp64 modules at the drivers' sizes;
 * QCART_SERVER_RESIDENT=0 turns it off), else 0; *calls: the requests the resident path has answered since the object
 * was created; *launches: resident kernel launches (each lives one lease, QCART_RESIDENT_LEASE_MS, default 20 ms) */
int qc_server_resident(const qc_server* s, int64_t* calls, int64_t* launches);
const char* qc_server_last_error(const qc_server* s);
/* marks the object dead (waiting clients fail with QCC_ENOSERVER) and unlinks it */
void qc_server_destroy(qc_server* s);

#ifdef __cplusplus
}
#endif
#endif
