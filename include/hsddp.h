/*
 * hsddp.h — C-ABI of the MI355X-native batched HS-DDP solver for the HKD quadruped model.
 *
 * Drop-in boundary for the hot path of heli-sudoo/HKD-MPC: one host call runs the reference's
 * MultiPhaseDDP::solve (HSDDPSolver/source/MultiPhaseDDP.cpp:232-428) for B independent
 * trajectories at once on one GPU.  Plain pointers and sizes only; no torch or Eigen types.
 *
 * Reference interfaces replaced (file:line in /root/reference):
 *   hsddp_default_options / hsddp_options     HSDDP_OPTION            HSDDPSolver/common/HSDDP_CompoundTypes.h:18-60
 *   hsddp_load_settings                       loadHSDDPSetting        HSDDPSolver/common/HSDDP_CompoundTypes.h:62-87
 *   hsddp_load_constraint_params              loadConstrintParameters HKDMPC/HKD-TrajOpt/HKDProblem.h:70-90
 *   hsddp_set_element_layouts                 HKDProblem::initialization's per-problem phase segmentation HKDProblem.cpp:40-68
 *   hsddp_create (+ problem descriptor)       HKDProblem::initialization/create_problem_one_phase/
 *                                             add_tconstr_one_phase   HKDMPC/HKD-TrajOpt/HKDProblem.cpp:15-111,225-310
 *                                             MultiPhaseDDP::set_multiPhaseProblem  MultiPhaseDDP.h:374-382
 *   hsddp_upload_problem (x0, references)     MultiPhaseDDP::set_initial_condition  MultiPhaseDDP.h:384;
 *                                             HKDSinglePhaseReference::get_reference_at_t HKDReference.cpp:8-57
 *   hsddp_upload_warm_start                   Trajectory::Xbar/Ubar/K warm start    TrajectoryManagement.h:54-77
 *   hsddp_upload/download_constraint_params   PathConstraintBase / TerminalConstraintBase params (ReB, AL)
 *                                             ConstraintsBase.h:88-183, 329-405
 *   hsddp_solve                               MultiPhaseDDP::solve                  MultiPhaseDDP.cpp:232-428
 *   hsddp_solve_begin/_iterate/_end           the same loop split at its inner iterations (:257-303 / :304-381 / :383-408)
 *   hsddp_download_trajectory                 Trajectory fields read by the caller  HKDMPC.cpp:243-298
 *   hsddp_download_element_info               get_actual_cost                       MultiPhaseDDP.h:416
 *   hsddp_download_solver_info                get_solver_info (per-iteration buffers) MultiPhaseDDP.cpp:532-541
 *   hsddp_load_quad_reference                 QuadReference::load_top_level_data   QuadReference.cpp:129-290
 *   hsddp_plan_phases                         HKDProblem::initialization (segmentation) HKDProblem.cpp:15-68
 *   hsddp_set_reference_table / _build_references  HKDSinglePhaseReference::get_reference_at_t HKDReference.cpp:8-57
 *   hsddp_advance / hsddp_get_phase_info      HKDProblem::update from the reference table   HKDProblem.cpp:117-222
 *   hsddp_shift / hsddp_update_problem        HKDProblem::update + HKDMPCSolver::update's re-solve
 *                                             setup (warm start reused)  HKDProblem.cpp:117-222; HKDMPC.cpp:96-143
 *   hsddp_set_layout                          a caller-side HKDProblem::update's layout + SinglePhase::
 *                                             update_SS_config (SS_set)  HKDProblem.cpp:203-217; SinglePhase.h:161-164
 *   hsddp_extract_commands(_async)            update_foot_placement + publish_mpc_cmd HKDMPC.cpp:207-298
 *   hsddp_hkd_dynamics                        HKD::Model::dynamics (hkinodyn)       HKDModel.h:33-45
 *   hsddp_hkd_dynamics_partial                HKD::Model::dynamics_partial          HKDModel.h:46-61
 *   hsddp_hkd_resetmap(_partial)              HKDReset::resetmap(_partial)          HKDReset.h:41-136
 *   hsddp_hkd_foot_position / _jacobian       compute_foot_position / comp_foot_jacob_{1..4}
 *                                             (CasadiGen/header/comp_foot_*.h via casadi_interface.cpp:5-80)
 *   hsddp_hkd_running_cost / _terminal_cost   HKDTrackingCost / HKDFootPlaceReg running_cost(_par),
 *                                             terminal_cost(_par)   HKDCost.h:8-99; HKDCost.cpp:5-63
 *   hsddp_hkd_grf_constraint                  GRFConstraint::compute_violation/_partial HKDConstraints.cpp:7-66
 *   hsddp_hkd_touchdown_constraint            TouchDownConstraint::compute_violation/_partial HKDConstraints.cpp:69-171
 *
 * Conventions
 *   - Return 0 on success, < 0 on error (hsddp_last_error() gives a message).  The reference
 *     reports failures with bool returns and printf (MultiPhaseDDP.cpp:421-427); here the per-
 *     element outcome is hsddp_element_info.status.
 *   - Caller owns host buffers; the library owns device buffers.  One HIP stream per handle.
 *     Not thread-safe per handle (the reference's solve is single-threaded per instance).
 *   - Arrays are element-major, fp64.  State slots: phase i owns N_i + 1 states (S = sum(N_i+1));
 *     control slots: N_i per phase (Kc = sum N_i).  Matrices in the solver API are row-major
 *     [row][col]; the model primitives write Eigen's column-major layout (as the reference's
 *     StateMap/ContrlMap buffers) — see each function.
 *   - Every path runs on the GPU.  A handle created without a usable device fails with
 *     HSDDP_ERR_DEVICE; there is no CPU fallback.
 */
#ifndef HSDDP_H
#define HSDDP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HSDDP_NX 24
#define HSDDP_NU 24
#define HSDDP_MAX_PHASES 16
/* TouchDownConstraint objects one phase can carry: HKDProblem::initialization registers one per
 * phase and HKDProblem::update one more at every step its last phase has reached its end
 * (HKDProblem.cpp:104,199-202); each keeps its own AL parameters. */
#define HSDDP_MAX_TD 4
/* longest regularisation schedule accepted: mu = max(mu * update_regularization, 1e-3) retries
 * of one failed backward sweep until mu > 1e2 (MultiPhaseDDP.cpp:150-167) */
#define HSDDP_MAX_REG_ATTEMPTS 64

enum {
    HSDDP_OK = 0,
    HSDDP_ERR_ARG = -1,
    HSDDP_ERR_DEVICE = -2,
    HSDDP_ERR_ALLOC = -3,
    HSDDP_ERR_IO = -4,
    HSDDP_ERR_UNSUPPORTED = -5,
};

/* Per-element solve outcome (replaces the reference's printf + `goto bad_solve`). */
enum {
    HSDDP_STATUS_OK = 0,            /* finished: converged or iteration budget spent */
    HSDDP_STATUS_REG_OVERFLOW = 1,  /* regularization exceeded 1e2 (MultiPhaseDDP.cpp:162-167) */
    /* (no other outcome: rollouts that break the 1e6 bound are the reference's rejected trials and
       keep any number of older constraint values, hsddp_download_constraint_values) */
};

/* POD mirror of HSDDP_OPTION (HSDDP_CompoundTypes.h:18-60), same field names and meaning. */
typedef struct hsddp_options {
    double alpha, gamma, update_penalty, update_relax, update_regularization, update_ReB;
    int max_DDP_iter, max_AL_iter, max_DDP_iter_runtime, max_AL_iter_runtime;
    double cost_thresh, tconstr_thresh, pconstr_thresh, dynamics_feas_thresh;
    double merit_rho, merit_scale, merit_offset;
    int AL_active, ReB_active, smooth_active, MS, nsteps_per_node;
    /* extension: throughput mode — disable the inner/outer early-termination tests so every
       element runs exactly max_AL_iter * max_DDP_iter inner iterations. */
    int no_early_exit;
} hsddp_options;

/* HKD cost weights (HKDCost.h:14-36, 56-69; HKDCost.cpp:49,63). */
typedef struct hsddp_hkd_weights {
    double q_eul[3], q_pos[3], q_omega[3], q_v[3], q_qJ;
    double qf_scale[24], qf_gain;
    double r_grf, r_qJd;
    double foot_w[3], foot_gain;
    double foot_term_cost, foot_term_grad;
} hsddp_hkd_weights;

/* ReB / AL initial parameters (settings/constraint_params.info:1-19, HKDConstraints.h:17). */
typedef struct hsddp_constraint_params {
    double grf_delta, grf_delta_min, grf_eps;   /* GRF_ReB */
    double swing_delta, swing_delta_min, swing_eps; /* Swing_ReB (read, unused by HKD: SwingConstraint is never added) */
    double td_sigma, td_sigma_max, td_lambda;   /* TD_AL */
    double mu_fric;                             /* GRFConstraint mu (0.7) */
    double ground_height;                       /* TouchDownConstraint ground height (0) */
} hsddp_constraint_params;

typedef struct hsddp_problem_desc {
    int device;                          /* HIP device ordinal */
    int batch;                           /* B independent trajectories */
    int n_phases;                        /* P <= HSDDP_MAX_PHASES */
    int horizons[HSDDP_MAX_PHASES];      /* N_i knots per phase (same for every element) */
    double dt;                           /* integration step (HKDMPC.cpp:28) */
    int ref_per_element;                 /* 0: one reference shared by the batch; 1: per element */
    hsddp_hkd_weights weights;
    hsddp_constraint_params cparams;
    /* extension: 1 = fp32 Riccati mode — LQ records, backward sweep,
       gains K and the linear rollout in fp32; dynamics, costs, line search and the AL/ReB outer
       loop stay fp64.  0 (default) = fp64 throughout, as the reference (T = double). */
    int riccati_fp32;
} hsddp_problem_desc;

typedef struct hsddp_element_info {
    double cost, feas, merit, max_tconstr, max_pconstr;
    int iters, outer_iters, status, n_ls_trials;
} hsddp_element_info;

typedef struct hsddp_stats {
    int inner_iterations;      /* inner-loop iterations launched (max over elements) */
    int outer_iterations;
    long long ls_trials;       /* line-search rollouts summed over elements */
    long long element_iterations; /* sum over elements of inner iterations (trajectory-iterations) */
    double ms_total;           /* device time of the solve (HIP events) */
    double ms_backward;        /* device time in the backward Riccati kernel (k_riccati) */
    double ms_lq, ms_forward, ms_other;
    int n_backward_launches;
    double ms_linear;          /* device time in the linear rollout kernel (k_lin_rollout) */
} hsddp_stats;

typedef struct hsddp_handle_t *hsddp_handle;

const char *hsddp_last_error(void);
const char *hsddp_version(void);

void hsddp_default_options(hsddp_options *opt);
void hsddp_default_weights(hsddp_hkd_weights *w);
void hsddp_default_constraint_params(hsddp_constraint_params *cp);
/* INFO-file loaders with the reference loaders' exact key sets (Boost INFO subset parser). */
int hsddp_load_settings(const char *path, hsddp_options *opt);
int hsddp_load_constraint_params(const char *path, hsddp_constraint_params *cp);

int hsddp_create(const hsddp_problem_desc *desc, hsddp_handle *out);
int hsddp_destroy(hsddp_handle h);
int hsddp_set_options(hsddp_handle h, const hsddp_options *opt);
/* The checks hsddp_set_options applies (host only, no device needed): alpha in (0, 1), non-negative
 * iteration budgets, update_regularization > 1 with at most HSDDP_MAX_REG_ATTEMPTS retries from
 * mu = 0 to mu > 1e2.  The reference accepts any factor and spins forever on a factor <= 1. */
int hsddp_validate_options(const hsddp_options *opt);

/* Per-element phase layouts (HKDProblem::initialization segments each problem's horizon by its own
 * gait, HKDProblem.cpp:40-68): element b has n_phases[b] phases of horizons[b][0 .. n_phases[b]-1]
 * knots (horizons is [B][HSDDP_MAX_PHASES]); every element's horizons must sum to the handle's Kc
 * (sum of desc->horizons).  Afterwards the per-element arrays of the solver API use the largest
 * layout as their stride: contacts [B][Pmax+1][4] (element b: rows 0 .. n_phases[b], row
 * n_phases[b] = the contact after its horizon), state-slot arrays [B][Smax][..] (element b: its
 * first S_b = Kc + n_phases[b] rows), per-phase arrays [B][Pmax][..]; the problem must be uploaded
 * again.  The MPC-side steps take every element's own layout (hsddp_shift_elements,
 * hsddp_advance, hsddp_build_references with phase_start_times NULL, hsddp_extract_commands). */
int hsddp_set_element_layouts(hsddp_handle h, const int *n_phases, const int *horizons);

/* contacts int32 [B][P+1][4] (row P: contact after the horizon, for the last phase's touchdown
 * constraint); x0 [B][24]; ref_x, ref_u [Bref][S][24]; ref_foot [Bref][S][12]. */
int hsddp_upload_problem(hsddp_handle h, const int *contacts, const double *x0, const double *ref_x,
                         const double *ref_u, const double *ref_foot);
/* Xbar [B][S][24], Ubar [B][Kc][24], K [B][Kc][24][24]; NULL keeps the current value (initially
 * Xbar = ref_x, Ubar = 0, K = 0 as HKDProblem.cpp:84-90 / TrajectoryManagement.cpp:5-35).  Also
 * resets X = Xbar, U = Ubar, Defect = dX = 0 and the constraint objects to those of a new problem:
 * ReB (delta, eps) = desc->cparams at every knot, one touchdown constraint per phase (the touchdown
 * legs from contact row i to row i + 1, none when there are none) with the initial AL parameters,
 * and zero stored constraint values (hsddp_download_constraint_values).  hsddp_update_problem, in
 * contrast, keeps all of these, as the reference's objects persist from tick to tick. */
int hsddp_upload_warm_start(hsddp_handle h, const double *Xbar, const double *Ubar, const double *K);
/* The constraint parameters the solve reads and updates (its update_AL_params / update_REB_params,
 * ConstraintsBase.h:160-176, 354-372), for callers that keep their constraint objects themselves
 * (the C++ facade's PathConstraintBase::params / TerminalConstraintBase::params):
 * reb_delta, reb_eps [B][Kc][20] (row 5 l + r of stance leg l, GRFConstraint row order);
 * td_legs [B][P][HSDDP_MAX_TD]: the touchdown constraints of each phase in registration order,
 * bit l = leg l (0: no constraint in that slot); al_sigma, al_lambda [B][P][HSDDP_MAX_TD][4] per
 * constraint and leg (entries of legs outside the mask are ignored).  Any pointer may be NULL
 * (kept / not read).  Upload after the problem's contacts (hsddp_upload_problem). */
int hsddp_upload_constraint_params(hsddp_handle h, const double *reb_delta, const double *reb_eps, const int *td_legs,
                                   const double *al_sigma, const double *al_lambda);
int hsddp_download_constraint_params(hsddp_handle h, double *reb_delta, double *reb_eps, int *td_legs,
                                     double *al_sigma, double *al_lambda);
/* The constraint objects' stored values after the last solve (IneqConstrData::g and TConstrData::h,
 * ConstraintsBase.h:12-55; GRFConstraint / TouchDownConstraint::compute_violation,
 * HKDConstraints.cpp:36-53, 79-120), which — like the reference's objects — live on from trial to
 * trial and from solve to solve: a rollout that returns at a diverging knot (SinglePhase.cpp:205-208)
 * leaves them as they were from there on, and a new problem's, a pushed-back knot's and a newly
 * registered touchdown constraint's are zero until a rollout computes them.  grf_g [B][Kc][20]:
 * row 5 l + r of stance leg l (0 for swing legs); td_h [B][P][HSDDP_MAX_TD][4]: the residual of
 * each touchdown constraint's legs (0 outside its mask).  Valid after hsddp_solve / solve_end,
 * before the next hsddp_shift.  Either pointer may be NULL. */
int hsddp_download_constraint_values(hsddp_handle h, double *grf_g, double *td_h);

/* MultiPhaseDDP::solve (MultiPhaseDDP.cpp:232-428) for every element.  With early exits on, each
 * inner iteration is replayed from a cached hipGraph and stats carries ms_total but no per-phase
 * times (ms_lq, ms_backward, ms_linear, ms_forward stay 0); the environment variable
 * HSDDP_NO_GRAPH=1, read at every call, issues launch by launch with the per-phase timers. */
int hsddp_solve(hsddp_handle h, hsddp_stats *stats);
/* Split form of hsddp_solve for timing a fixed number of inner iterations (throughput mode):
 * begin = initial rollout + first outer prologue; iterate = n inner iterations of every active
 * element (MultiPhaseDDP.cpp:304-381); end = AL/ReB updates + outer tests. */
int hsddp_solve_begin(hsddp_handle h);
int hsddp_iterate(hsddp_handle h, int n, hsddp_stats *stats);
int hsddp_solve_end(hsddp_handle h);

int hsddp_download_trajectory(hsddp_handle h, double *Xbar, double *Ubar, double *K);
/* X, U, Defect, dX, dU (any may be NULL) — the working trajectory (quirk A2 state). */
int hsddp_download_working(hsddp_handle h, double *X, double *U, double *Defect, double *dX, double *dU);
int hsddp_download_element_info(hsddp_handle h, hsddp_element_info *info);
/* MultiPhaseDDP::get_solver_info (MultiPhaseDDP.cpp:532-541): per element, the buffered
 * (actual cost, dynamics feasibility, max terminal-constraint violation, max path-constraint
 * violation) of the last solve — the initial entry after the first rollout and one per inner
 * iteration that passed the later-termination test (:277-280, :368-371).  Arrays [B][capacity]
 * (any may be NULL); count [B] receives the entries stored (at most capacity; the rest are 0).
 * The handle keeps 1 + max_AL_iter * max_DDP_iter entries of its current options. */
int hsddp_download_solver_info(hsddp_handle h, int capacity, float *cost, float *dyn_feas, float *eqn_feas,
                               float *ineq_feas, int *count);
/* The LQ model of the last LQ_approximation (SinglePhase.cpp:264-296; the working point X, U of
 * the last inner iteration, quirk A2), expanded from the device's compact record into the
 * reference Trajectory's dense blocks (TrajectoryManagement.h:65-81, RCostData
 * HSDDP_CompoundTypes.h:91-122): A, B [B][Kc][24][24] (row-major, discrete dynamics Jacobians),
 * l [B][Kc] running cost of the last compute_cost (the last rollout's trajectory, SinglePhase.cpp:
 * 235-262), lx, lu [B][Kc][24], lxx, luu [B][Kc][24][24] (lux = 0, no outputs).
 * Any pointer may be NULL. */
int hsddp_download_lq(hsddp_handle h, double *A, double *B, double *l, double *lx, double *lu, double *lxx,
                      double *luu);
/* The terminal data of every phase (TCostData, HSDDP_CompoundTypes.h:125-150, with AL terms;
 * SinglePhase.cpp:286-295) and the reset-map Jacobian at its end (HKDReset.h:78-136; zero after
 * the last phase): Phi [B][P], Phix [B][P][24], Phixx, Px [B][P][24][24]; any may be NULL. */
int hsddp_download_terminal(hsddp_handle h, double *Phi, double *Phix, double *Phixx, double *Px);
/* Value-function export (SinglePhase::get_value_approx, SinglePhaseBase.h:45): when on, every
 * sweep stores G[0], H[0] of each phase (with the Defect[0] term, SinglePhase.cpp:365); regularisation
 * retries then run in the sweep kernel itself.  hsddp_download_value: G [B][P][24], H [B][P][24][24]
 * of the last successful sweep.  Off by default (the solver itself needs only the phase-boundary
 * transfer it does in registers). */
int hsddp_set_value_export(hsddp_handle h, int on);
int hsddp_download_value(hsddp_handle h, double *G, double *H);
int hsddp_synchronize(hsddp_handle h);
size_t hsddp_device_bytes(hsddp_handle h);

/* ---- batched reference construction ----------------------------------
 * One sample of a quad_reference.csv file (QuadAugmentedState, Reference/QuadReference.h:14-65). */
typedef struct hsddp_quad_state {
    double body_state[12];       /* eul, pos, omega, vWorld */
    double qJ[12], qJd[12], foot_placements[12], grf[12], torque[12];
    int contact[4];
    double status_dur[4];
} hsddp_quad_state;

/* QuadReference::load_top_level_data (QuadReference.cpp:129-255, reorder_states :257-290): parse a
 * quad_reference.csv (values rounded through float as std::stof / std::stoi).  Writes dt and up to
 * `capacity` samples into out (out may be NULL to count); returns the number of samples (< 0 on
 * error). */
int hsddp_load_quad_reference(const char *path, int reorder, float *dt, hsddp_quad_state *out, int capacity);

/* HKDProblem::initialization's phase segmentation (HKDProblem.cpp:15-68) on a reference window
 * (QuadReference::initialize: window[0] = the current sample, n_window >= round(plan/dt_ref) + 2),
 * with the float time arithmetic and sample rounding of QuadReference::get_contact_at_t
 * (QuadReference.cpp:78-100): horizons, phase contacts (row n_phases = the contact at
 * plan_duration + dt_mpc, add_tconstr_one_phase :272-276), contact durations, float start / end
 * times. */
typedef struct hsddp_phase_plan {
    int n_phases;
    int horizons[HSDDP_MAX_PHASES];
    int contacts[HSDDP_MAX_PHASES + 1][4];
    double durations[HSDDP_MAX_PHASES][4];
    float start_times[HSDDP_MAX_PHASES], end_times[HSDDP_MAX_PHASES];
} hsddp_phase_plan;
int hsddp_plan_phases(const hsddp_quad_state *window, int n_window, float dt_ref, float plan_duration, float dt_sim,
                      float dt_mpc, hsddp_phase_plan *plan);

/* The reference sample table to the device (once per file): n samples, dt_ref. */
int hsddp_set_reference_table(hsddp_handle h, const hsddp_quad_state *table, int n, float dt_ref);
/* HKDSinglePhaseReference::get_reference_at_t (HKDReference.cpp:8-57) at every state slot of every
 * element, on the device: slot k of phase i reads time t = start_i + k dt_sim (start_i =
 * phase_start_times[i] - phase_start_times[0] as float, or the knot offset times dt_sim when
 * phase_start_times is NULL), snapped to a sample as get_a_reference_ptr_at_t (QuadReference.cpp:
 * 60-76, clamped to the window end window_len - 1) of element b's window, which starts at table
 * sample window_start[b] (one value when the references are shared, ref_per_element = 0).
 * ref_x = [body_state, foot_placements (stance) | qJ (swing)], ref_u = [grf, qJd], ref_foot =
 * foot_placements.  Afterwards hsddp_upload_problem / hsddp_update_problem take NULL references
 * and keep these. */
int hsddp_build_references(hsddp_handle h, const int *window_start, int window_len, const float *phase_start_times,
                           float dt_sim);
/* The references the solve reads (uploaded or built): ref_x, ref_u [Bref][S][24], ref_foot [Bref][S][12]. */
int hsddp_download_references(hsddp_handle h, double *ref_x, double *ref_u, double *ref_foot);

/* ---- receding-horizon update -----------------------------------------
 * HKDProblem::update (HKDProblem.cpp:117-222) for n_steps simulation steps, on the warm start held
 * on the device.  Per step: the first phase drops its first knot, or is removed when it has one
 * knot left; the last phase grows by one knot holding a copy of X.back() with zero control and
 * gain, or — when contact_change[j] (the contact at the new horizon end differs from the last
 * phase's) and the last phase has already seen a change (is_phase_reach_end) — a new one-knot
 * phase with a zero trajectory is appended.  Afterwards Ubar of the first knot is zeroed and every
 * phase gets all its states as shooting states except a last phase of horizon <= 2, which keeps its
 * set (empty for a new phase; its states are then simulated, SinglePhase.cpp:185-222).  The total
 * number of control knots is unchanged.  The flags are shared by the batch (hsddp_shift_elements:
 * per element).
 * After a shift, hsddp_update_problem must upload contacts / x0 / references of the new layout
 * before the next solve. */
int hsddp_shift(hsddp_handle h, int n_steps, const int *contact_change);
/* hsddp_shift with a contact-change flag per element and step: contact_change [B][n_steps].  Each
 * element's phases evolve by its own flags (robots crossing contact boundaries at different
 * knots), so the handle moves to per-element layouts (as hsddp_set_element_layouts) unless every
 * element ends on the same one; hsddp_shift on such a handle shifts every element by the shared
 * flags from its own layout. */
int hsddp_shift_elements(hsddp_handle h, int n_steps, const int *contact_change);
/* every element's layout: n_phases [B], horizons, shooting states, is_phase_reach_end [B][16] (any NULL) */
int hsddp_get_element_layouts(hsddp_handle h, int *n_phases, int *horizons, int *shooting, int *reach_end);
/* current layout: n_phases, horizons[16], shooting states[16], is_phase_reach_end[16] (any NULL);
 * HSDDP_ERR_UNSUPPORTED with per-element layouts (hsddp_get_element_layouts) */
int hsddp_get_layout(hsddp_handle h, int *n_phases, int *horizons, int *shooting, int *reach_end);
/* A new shared layout on a live handle, for callers that run HKDProblem::update's bookkeeping
 * themselves (the C++ facade: SinglePhase::pop_front / push_back_default on the host Trajectory,
 * HKDProblem.cpp:117-222; update_SS_config, SinglePhase.h:161-164): n_phases phases of horizons[i]
 * knots summing to the handle's Kc, shooting[i] = the size of phase i's SS_set {0 .. shooting[i]-1}
 * (NULL: N_i + 1 each; below N_i + 1 only in the last phase — HSDDP_ERR_UNSUPPORTED elsewhere),
 * reach_end[i] = is_phase_reach_end (NULL: 0).  No device work and no reallocation; the handle then
 * needs hsddp_upload_problem (and a warm start) of the new layout before it solves. */
int hsddp_set_layout(hsddp_handle h, int n_phases, const int *horizons, const int *shooting, const int *reach_end);
/* as hsddp_upload_problem, but keeps the warm start Xbar / Ubar / K (the MPC update's reuse of the
 * previous solution) and the constraint parameters: HKDProblem::update's reset_params is a no-op
 * (ConstraintsBase.h:165-167, 341-348), so the per-knot ReB parameters and every touchdown
 * constraint's AL parameters carry over from the previous solve (shifted with their knots and phases
 * by hsddp_shift / hsddp_advance, which also append the touchdown constraints add_tconstr_one_phase
 * registers: their legs are the new contact rows' touchdown legs).  The working trajectory (X, U,
 * Defect) and the constraint objects' stored values carry over too (shifted alike): a solve whose
 * initial rollout diverges keeps them past its break, as the reference's objects do.  Resets the
 * per-element solver state (dX, dU and du keep their values: the next solve rewrites them before
 * any line-search trial reads them; with MS false dX is reset to 0). */
int hsddp_update_problem(hsddp_handle h, const int *contacts, const double *x0, const double *ref_x,
                         const double *ref_u, const double *ref_foot);

/* HKDProblem::update (HKDProblem.cpp:117-222) driven by the reference table, for handles whose
 * references were built by hsddp_build_references: n_steps simulation steps of the window
 * (QuadReference::step), each with the contact at the new horizon end of every element's own
 * window deciding that element's phase growth, the last phase's next contact at plan_duration +
 * dt_mpc once it has reached its end (add_tconstr_one_phase), new phases' contact durations; then
 * the shift (hsddp_shift when the batch agrees on every step's flag, else hsddp_shift_elements:
 * per-element layouts, which need per-element references), the new layouts' references and
 * hsddp_update_problem with these contacts and x0 [B][24].  contact_change [n_steps] (may be NULL)
 * receives, per step, whether any element saw a contact change.  x0 NULL: the inputs are left
 * pending — read the new first phase's contact (hsddp_get_phase_info), form x0 from it
 * (compute_hkd_state, HKDMPC.cpp:132-134) and call hsddp_update_problem(h, NULL, x0, NULL, NULL,
 * NULL), where NULL contacts are the ones derived here.  The caller's whole MPC tick is
 * hsddp_advance + hsddp_solve + hsddp_extract_commands (HKDMPCSolver::update, HKDMPC.cpp:96-165).
 * A phase that would carry more than HSDDP_MAX_TD touchdown constraints keeps its first
 * HSDDP_MAX_TD (the later ones are not registered) and the call returns HSDDP_ERR_UNSUPPORTED after
 * the whole step, on either shift path: layout, references, contacts, x0, durations and clock are
 * the new step's and the handle solves (hsddp_shift / hsddp_shift_elements return the same status
 * after their shift).  The reference registers one constraint at every step a last phase has
 * reached its end (HKDProblem.cpp:199-202); one step later the contact at the horizon end differs
 * and a new phase starts, so with one reference sample per simulation step a phase carries at most
 * two (its initial one and one on reaching its end) — the limit is only met by contact sequences
 * that change faster than the simulation step (tests/test_gpu_td_overflow.py). */
int hsddp_advance(hsddp_handle h, int n_steps, float plan_duration, float dt_mpc, const double *x0,
                  int *contact_change);
/* The handle's phase bookkeeping: contacts [B][P+1][4] (row P: the last phase's next contact) and,
 * for references built from a table, the phases' contact durations [B][P][4] (either may be NULL). */
int hsddp_get_phase_info(hsddp_handle h, int *contacts, double *durations);

/* ---- MPC command extraction ------------------------------------------
 * Mirror of hkd_command_lcmt (lcmtypes/hkd_command_lcmt.lcm:1-11), field for field. */
#define HSDDP_CMD_STEPS 10
typedef struct hsddp_mpc_command {
    int N_mpcsteps;                       /* nsteps_between_mpc + 7 (HKDMPC.cpp:232-235) */
    double mpc_times[HSDDP_CMD_STEPS];    /* mpc_time + k dt_mpc */
    float hkd_controls[HSDDP_CMD_STEPS][24];   /* Ubar */
    float des_body_state[HSDDP_CMD_STEPS][12]; /* Xbar body states */
    int contacts[HSDDP_CMD_STEPS][4];
    double statusTimes[HSDDP_CMD_STEPS][4];    /* contact durations of the knot's phase */
    float foot_placement[12];             /* next touchdown foot positions (update_foot_placement) */
    float feedback[HSDDP_CMD_STEPS][12][12];   /* K(0:12, 0:12) */
    float solve_time;
} hsddp_mpc_command;

/* HKDMPCSolver::update_foot_placement + publish_mpc_cmd (HKDMPC.cpp:207-298) for every element,
 * on the device, from the solved trajectory.  status_durations [Bd][P][4] (Bd = 1 or B; NULL = 0)
 * are the phases' contact durations (HKDProblemData::contact_durations); foot_placements [Bf][12]
 * (Bf = 1 or B; NULL = 0) the current foot positions, kept for legs without a touchdown in the
 * first five phase transitions; out [B] host array.  Rows k >= N_mpcsteps are zero. */
int hsddp_extract_commands(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                           const double *status_durations, int durations_per_element,
                           const float *foot_placements, int feet_per_element, float solve_time,
                           hsddp_mpc_command *out);
/* hsddp_extract_commands without waiting for the records: the kernel runs on the handle's stream
 * and the [B] records (7.8 KB each) cross PCIe into one of two pinned host buffers of the handle on a
 * copy stream of their own, so the copy overlaps whatever the caller issues next (the next tick's
 * hsddp_advance / hsddp_solve).  ticket receives the buffer (0 or 1); hsddp_commands_wait(h,
 * ticket, &records) waits for that copy and points records at the buffer, which stays valid until
 * the extraction after next reuses it.  status_durations and foot_placements are read before the
 * call returns (the caller may release them). */
int hsddp_extract_commands_async(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                                 const double *status_durations, int durations_per_element,
                                 const float *foot_placements, int feet_per_element, float solve_time, int *ticket);
int hsddp_commands_wait(hsddp_handle h, int ticket, const hsddp_mpc_command **records);
/* The same into device memory: out_device [B] hsddp_mpc_command on the handle's device (no host
 * copy) — the optional first-knots command block of the final multi-GPU gather (SURVEY.md §8(e),
 * HKDMPC.cpp:254-286), gathered by the caller's collective straight from HBM. */
int hsddp_extract_commands_device(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                                  const double *status_durations, int durations_per_element,
                                  const float *foot_placements, int feet_per_element, float solve_time,
                                  void *out_device);

/* ---- batched model primitives (device pointers, n points, async on `stream` (NULL = default)) */
/* xn[n][24] = hkinodyn(x[n][24], u[n][24], dt, c[n][4]) */
int hsddp_hkd_dynamics(const double *x, const double *u, const double *c, double dt, double *xn,
                       int n, void *stream);
/* A[n][24*24], B[n][24*24] column-major (Eigen StateMap/ContrlMap memory layout) */
int hsddp_hkd_dynamics_partial(const double *x, const double *u, const double *c, double dt,
                               double *A, double *B, int n, void *stream);
/* p[n][3] = compute_foot_position(pos, eul, qleg, leg+1) with q = x[12+3leg..], pos = x[3..5], eul = x[0..2]; leg[n] */
int hsddp_hkd_foot_position(const double *x, const int *leg, double *p, int n, void *stream);
/* J[n][3*18] column-major, columns [pos(3) | eul(3) | qJ(12)] as comp_foot_jacob_{leg+1} */
int hsddp_hkd_foot_jacobian(const double *x, const int *leg, double *J, int n, void *stream);
/* c, cn int32 [n][4] */
int hsddp_hkd_resetmap(const double *x, const int *c, const int *cn, double *xn, int n, void *stream);
/* Px[n][24*24] column-major */
int hsddp_hkd_resetmap_partial(const double *x, const int *c, const int *cn, double *Px, int n,
                               void *stream);

/* HKD cost and constraint plugins at n points (the bodies of the C++ facade's hkd:: plugins; the
 * solver evaluates the same terms inside its own kernels).  c, cn int32 [n][4]; xr, ur [n][24] and
 * pf [n][12] the knot's references (ref_x, ref_u, ref_foot of hsddp_upload_problem).
 * terms: HSDDP_TERM_TRACKING (HKDTrackingCost) | HSDDP_TERM_FOOT (HKDFootPlaceReg).
 * Running cost (RCostData, HSDDP_CompoundTypes.h:91-122): l [n], lx, lu [n][24], lxx, luu [n][24*24]
 * (symmetric; lux = 0).  Terminal cost (TCostData :125-150): Phi [n], Phix [n][24], Phixx [n][24*24].
 * Any output may be NULL. */
#define HSDDP_TERM_TRACKING 1
#define HSDDP_TERM_FOOT 2
int hsddp_hkd_running_cost(const double *x, const double *u, const int *c, const double *xr, const double *ur,
                           const double *pf, const hsddp_hkd_weights *w, double dt, int terms, double *l, double *lx,
                           double *lu, double *lxx, double *luu, int n, void *stream);
int hsddp_hkd_terminal_cost(const double *x, const int *c, const double *xr, const double *pf,
                            const hsddp_hkd_weights *w, int terms, double *Phi, double *Phix, double *Phixx, int n,
                            void *stream);
/* GRFConstraint: 5 friction-pyramid rows (A_leg, HKDConstraints.cpp:13-18) per stance leg in leg order,
 * g [n][20] = A u, gu [n][20][24] = A rows (IneqConstrData g, gu); rows past 5 x (stance legs) are 0 */
int hsddp_hkd_grf_constraint(const double *u, const int *c, double mu, double *g, double *gu, int n, void *stream);
/* TouchDownConstraint: one row per leg touching down (c = 0, cn = 1) in leg order, h [n][4] = foot
 * height - ground, hx [n][4][24] its state gradient (TConstrData h, hx); unused rows 0 */
int hsddp_hkd_touchdown_constraint(const double *x, const int *c, const int *cn, double ground, double *h, double *hx,
                                   int n, void *stream);

/* device memory helpers for the primitives (so callers without a HIP runtime binding can use them) */
void *hsddp_device_alloc(size_t bytes, int device);
int hsddp_device_free(void *p);
int hsddp_memcpy_h2d(void *dst, const void *src, size_t bytes);
int hsddp_memcpy_d2h(void *dst, const void *src, size_t bytes);
int hsddp_device_synchronize(int device);

#ifdef __cplusplus
}
#endif
#endif /* HSDDP_H */
