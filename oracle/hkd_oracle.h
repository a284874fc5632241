/*
 * hkd_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference HKD-MPC hot path (heli-sudoo/HKD-MPC @ 2024_08_07):
 *   - the HKD model (CasADi-generated kernels restated by hand), hkd_model_ref.c
 *   - the multi-phase HS-DDP solver (MultiPhaseDDP / SinglePhase / ConstraintsBase / HKD costs),
 *     hsddp_oracle.c
 * It exists only to check the HIP product path (tests/, __graft_entry__.smoke(), bench.py's
 * cpu_baseline leg).  The product library never links or calls it.
 *
 * Parity pinning: the model functions are pinned against the reference's own CasADi kernels
 * (oracle/_ref, golden fixtures in tests/golden/).  The solver restatement follows the
 * reference line by line; the reference solver itself cannot be built here (Eigen/Boost/LCM
 * absent), so solver-level parity is pinned by known-answer tests (LQR one-step convergence,
 * discrete Riccati gains, finite-difference checks) — see DESIGN.md §Parity.
 *
 * Conventions: all matrices row-major, double precision.  State x[24] = [eul(yaw,pitch,roll),
 * pos, omega_body, v_world, qdummy(12)]; control u[24] = [GRF(12), qJd(12)]; contact c[4]
 * as doubles in {0,1}; leg order FR, FL, HR, HL.
 */
#ifndef HKD_ORACLE_H
#define HKD_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

#define ORC_NX 24
#define ORC_NU 24

/* ---- model (hkd_model_ref.c) ---------------------------------------------------------- */
void orc_hkd_step(const double *x, const double *u, double dt, const double *c, double *x_next);
void orc_hkd_partial(const double *x, const double *u, double dt, const double *c,
                     double *A /*24x24*/, double *B /*24x24*/);
void orc_foot_position(int leg, const double *pos, const double *eul, const double *qleg, double *p);
void orc_foot_jacobian(int leg, const double *pos, const double *eul, const double *qleg,
                       double *J /*3x18: [pos | eul | qJ(12)]*/);
void orc_resetmap(const double *x, const int *c, const int *cn, double *x_next);
void orc_resetmap_partial(const double *x, const int *c, const int *cn, double *Px /*24x24*/);

/* ---- solver (hsddp_oracle.c) ---------------------------------------------------------- */
typedef struct {
    double alpha, gamma, update_penalty, update_relax, update_regularization, update_ReB;
    int max_DDP_iter, max_AL_iter, max_DDP_iter_runtime, max_AL_iter_runtime;
    double cost_thresh, tconstr_thresh, pconstr_thresh, dynamics_feas_thresh;
    double merit_rho, merit_scale, merit_offset;
    int AL_active, ReB_active, smooth_active, MS, nsteps_per_node;
    int no_early_exit; /* throughput mode: run exactly max_DDP_iter inner iterations */
} orc_options;

typedef struct {
    double q_eul[3], q_pos[3], q_omega[3], q_v[3], q_qJ; /* HKDCost.h:111-119 */
    double qf_scale[24], qf_gain;                         /* HKDCost.h:123-127 */
    double r_grf, r_qJd;                                  /* HKDCost.h:130-133 */
    double foot_w[3], foot_gain;                          /* HKDCost.h:153-166 */
    double foot_term_cost, foot_term_grad;                /* HKDCost.cpp:49,63-64 */
} orc_weights;

#define ORC_MAX_TD 4 /* touchdown constraints per phase (HSDDP_MAX_TD) */

typedef struct {
    int n_phases;
    const int *horizons;      /* [P] */
    double dt;
    double mu_fric;           /* HKDConstraints.h:17 */
    double grf_delta, grf_delta_min, grf_eps; /* constraint_params.info:1-6 */
    double td_sigma, td_sigma_max, td_lambda; /* constraint_params.info:15-19 */
    double ground_height;
    orc_weights w;
    const int *shooting;      /* [P] shooting states per phase: SS_set = {0 .. n-1}
                                 (SinglePhase::update_SS_config, SinglePhase.h:161-164); NULL = all */
} orc_problem;

typedef struct {
    /* per-element inputs */
    const int *contacts;      /* [P+1][4]; row P = contact after the horizon (TD of last phase) */
    const double *x0;         /* [24] */
    const double *ref_x;      /* [S][24]  reference state at every state slot */
    const double *ref_u;      /* [S][24]  reference control (rows at terminal slots unused) */
    const double *ref_foot;   /* [S][12]  reference foot placements */
    /* per-element state (in/out), slot-major */
    double *Xbar, *X, *Defect, *Defect_bar, *dX; /* [S][24] */
    double *Ubar, *U, *dU;                       /* [Kc][24] */
    double *K;                                   /* [Kc][24][24] */
    double *reb_delta, *reb_eps;                 /* [Kc][20] (leg*5+row) */
    /* TouchDownConstraint objects of each phase, in registration order (HKDProblem.cpp:104,
       199-202): legs (bit l = leg l, 0 = no constraint) and AL parameters per constraint and leg */
    double *al_sigma, *al_lambda;                /* [P][ORC_MAX_TD][4] */
    int *td_mask;                                /* [P][ORC_MAX_TD] */
    /* the constraint objects' stored values (IneqConstrData::g, TConstrData::h, ConstraintsBase.h:
       12-55), which live on in the objects from solve to solve: a rollout that returns at a knot
       (SinglePhase.cpp:205-208) leaves them as they were from there on.  GRF values per control
       slot and row [Kc][20]; touchdown residuals per constraint and leg [P][ORC_MAX_TD][4].  Zero
       for a new problem and for knots / constraints the receding-horizon update adds (create_data,
       PathConstraintBase::push_back).  NULL: zeros at the start of the solve. */
    double *grf_g, *td_h;
    /* outputs */
    double cost, feas, merit, max_tconstr, max_pconstr;
    int iters, outer_iters, status, n_ls_trials;
    /* get_solver_info buffers (MultiPhaseDDP.cpp:277-280, 368-371, 532-541): hist_cap entries of
       (cost, feas, max_tconstr, max_pconstr) as float; NULL = not recorded.  hist_n: entries pushed */
    float *hist;
    int hist_cap, hist_n;
    /* diagnostics: the initial rollout broke the 1e6 bound (SinglePhase.cpp:205-208); line-search
       trials that broke it */
    int diverged_init, n_diverged;
} orc_element;

void orc_default_options(orc_options *o);
void orc_default_weights(orc_weights *w);
/* One knot + phase end alone: l, Phi, lx, lu, lxx, luu, lux, Phix, Phixx, A, B (see the .c) */
void orc_knot_eval(const orc_problem *p, const orc_options *o, const int *c, const int *cn, const double *x,
                   const double *u, const double *xr, const double *ur, const double *pf, const double *x_end,
                   const double *xr_end, const double *pf_end, const double *reb_delta, const double *reb_eps,
                   const double *sigma, const double *lambda, double *out);
/* Full MultiPhaseDDP::solve restatement (MultiPhaseDDP.cpp:232-428) on one element. */
int orc_solve(const orc_problem *p, const orc_options *o, orc_element *e);
/* Batch driver: threads over elements (CPU baseline). */
int orc_solve_batch(const orc_problem *p, const orc_options *o, orc_element *elems, int n, int n_threads);

/* Component entry points (for per-pass tests). */
/* SinglePhase::backward_sweep on caller-supplied time-invariant LQ data (the outside Riccati pin) */
int orc_riccati_lq(int N, const double *A, const double *B, const double *lxx, const double *luu, const double *lx,
                   const double *lu, const double *Phix, const double *Phixx, double reg, double *K0, double *dU0,
                   double *G0, double *H0);
/* a new problem's constraint parameters: ReB at every knot, one touchdown constraint per phase
   (contact row i -> i + 1, HKDProblem.cpp:104) with the initial AL parameters; needs e->contacts */
void orc_init_element(const orc_problem *p, orc_element *e);

#ifdef __cplusplus
}
#endif
#endif
