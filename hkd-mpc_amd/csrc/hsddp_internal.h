// hsddp_internal.h — device data layout and kernel interface of the batched HS-DDP solver.
//
// HBM layout (element-major, fp64; b = element, s = state slot, kc = control slot):
//   X3, D3 [3], dX                    [B][S][24]     X3: the nominal Xbar, the working X and the trial
//                                                     rows (sel); D3: the Defect of each buffer's rows
//   U3 [3], dU, du                    [B][Kc][24]     du = dU + K dX (linear-rollout control step)
//   K                                 [B][Kc][12][24] row-major, coupled controls only (below)
//   lq                                [B][Kc][LQW]    compact LQ model of one knot (below)
//   term                              [B][P][TW]      Phix | Phixx | Px (reset-map Jacobian at X_i[N])
//   reb_delta, reb_eps                [B][Kc][20]     ReB params, index leg*5 + row
//   td_mask                           [B][P][MTD]     touchdown constraints of each phase (bit l = leg l;
//                                                     TD_PENDING, TD_STALE below)
//   cf_u, cf_flag                     [B][Kc][12], [B][Kc]  stored GRF values not from U (below)
//   al_sigma, al_lambda               [B][P][MTD][4]  their AL parameters, per constraint and leg
//   term_h                            [B][P][4]       foot heights at the phase end (constraint legs)
//   slot_cost, slot_feas, slot_viol   [B][S]          per-slot partial sums for per-element reductions
//   fp32 Riccati mode (Params::fp32): lq32 [B][Kc][LQW32], K32 [B][Kc][12][24], def32 [B][S][24]
//   replace lq and K (the fp64 copies are not allocated) and mirror Defect for the sweep
// One element's data is contiguous, so the per-element backward kernel streams it coalesced.
#pragma once

#include <hip/hip_runtime.h>
#include "hkd_model.h"

namespace hsddp {

constexpr int NX = 24;
constexpr int NN = 576;
constexpr int MAXP = 16;
constexpr int LS_LIVE = 128;  // line-search trials with a liveness flag (later ones run unconditionally)
// TouchDownConstraint objects per phase (HSDDP_MAX_TD): HKDProblem::initialization registers one
// per phase and HKDProblem::update one more at every step the last phase has reached its end
// (HKDProblem.cpp:104,199-202); each keeps its own AL parameters, which persist across MPC ticks
// (reset_params is a no-op, ConstraintsBase.h:341-348).  A mask of TD_PENDING is resolved to the
// touchdown legs of the phase's contact rows (c_i -> c_{i+1}) when the next contacts are uploaded.
constexpr int MTD = 4;
constexpr int TD_PENDING = 0x10;
// Gains are stored for the 12 controls whose B column is non-zero: row q (0..11) is control
// u = q when leg q/3 is in stance, u = 12 + q when it swings.  The other 12 rows of the
// reference's 24 x 24 K are exactly zero (hsddp_sweep.hip) and are expanded on
// download.
constexpr int KCW = 12 * 24;

// compact LQ record per control slot.  Every piece starts at an even index (16-byte aligned in
// fp64); the slot after SE and after SW is an exact zero (written by k_lq) that the sweep's
// lane-indexed reads use for structurally absent entries.
constexpr int LQ_SE = 0;                 // 15  A - I, eul rows (+1 zero), row-major [3][5]
constexpr int LQ_SW = 16;                // 51  A - I, omega rows (+1 zero), column-major [17][3]
constexpr int LQ_BW = 68;                // 36  B, omega rows x GRF cols, column-major [12][3]
constexpr int LQ_LX = 104;               // 24
constexpr int LQ_LU = 128;               // 24
constexpr int LQ_RB = 152;               // 24  dt * ReB Hessian, 4 legs x sym 3x3 (00,01,02,11,12,22)
constexpr int LQW = 176;
constexpr int LQW32 = 192;               // fp32 record stride: 6 whole 128-byte lines (176 values + zeros)
// record position of omega-row r (0..2) x sparse column q of A - I, and of B's omega row r x GRF
// column k: column-major, so k_lq emits the pieces in position order (hkd_partial_emit) and
// stores them through its LDS stage in contiguous chunks
constexpr int sw_at(int r, int q) { return LQ_SW + 3 * q + r; }
constexpr int bw_at(int r, int k) { return LQ_BW + 3 * k + r; }
static_assert(LQ_SE + 15 < LQ_SW && LQ_SW + 51 < LQ_BW && LQ_BW + 36 == LQ_LX && LQ_LX + 24 == LQ_LU &&
              LQ_LU + 24 == LQ_RB && LQ_RB + 24 == LQW, "record layout");

// longest regularisation schedule of one failed sweep (HSDDP_MAX_REG_ATTEMPTS, include/hsddp.h)
constexpr int MAX_REG_ATTEMPTS = 64;

// per-phase terminal record: Phix, Phixx, Px, each piece starting on a 128-byte line and the record
// a whole number of lines (a line written in two halves at different times costs a second write)
constexpr int TM_PHIX = 0;
constexpr int TM_PHIXX = 32;
constexpr int TM_PX = TM_PHIXX + NN;
constexpr int TW = TM_PX + NN;           // 1184
static_assert(TM_PHIXX % 16 == 0 && TM_PX % 16 == 0 && TW % 16 == 0, "terminal record lines");

// Phase layout of one element: P phases of N_i knots, state slots s0_i .. s0_i + N_i, control slots
// k0_i .. k0_i + N_i - 1, shooting states ss_i; S = sum(N_i + 1).  Per-element layouts
// (hsddp_set_element_layouts) all have the handle's Kc.
struct Layout {
    int P, S, has_tail, pad;
    int N[MAXP], s0[MAXP], k0[MAXP], ss[MAXP];
};

struct Params {
    // B elements; P, S: the handle's layout (with per-element layouts: the largest P and S, the
    // strides of the per-phase and per-slot buffers); Kc control slots of every element
    int B, P, S, Kc;
    int N[MAXP], s0[MAXP], k0[MAXP];
    int ref_per_element;
    double dt, dt_m /* dt / mass, = dt * c / mass for c = 1 */, mu, grf_delta, grf_delta_min, grf_eps, td_sigma, td_sigma_max, td_lambda, ground;
    // HKD weights
    double qbase[12], q_qJ, qf_scale[24], qf_gain, r_grf, r_qJd, foot_w[3], foot_gain, foot_term_cost, foot_term_grad;
    // HSDDP_OPTION
    double alpha, gamma, update_penalty, update_relax, update_regularization, update_ReB;
    double cost_thresh, tconstr_thresh, pconstr_thresh, feas_thresh, merit_scale, merit_offset;
    int AL_active, ReB_active, no_early_exit;
    int reb_uniform;  // every ReB (delta, eps) equals (grf_delta, grf_eps): per-knot arrays not read
    double grf_inv_delta, grf_log_delta;  // 1 / grf_delta, log(grf_delta): the uniform ReB terms' constants
    int lq_slots;     // k_lq recomputes the running costs and |Defect|^2 of the slots (0: the last
                      // rollout's values still hold for the working trajectory and the cost parameters)
    int fp32;         // fp32 Riccati mode (config C5): LQ records, sweep, gains and linear rollout in fp32
    // shooting states per phase, SS_set = {0 .. ss-1} (SinglePhase::update_SS_config,
    // SinglePhase.h:161-164): N_i + 1 except a new last phase of horizon <= 2 after a receding-
    // horizon shift (HKDProblem.cpp:203-216); has_tail: some phase has non-shooting states
    int ss[MAXP];
    int has_tail;
    // parallel regularisation retries (k_riccati_retry): elements whose first sweep fails the PSD
    // test, up to retry_cap of them per launch, evaluate the next retry_m values of the mu schedule
    // of backward_sweep_regularized (MultiPhaseDDP.cpp:141-181) at once; 0 = sequential only
    int retry_cap, retry_m;
    int hcap;  // solver-info history entries per element (Bufs::hist)
    int elem_layout;  // 1: element b's layout is Bufs::lay[b] (N, s0, k0, ss above unused)
    int n_pairs;      // sweep waves: Bufs::pairs [n_pairs][2] (elem_layout), else ceil(B / 2)
    int store_value;  // the sweep writes G[0], H[0] of every phase (Bufs::value0)
    // single shooting (HSDDP_OPTION::MS = false, MultiPhaseDDP.cpp:326-331; SinglePhase.cpp:211-220):
    // no linear rollout, the sweep forms dV_1 / dV_2 (SinglePhase.cpp:359-362) and the merit, and the
    // rollout simulates every phase from its first state (k_rollout_ss)
    int ms0;
    // diagnostic (HSDDP_TRACE=1, read at create / option changes): every finished line search records
    // (trials, accepted, the sweep's regularisation) of its inner iteration in Bufs::dbg (k_decide)
    int trace;
};

// one element deferred to the parallel retry: its index and the regularisation of its failed sweep
struct RetryEntry {
    int b, pad;
    double reg;
};

// The constraint objects' stored values (IneqConstrData::g, TConstrData::h; ConstraintsBase.h:
// 12-55) live on from trial to trial and from solve to solve.  A rollout that returns at the knot
// whose simulated state breaks the 1e6 bound (SinglePhase.cpp:205-208) computes no constraint
// value from there on, and a new problem, a pushed-back knot and a new touchdown constraint start
// from zero (create_data, PathConstraintBase::push_back).  Stored explicitly only where they are
// not a function of the working rows:
//  * GRF (g = A_leg f): Bufs::cf_flag[b][kc] = 1 when the stored values of control knot kc come
//    from the forces Bufs::cf_u[b][kc] (the break knot's earlier control row; zeros for a new
//    problem) rather than from the working control row U[kc];
//  * touchdown (h = foot height at X_i[N] - ground): a constraint whose h was never computed since
//    it was registered (0) carries TD_STALE in its td_mask entry; every other one's h is that of
//    the working X_i[N] (the rollout that computes h also sets X_i[N], SinglePhase.cpp:196-227).
// ElemState::ovr / td_stale: some flag of the element may be set; both survive k_reset_elements.
// The per-knot GRF flags are read only while ovr is 1 (their contents are arbitrary while it is 0:
// the fix-up that sets it clears them first, and the shift carries them only then).  A rollout
// that passes every knot resets ovr; one that completes phase i clears its TD_STALE bits (k_decide).
constexpr int TD_STALE = 0x20;

struct ElemState {
    double cost, feas, merit, merit_rho, dV1, dV2, reg;
    double max_t, max_p, max_t_prev, max_p_prev, cost_prev, merit_prev, feas_prev;
    int done, inner_done, ls_active, accepted, status, iters, outer_iters, n_ls;
    int hist_n;  // entries pushed to the solver-info history (MultiPhaseDDP.cpp:277-280, 368-371)
    int ovr, td_stale;  // (above; persistent across solves)
};

struct Bufs {
    const int *contacts;                   // [B][P+1][4]
    const double *x0;                      // [B][24]
    const double *ref_x, *ref_u, *ref_foot; // [Bref][S][24|24|12]
    // the same references entry-major, for kernels with one slot per lane (a lane's entry j is next to
    // its neighbours': one contiguous piece per wave instead of 64 rows): [REF_COLS][ref_tw], column
    // r = (ref_per_element ? b : 0) S + s, entries ref_x 0 .. 23, ref_u 24 .. 47, ref_foot 48 .. 59.
    // Refreshed from the rows by launch_ref_columns whenever the rows change (hsddp_api.cpp)
    double *ref_t;
    size_t ref_tw;
    // Trajectory::update_nominal_vals without copies: each element's nominal (Xbar, Ubar) and working
    // (X, U, Defect) rows live in two of three buffers, sel[b] bits 0-1 = the nominal's index, bits
    // 2-3 = the working one's.  A line-search trial writes the third (trial_buf: neither, so that a
    // diverged trial can keep the working rows past its break); accepting it makes it the nominal
    // and the working buffer, rejecting it the working one (quirk A2).
    // One allocation per set, buffer q at q x the set's stride (xbuf / dbuf / ubuf): kernels hold one
    // base pointer per set, not three.
    double *X3, *D3, *dX;                  // X3, D3: [3][B][S_cap][24]
    double *U3, *dU, *du;                  // U3: [3][B][Kc][24]
    size_t xs3, us3;                       // set strides (doubles): B x S_cap x 24, B x Kc x 24
    int rows3, urows3;                     // the same in rows: B x S_cap, B x Kc
    int *sel;                              // [B]
    double *cf_u;                          // [B][Kc][12] forces of the stored GRF values where cf_flag
    int *cf_flag;                          // [B][Kc] (above)
    double *K, *lq, *term;
    double *reb_delta, *reb_eps, *al_sigma, *al_lambda, *term_h;
    int *td_mask;                          // [B][P][MTD] (0: no constraint in that slot)
    double *slot_cost, *slot_feas, *slot_viol;
    int *slot_div;
    // fp32 Riccati mode only: LQ records [B][Kc][LQW32], gains [B][Kc][KCW], Defect copy [B][S][24]
    float *lq32, *K32, *def32;
    ElemState *el;
    int *counter;                          // [8] host-visible activity counters [0..2], stat sums [4..5]
    // [LS_LIVE] per line-search trial t of the current inner iteration: 1 when an element is still
    // searching after trial t (k_decide), zeroed at the iteration's start (k_lq): later trials of a
    // batch with none left return at once
    int *ls_live;
    // parallel regularisation retries: deferred elements [retry_cap], their count, per attempt a
    // success flag [retry_cap][retry_m] and the attempt's gains / dU rows [retry_cap][retry_m][Kc][..]
    RetryEntry *retry_list;
    int *retry_count, *retry_flag;
    void *retry_K;                         // real (fp64, or fp32 in the C5 mode) [..][KCW]
    double *retry_dU;                      // [..][24]
    double *retry_dv;                      // [retry_cap][retry_m] the attempt's sum of Qu^T dU (single shooting)
    unsigned long long *dbg;               // [B][16] diagnostic builds only (in-kernel stamps)
    // get_solver_info buffers (MultiPhaseDDP.cpp:532-541): per element hcap entries of
    // (actual_cost, dynamics feasibility, max terminal violation, max path violation)
    float *hist;                           // [B][hcap][4]
    const Layout *lay;                     // [B] per-element layouts (Params::elem_layout)
    const int *pairs;                      // [n_pairs][2] the sweep's element pairs (same layout; -1 = none)
    double *value0;                        // [B][P][24 + 576]: G[0], H[0] per phase (store_value)
};

// kernel launchers (hsddp_kernels.hip)
// tix: the trial's index in the inner iteration's line search (-1: the initial rollout)
// (last: this trial is the search's last step size — used when the rollout launch also decides)
void launch_rollout(const Params &p, const Bufs &d, double eps, int last, int init, int tix, hipStream_t st);
void launch_decide(const Params &p, const Bufs &d, double eps, int last, int init, int tix, hipStream_t st);
// nominal rows of every element into buffer 0 (Bufs::sel bit 0 cleared), for host transfers
void launch_normalize(const Params &p, const Bufs &d, hipStream_t st);
// every element's working rows back at its nominal ones (sel), its Defect rows zero
void launch_reset_working(const Params &p, const Bufs &d, hipStream_t st);
void launch_lq(const Params &p, const Bufs &d, hipStream_t st);
void launch_riccati(const Params &p, const Bufs &d, hipStream_t st);
void launch_lin_rollout(const Params &p, const Bufs &d, hipStream_t st);
void launch_outer_begin(const Params &p, const Bufs &d, hipStream_t st);
void launch_reb_update(const Params &p, const Bufs &d, hipStream_t st);
void launch_outer_end(const Params &p, const Bufs &d, hipStream_t st);
void launch_reset_elements(const Params &p, const Bufs &d, hipStream_t st);
void launch_init_params(const Params &p, const Bufs &d, hipStream_t st);
// TD_PENDING touchdown masks resolved from the contact rows (after new contacts are uploaded)
void launch_resolve_td(const Params &p, const Bufs &d, hipStream_t st);
// Bufs::ref_t from the reference rows (Bref x S columns)
constexpr int REF_COLS = 24 + 24 + 12;  // (ref_x, ref_u, ref_foot widths)
void launch_ref_columns(const Params &p, const Bufs &d, int Bref, hipStream_t st);
void launch_count(const Params &p, const Bufs &d, int which, hipStream_t st);
void launch_stat_sums(const Params &p, const Bufs &d, hipStream_t st);
// dst[c][n] = src[n] for c < copies
void launch_broadcast(double *dst, const double *src, size_t n, size_t copies, hipStream_t st);

// model primitives
void launch_model_dynamics(const double *x, const double *u, const double *c, double dt, double *xn, int n,
                           hipStream_t st);
void launch_model_partial(const double *x, const double *u, const double *c, double dt, double *A, double *B,
                          int n, hipStream_t st);
void launch_model_foot(const double *x, const int *leg, double *p, double *J, int n, hipStream_t st);
void launch_model_reset(const double *x, const int *c, const int *cn, double *xn, double *Px, int n,
                        hipStream_t st);
void launch_model_running_cost(const Params &p, const double *x, const double *u, const int *c, const double *xr,
                               const double *ur, const double *pf, int terms, double *l, double *lx, double *lu,
                               double *lxx, double *luu, int n, hipStream_t st);
void launch_model_terminal_cost(const Params &p, const double *x, const int *c, const double *xr, const double *pf,
                                int terms, double *Phi, double *Phix, double *Phixx, int n, hipStream_t st);
void launch_model_grf(const double *u, const int *c, double mu, double *g, double *gu, int n, hipStream_t st);
void launch_model_touchdown(const double *x, const int *c, const int *cn, double ground, double *h, double *hx, int n,
                            hipStream_t st);

}  // namespace hsddp
