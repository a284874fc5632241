/*
 * hsddp_oracle.c — TEST INFRASTRUCTURE ONLY (see hkd_oracle.h).
 *
 * Line-by-line CPU restatement of the reference multi-phase HS-DDP solve for the HKD problem:
 *   MultiPhaseDDP::solve / line_search / backward_sweep(_regularized) / linear_rollout /
 *     hybrid_rollout / compute_cost / measure_dynamics_feasibility
 *                                           HSDDPSolver/source/MultiPhaseDDP.cpp:20-530
 *   SinglePhase::{linear_rollout, hybrid_rollout, compute_cost, LQ_approximation,
 *     backward_sweep, update_*_with_*}     HSDDPSolver/source/SinglePhase.cpp:144-426
 *   ReB / AL closed forms and parameter updates    HSDDPSolver/header/ConstraintsBase.h:168-399
 *   HKD costs        HKDMPC/HKD-TrajOpt/HKDCost.{h,cpp}; SinglePhaseInterface.cpp:55-166
 *   HKD constraints  HKDMPC/HKD-TrajOpt/HKDConstraints.cpp:7-171
 *   HKD reset map    HKDMPC/HKD-TrajOpt/HKDReset.h:41-136 (via hkd_model_ref.c)
 * with Eigen's LDLT PSD test (diagonal pivoting, Eigen 3.3 sign rules; Eigen is not vendored by
 * the reference — version unpinned, README.md:11) and an explicit partial-pivot LU inverse for
 * Matrix::inverse().  Every quirk of SURVEY.md Appendix A is reproduced; note that with
 * alpha = 0.1 the line search `while (eps > 1e-3)` runs FOUR trials (1, .1, .01, .001) because
 * 0.1*0.1*0.1 rounds above 1e-3 in binary64.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <stdio.h>
#include "hkd_oracle.h"

#define NX 24
#define NN 576
#define MAXP 64

/* ----------------------------------------------------------------------------------------- */
void orc_default_options(orc_options *o)
{
    /* HSDDP_OPTION defaults (HSDDP_CompoundTypes.h:18-60) overlaid with the values
       loadHSDDPSetting reads from settings/ddp_setting.info (:62-87).  update_regularization and
       smooth_active are NOT read by the loader, so they keep their defaults (quirk A1). */
    o->alpha = 0.1; o->gamma = 0.01; o->update_penalty = 5; o->update_relax = 1;
    o->update_regularization = 2; o->update_ReB = 1;
    o->max_DDP_iter = 10; o->max_AL_iter = 5; o->max_DDP_iter_runtime = 1; o->max_AL_iter_runtime = 2;
    o->cost_thresh = 1e-3; o->tconstr_thresh = 1e-3; o->pconstr_thresh = 1e-3; o->dynamics_feas_thresh = 1e-3;
    o->merit_rho = 1e4; o->merit_scale = 0.2; o->merit_offset = 1e2;
    o->AL_active = 1; o->ReB_active = 1; o->smooth_active = 0; o->MS = 1; o->nsteps_per_node = 1;
    o->no_early_exit = 0;
}

void orc_default_weights(orc_weights *w)
{
    /* HKDTrackingCost (HKDCost.h:8-38), HKDFootPlaceReg (HKDCost.h:41-70, HKDCost.cpp:49,63) */
    const double qe[3] = {1, 4, 5}, qp[3] = {1, 1, 30}, qo[3] = {.2, .2, .2}, qv[3] = {4, 1, .5};
    const double sc[24] = {1, 1, 2, 1, 1, 20, .3, .3, .3, 1, 3, 1,
                           .01, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01};
    for (int i = 0; i < 3; ++i) { w->q_eul[i] = qe[i]; w->q_pos[i] = qp[i]; w->q_omega[i] = qo[i]; w->q_v[i] = qv[i]; }
    w->q_qJ = 0.2;
    for (int i = 0; i < 24; ++i) w->qf_scale[i] = sc[i];
    w->qf_gain = 20; w->r_grf = 0.2; w->r_qJd = 0.1;
    w->foot_w[0] = 3; w->foot_w[1] = 1; w->foot_w[2] = 0; w->foot_gain = 20;
    w->foot_term_cost = 10; w->foot_term_grad = 20;
}

/* ----------------------------------------------------------------------------------------- */
typedef struct {
    const orc_problem *p;
    const orc_options *o;
    orc_element *e;
    int P, S, Kc;
    int N[MAXP], s0[MAXP], k0[MAXP];
    int c[MAXP + 1][4];
    /* phase-constant cost matrices (diagonals) */
    double Qd[MAXP][NX], Qfd[MAXP][NX], Rd[NX];
    double Qfoot[MAXP][12];
    /* LQ data */
    double *A, *B;                      /* [Kc][NN] */
    double *l, *lx, *lu, *lxx, *luu, *lux; /* per control slot */
    double *Phi, *Phix, *Phixx;         /* per phase */
    double *G, *H;                      /* per state slot */
    double *Xsim;                       /* [S][NX] */
    double *g;                          /* [Kc][20] stored GRF constraint values (orc_element.grf_g) */
    double *td_h;                       /* [P][ORC_MAX_TD][4] stored touchdown values (orc_element.td_h) */
    double hx[MAXP][4][NX];
    double pviol[MAXP], tviol[MAXP];
    double phase_cost[MAXP], dV1p[MAXP], dV2p[MAXP];
    /* multi-phase scalars (MultiPhaseDDP.h:437-451) */
    double actual_cost, merit, feas, dV_1, dV_2, max_tconstr, max_pconstr, max_tconstr_prev,
        max_pconstr_prev, merit_rho;
    int n_ls;
} ctx_t;

static int n_stance(const int *c) { return c[0] + c[1] + c[2] + c[3]; }
/* the legs of phase i's touchdown constraints (union of their masks) */
static int td_legs(const orc_element *e, int i)
{
    int u = 0;
    for (int j = 0; j < ORC_MAX_TD; ++j) u |= e->td_mask[i * ORC_MAX_TD + j];
    return u & 15;
}
static int n_touchdown(const int *c, const int *cn)
{
    int n = 0;
    for (int l = 0; l < 4; ++l) n += (c[l] == 0 && cn[l] == 1);
    return n;
}

static void setup_costs(ctx_t *C)
{
    const orc_weights *w = &C->p->w;
    for (int i = 0; i < C->P; ++i) {
        double *q = C->Qd[i];
        for (int j = 0; j < 3; ++j) { q[j] = w->q_eul[j]; q[3 + j] = w->q_pos[j]; q[6 + j] = w->q_omega[j]; q[9 + j] = w->q_v[j]; }
        for (int l = 0; l < 4; ++l)
            for (int j = 0; j < 3; ++j) q[12 + 3 * l + j] = w->q_qJ * (1 - C->c[i][l]);
        for (int j = 0; j < NX; ++j) C->Qfd[i][j] = w->qf_gain * w->qf_scale[j] * q[j]; /* Qf = 20 diag(scale) Q */
        for (int l = 0; l < 4; ++l)
            for (int j = 0; j < 3; ++j) C->Qfoot[i][3 * l + j] = w->foot_gain * w->foot_w[j] * C->c[i][l];
    }
    for (int j = 0; j < 12; ++j) { C->Rd[j] = w->r_grf; C->Rd[12 + j] = w->r_qJd; }
}

/* foot regularisation residual d_prel (HKDCost.cpp:10-13) */
static void foot_residual(const ctx_t *C, int s, const double *x, double *d)
{
    const double *xr = C->e->ref_x + (size_t)s * NX, *pf = C->e->ref_foot + (size_t)s * 12;
    for (int l = 0; l < 4; ++l)
        for (int j = 0; j < 3; ++j)
            d[3 * l + j] = (x[12 + 3 * l + j] - x[3 + j]) - (pf[3 * l + j] - xr[3 + j]);
}

/* D^T W d with D = dprel_dx (HKDCost.h:157-164):  rows 3l+j: -c_l at col 3+j, +c_l at col 12+3l+j */
static void foot_grad(const int *c, const double *W, const double *d, double scale, double *gx)
{
    for (int l = 0; l < 4; ++l)
        for (int j = 0; j < 3; ++j) {
            double v = scale * c[l] * W[3 * l + j] * d[3 * l + j];
            gx[3 + j] += -v;
            gx[12 + 3 * l + j] += v;
        }
}

static void foot_hess(const int *c, const double *W, double scale, double *Hx)
{
    for (int l = 0; l < 4; ++l)
        for (int j = 0; j < 3; ++j) {
            double v = scale * c[l] * c[l] * W[3 * l + j];
            int a = 3 + j, b = 12 + 3 * l + j;
            Hx[a * NX + a] += v; Hx[b * NX + b] += v;
            Hx[a * NX + b] -= v; Hx[b * NX + a] -= v;
        }
}

/* GRF friction pyramid rows (HKDConstraints.cpp:7-37, mu = 0.7) applied to leg l's force */
static void grf_rows(double mu, const double *f, double *g)
{
    g[0] = f[2];
    g[1] = -f[0] + mu * f[2];
    g[2] = f[0] + mu * f[2];
    g[3] = -f[1] + mu * f[2];
    g[4] = f[1] + mu * f[2];
}
static const double GRF_ROW[5][3] = {{0, 0, 1}, {-1, 0, 1}, {1, 0, 1}, {0, -1, 1}, {0, 1, 1}}; /* z coef * mu */

/* ---- phase-level routines ----------------------------------------------------------------- */

/* SinglePhase::hybrid_rollout (SinglePhase.cpp:181-233).  Shooting states SS_set = {0 .. ss-1}
   (every state unless orc_problem.shooting says otherwise: HKDProblem::update leaves a new last
   phase of horizon <= 2 with an empty set, HKDProblem.cpp:203-216): X = Xbar + eps dX there,
   X = Xsim (X[0] = x_init) elsewhere. */
static int phase_hybrid_rollout(ctx_t *C, int i, double eps, const double *x_init)
{
    orc_element *e = C->e;
    const int N = C->N[i], s0 = C->s0[i], k0 = C->k0[i];
    const int ss = C->p->shooting ? C->p->shooting[i] : N + 1;
    double cd[4];
    for (int l = 0; l < 4; ++l) cd[l] = C->c[i][l];
    double *X = e->X, *Xbar = e->Xbar, *U = e->U, *Ubar = e->Ubar;
    memcpy(C->Xsim + (size_t)s0 * NX, x_init, sizeof(double) * NX);
    if (ss > 0)
        for (int j = 0; j < NX; ++j) X[s0 * NX + j] = Xbar[s0 * NX + j] + eps * e->dX[s0 * NX + j];
    else
        memcpy(X + (size_t)s0 * NX, x_init, sizeof(double) * NX);
    double pv = 0;
    for (int k = 0; k < N; ++k) {
        int s = s0 + k, kc = k0 + k;
        const double *Kk = e->K + (size_t)kc * NN;
        double dx[NX];
        for (int j = 0; j < NX; ++j) dx[j] = X[s * NX + j] - Xbar[s * NX + j];
        for (int r = 0; r < NX; ++r) {
            double acc = 0;
            for (int j = 0; j < NX; ++j) acc += Kk[r * NX + j] * dx[j];
            U[kc * NX + r] = Ubar[kc * NX + r] + eps * e->dU[kc * NX + r] + acc;
        }
        double *xs = C->Xsim + (size_t)(s + 1) * NX;
        orc_hkd_step(X + s * NX, U + kc * NX, C->p->dt, cd, xs);
        double nrm = 0;
        for (int j = 0; j < NX; ++j) nrm += xs[j] * xs[j];
        if (sqrt(nrm) > 1e6) return 0;
        if (k + 1 < ss && C->o->MS)
            for (int j = 0; j < NX; ++j) X[(s + 1) * NX + j] = Xbar[(s + 1) * NX + j] + eps * e->dX[(s + 1) * NX + j];
        else
            memcpy(X + (size_t)(s + 1) * NX, xs, sizeof(double) * NX);
        /* GRFConstraint::compute_violation + update_max_violation(k) */
        if (n_stance(C->c[i])) {
            double mk = 0;
            for (int l = 0; l < 4; ++l) {
                if (!C->c[i][l]) continue;
                double *gg = C->g + (size_t)kc * 20 + 5 * l;
                grf_rows(C->p->mu_fric, U + kc * NX + 3 * l, gg);
                for (int r = 0; r < 5; ++r) mk = fmin(mk, gg[r]);
            }
            pv = fmin(pv, mk);
        }
    }
    C->pviol[i] = pv;
    /* TouchDownConstraint::compute_violation at X[N] (HKDConstraints.cpp:69-118) of every
       touchdown constraint of the phase: the foot heights of their legs */
    double tv = 0;
    const double *xN = X + (size_t)(s0 + N) * NX;
    const int tdu = td_legs(C->e, i);
    double hl[4] = {0, 0, 0, 0};
    for (int l = 0; l < 4; ++l) {
        if (!((tdu >> l) & 1)) continue;
        double pf[3];
        orc_foot_position(l, xN + 3, xN, xN + 12 + 3 * l, pf);
        hl[l] = pf[2] - C->p->ground_height;
        tv = fmax(tv, fabs(hl[l]));
    }
    /* each constraint's data[i].h for its impact feet */
    for (int j = 0; j < ORC_MAX_TD; ++j) {
        const int m = e->td_mask[i * ORC_MAX_TD + j];
        for (int l = 0; l < 4; ++l)
            if ((m >> l) & 1) C->td_h[(i * ORC_MAX_TD + j) * 4 + l] = hl[l];
    }
    C->tviol[i] = tv;
    /* compute_defect (TrajectoryManagement.cpp:210-217) */
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < NX; ++j)
            e->Defect[(s0 + k) * NX + j] = C->Xsim[(s0 + k) * NX + j] - X[(s0 + k) * NX + j];
    return 1;
}

/* ReB closed forms (ConstraintsBase.h:204-263) */
static double reb_cost(double g, double delta)
{
    if (g > delta) return -log(g);
    double t = (g - 2 * delta) / delta;
    return .5 * (t * t - 1) - log(delta);
}
static void reb_derivs(double g, double delta, double *d1, double *d2)
{
    if (g > delta) { *d1 = -1.0 / g; *d2 = pow(g, -2); }
    else { *d1 = (g - 2 * delta) / delta / delta; *d2 = pow(delta, -2); }
}

/* SinglePhase::compute_cost (SinglePhase.cpp:235-262) */
static void phase_compute_cost(ctx_t *C, int i)
{
    orc_element *e = C->e;
    const int N = C->N[i], s0 = C->s0[i], k0 = C->k0[i];
    const double dt = C->p->dt;
    double cost = 0;
    for (int k = 0; k < N; ++k) {
        int s = s0 + k, kc = k0 + k;
        const double *x = e->X + s * NX, *u = e->U + kc * NX;
        const double *xr = e->ref_x + (size_t)s * NX, *ur = e->ref_u + (size_t)s * NX;
        /* QuadraticTrackingCost::running_cost (SinglePhaseInterface.cpp:55-71) */
        double lt = 0, lu_ = 0;
        for (int j = 0; j < NX; ++j) { double d = x[j] - xr[j]; lt += d * C->Qd[i][j] * d; }
        lt = 0.5 * lt;
        for (int j = 0; j < NX; ++j) { double d = u[j] - ur[j]; lu_ += d * C->Rd[j] * d; }
        lt += 0.5 * lu_;
        lt *= dt;
        /* HKDFootPlaceReg::running_cost (HKDCost.cpp:5-20) */
        double d[12], lf = 0;
        foot_residual(C, s, x, d);
        for (int j = 0; j < 12; ++j) lf += d[j] * C->Qfoot[i][j] * d[j];
        lf = .5 * lf;
        lf *= dt;
        double l = 0 + lt + lf;
        if (C->o->ReB_active && n_stance(C->c[i])) {
            double rc = 0;
            for (int lg = 0; lg < 4; ++lg) {
                if (!C->c[i][lg]) continue;
                for (int r = 0; r < 5; ++r) {
                    int q = kc * 20 + 5 * lg + r;
                    rc += e->reb_eps[q] * reb_cost(C->g[q], e->reb_delta[q]);
                }
            }
            l += dt * rc;
        }
        C->l[kc] = l;
        cost += l;
    }
    /* terminal: QuadraticTrackingCost::terminal_cost + HKDFootPlaceReg::terminal_cost */
    int s = s0 + N;
    const double *x = e->X + s * NX, *xr = e->ref_x + (size_t)s * NX;
    double phi = 0;
    for (int j = 0; j < NX; ++j) { double d = x[j] - xr[j]; phi += d * C->Qfd[i][j] * d; }
    phi *= 0.5;
    double d[12], pf = 0;
    foot_residual(C, s, x, d);
    for (int j = 0; j < 12; ++j) pf += d[j] * C->Qfoot[i][j] * d[j];
    phi = 0 + phi + C->p->w.foot_term_cost * pf;
    if (C->o->AL_active) { /* update_terminal_cost_with_tconstr (SinglePhase.cpp:401-411): per
                               constraint, compute_AL_cost (ConstraintsBase.h:374-382), Phi += */
        for (int j = 0; j < ORC_MAX_TD; ++j) {
            const int m = e->td_mask[i * ORC_MAX_TD + j];
            if (!m) continue;
            double al = 0;
            for (int l = 0; l < 4; ++l) {
                if (!((m >> l) & 1)) continue;
                const int q = (i * ORC_MAX_TD + j) * 4 + l;
                double sg = e->al_sigma[q], lm = e->al_lambda[q], hh = C->td_h[q];
                al += 0.5 * sg * hh * hh;
                al += lm * hh;
            }
            phi += al;
        }
    }
    C->Phi[i] = phi;
    C->phase_cost[i] = cost + phi;
}

/* SinglePhase::LQ_approximation (SinglePhase.cpp:264-296) */
static void phase_LQ(ctx_t *C, int i)
{
    orc_element *e = C->e;
    const int N = C->N[i], s0 = C->s0[i], k0 = C->k0[i];
    const double dt = C->p->dt;
    double cd[4];
    for (int l = 0; l < 4; ++l) cd[l] = C->c[i][l];
    for (int k = 0; k < N; ++k) {
        int s = s0 + k, kc = k0 + k;
        const double *x = e->X + s * NX, *u = e->U + kc * NX;
        const double *xr = e->ref_x + (size_t)s * NX, *ur = e->ref_u + (size_t)s * NX;
        orc_hkd_partial(x, u, dt, cd, C->A + (size_t)kc * NN, C->B + (size_t)kc * NN);
        double *lx = C->lx + kc * NX, *lu = C->lu + kc * NX;
        double *lxx = C->lxx + (size_t)kc * NN, *luu = C->luu + (size_t)kc * NN, *lux = C->lux + (size_t)kc * NN;
        memset(lx, 0, sizeof(double) * NX); memset(lu, 0, sizeof(double) * NX);
        memset(lxx, 0, sizeof(double) * NN); memset(luu, 0, sizeof(double) * NN); memset(lux, 0, sizeof(double) * NN);
        for (int j = 0; j < NX; ++j) {
            lx[j] += dt * C->Qd[i][j] * (x[j] - xr[j]);
            lu[j] += dt * C->Rd[j] * (u[j] - ur[j]);
            lxx[j * NX + j] += dt * C->Qd[i][j];
            luu[j * NX + j] += dt * C->Rd[j];
        }
        double d[12];
        foot_residual(C, s, x, d);
        foot_grad(C->c[i], C->Qfoot[i], d, dt, lx);
        foot_hess(C->c[i], C->Qfoot[i], dt, lxx);
        if (C->o->ReB_active && n_stance(C->c[i])) { /* update_running_cost_par_with_pconstr */
            double gu[NX], hu[NN];
            memset(gu, 0, sizeof(gu)); memset(hu, 0, sizeof(hu));
            for (int lg = 0; lg < 4; ++lg) {
                if (!C->c[i][lg]) continue;
                for (int r = 0; r < 5; ++r) {
                    int q = kc * 20 + 5 * lg + r;
                    double d1, d2, ep = e->reb_eps[q], row[3];
                    reb_derivs(C->g[q], e->reb_delta[q], &d1, &d2);
                    for (int j = 0; j < 3; ++j) row[j] = (j == 2) ? GRF_ROW[r][2] * C->p->mu_fric : GRF_ROW[r][j];
                    if (r == 0) row[2] = 1.0;
                    for (int a = 0; a < 3; ++a) {
                        gu[3 * lg + a] += ep * d1 * row[a];
                        for (int b = 0; b < 3; ++b) hu[(3 * lg + a) * NX + 3 * lg + b] += ep * (d2 * row[a] * row[b]);
                    }
                }
            }
            for (int j = 0; j < NX; ++j) lu[j] += dt * gu[j];
            for (int j = 0; j < NN; ++j) luu[j] += dt * hu[j];
        }
    }
    /* terminal partials */
    int s = s0 + N;
    const double *x = e->X + s * NX, *xr = e->ref_x + (size_t)s * NX;
    double *Px_ = C->Phix + (size_t)i * NX, *Pxx = C->Phixx + (size_t)i * NN;
    memset(Px_, 0, sizeof(double) * NX); memset(Pxx, 0, sizeof(double) * NN);
    for (int j = 0; j < NX; ++j) { Px_[j] += C->Qfd[i][j] * (x[j] - xr[j]); Pxx[j * NX + j] += C->Qfd[i][j]; }
    double d[12];
    foot_residual(C, s, x, d);
    foot_grad(C->c[i], C->Qfoot[i], d, C->p->w.foot_term_grad, Px_);
    foot_hess(C->c[i], C->Qfoot[i], C->p->w.foot_term_grad, Pxx);
    if (C->o->AL_active) { /* TouchDownConstraint::compute_partial (HKDConstraints.cpp:120-171) of the
                               constraint legs, then per constraint compute_AL_partials
                               (ConstraintsBase.h:383-399) and Phix += grad, Phixx += hess
                               (update_terminal_cost_par_with_tconstr, SinglePhase.cpp:414-426) */
        const int tdu = td_legs(e, i);
        for (int l = 0; l < 4; ++l) {
            if (!((tdu >> l) & 1)) continue;
            double J[54], hxv[NX];
            orc_foot_jacobian(l, x + 3, x, x + 12 + 3 * l, J);
            memset(hxv, 0, sizeof(hxv));
            for (int j = 0; j < 3; ++j) { hxv[j] = J[2 * 18 + 3 + j]; hxv[3 + j] = J[2 * 18 + j]; }
            for (int j = 0; j < 12; ++j) hxv[12 + j] = J[2 * 18 + 6 + j];
            memcpy(C->hx[i][l], hxv, sizeof(hxv));
        }
        for (int j = 0; j < ORC_MAX_TD; ++j) {
            const int m = e->td_mask[i * ORC_MAX_TD + j];
            if (!m) continue;
            double grad[NX], hess[NN];
            memset(grad, 0, sizeof grad);
            memset(hess, 0, sizeof hess);
            for (int l = 0; l < 4; ++l) {
                if (!((m >> l) & 1)) continue;
                const int q = (i * ORC_MAX_TD + j) * 4 + l;
                const double *hxv = C->hx[i][l];
                double sg = e->al_sigma[q], lm = e->al_lambda[q], hh = C->td_h[q];
                double a1 = sg * hh + lm, a2 = sg * (1 + hh) + lm; /* quirk A4 */
                for (int a = 0; a < NX; ++a) {
                    grad[a] += a1 * hxv[a];
                    for (int b = 0; b < NX; ++b) hess[a * NX + b] += a2 * (hxv[a] * hxv[b]);
                }
            }
            for (int a = 0; a < NX; ++a) Px_[a] += grad[a];
            for (int a = 0; a < NN; ++a) Pxx[a] += hess[a];
        }
    }
}

/* ---- dense helpers ------------------------------------------------------------------------ */
static void matT_vec(const double *M, const double *v, double *o) /* o = M^T v */
{
    for (int j = 0; j < NX; ++j) o[j] = 0;
    for (int i = 0; i < NX; ++i) {
        double vi = v[i];
        if (vi == 0) continue;
        for (int j = 0; j < NX; ++j) o[j] += M[i * NX + j] * vi;
    }
}
static void mat_vec(const double *M, const double *v, double *o)
{
    for (int i = 0; i < NX; ++i) {
        double a = 0;
        for (int j = 0; j < NX; ++j) a += M[i * NX + j] * v[j];
        o[i] = a;
    }
}
static void mat_mul(const double *X, const double *Y, double *Z) /* Z = X Y */
{
    for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) {
            double a = 0;
            for (int k = 0; k < NX; ++k) a += X[i * NX + k] * Y[k * NX + j];
            Z[i * NX + j] = a;
        }
}
static void matT_mul(const double *X, const double *Y, double *Z) /* Z = X^T Y */
{
    for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) {
            double a = 0;
            for (int k = 0; k < NX; ++k) a += X[k * NX + i] * Y[k * NX + j];
            Z[i * NX + j] = a;
        }
}

/* Eigen 3.3 LDLT<MatrixXd>::compute(M).isPositive(): symmetric diagonal pivoting on the lower
 * triangle (ldlt_inplace<Lower>::unblocked), sign tracking PositiveSemiDef/NegativeSemiDef/
 * Indefinite/ZeroSign; isPositive() == (sign == PositiveSemiDef || sign == ZeroSign). */
static int eigen_ldlt_is_positive(const double *M)
{
    enum { ZeroSign, PositiveSemiDef, NegativeSemiDef, Indefinite };
    double W[NN], temp[NX];
    for (int i = 0; i < NX; ++i)
        for (int j = 0; j < NX; ++j) W[i * NX + j] = (i >= j) ? M[i * NX + j] : M[j * NX + i];
    int sign = ZeroSign;
    int found_zero_pivot = 0;
    for (int k = 0; k < NX; ++k) {
        int big = k;
        double bv = fabs(W[k * NX + k]);
        for (int i = k + 1; i < NX; ++i)
            if (fabs(W[i * NX + i]) > bv) { bv = fabs(W[i * NX + i]); big = i; }
        if (big != k) { /* symmetric permutation */
            for (int j = 0; j < NX; ++j) { double t = W[k * NX + j]; W[k * NX + j] = W[big * NX + j]; W[big * NX + j] = t; }
            for (int j = 0; j < NX; ++j) { double t = W[j * NX + k]; W[j * NX + k] = W[j * NX + big]; W[j * NX + big] = t; }
        }
        int rs = NX - k - 1;
        if (k > 0) {
            double s = 0;
            for (int j = 0; j < k; ++j) temp[j] = W[j * NX + j] * W[k * NX + j];
            for (int j = 0; j < k; ++j) s += W[k * NX + j] * temp[j];
            W[k * NX + k] -= s;
            for (int r = k + 1; r < NX; ++r) {
                double a = 0;
                for (int j = 0; j < k; ++j) a += W[r * NX + j] * temp[j];
                W[r * NX + k] -= a;
            }
        }
        double akk = W[k * NX + k];
        int valid = fabs(akk) > 0;
        if (k == 0 && !valid) return 1; /* whole diagonal zero: ZeroSign -> isPositive */
        if (rs > 0 && valid)
            for (int r = k + 1; r < NX; ++r) W[r * NX + k] /= akk;
        if (!valid) found_zero_pivot = 1; /* (ret flag is irrelevant to isPositive) */
        if (sign == PositiveSemiDef) { if (akk < 0) sign = Indefinite; }
        else if (sign == NegativeSemiDef) { if (akk > 0) sign = Indefinite; }
        else if (sign == ZeroSign) { if (akk > 0) sign = PositiveSemiDef; else if (akk < 0) sign = NegativeSemiDef; }
        /* the full symmetric swap above reproduces Eigen's lower-triangle swaps exactly; the
           stale upper-triangle entries it moves around are never read */
    }
    (void)found_zero_pivot;
    return sign == PositiveSemiDef || sign == ZeroSign;
}

/* Matrix<double,24,24>::inverse() via LU with partial pivoting */
static void lu_inverse(const double *M, double *Inv)
{
    double LU[NN];
    int piv[NX];
    memcpy(LU, M, sizeof(LU));
    for (int i = 0; i < NX; ++i) piv[i] = i;
    for (int k = 0; k < NX; ++k) {
        int p = k;
        double pv = fabs(LU[k * NX + k]);
        for (int i = k + 1; i < NX; ++i)
            if (fabs(LU[i * NX + k]) > pv) { pv = fabs(LU[i * NX + k]); p = i; }
        if (p != k) {
            for (int j = 0; j < NX; ++j) { double t = LU[k * NX + j]; LU[k * NX + j] = LU[p * NX + j]; LU[p * NX + j] = t; }
            int t = piv[k]; piv[k] = piv[p]; piv[p] = t;
        }
        double d = LU[k * NX + k];
        for (int i = k + 1; i < NX; ++i) {
            double f = LU[i * NX + k] / d;
            LU[i * NX + k] = f;
            for (int j = k + 1; j < NX; ++j) LU[i * NX + j] -= f * LU[k * NX + j];
        }
    }
    for (int col = 0; col < NX; ++col) {
        double y[NX];
        for (int i = 0; i < NX; ++i) {
            double a = (piv[i] == col) ? 1.0 : 0.0;
            for (int j = 0; j < i; ++j) a -= LU[i * NX + j] * y[j];
            y[i] = a;
        }
        for (int i = NX - 1; i >= 0; --i) {
            double a = y[i];
            for (int j = i + 1; j < NX; ++j) a -= LU[i * NX + j] * y[j];
            y[i] = a / LU[i * NX + i];
        }
        for (int i = 0; i < NX; ++i) Inv[i * NX + col] = y[i];
    }
}

/* SinglePhase::backward_sweep (SinglePhase.cpp:298-367) */
static int phase_backward(ctx_t *C, int i, double reg, const double *Gp, const double *Hp)
{
    orc_element *e = C->e;
    const int N = C->N[i], s0 = C->s0[i], k0 = C->k0[i];
    double *G = C->G, *H = C->H;
    int success = 1;
    for (int j = 0; j < NX; ++j) G[(s0 + N) * NX + j] = C->Phix[i * NX + j] + Gp[j];
    for (int j = 0; j < NN; ++j) H[(size_t)(s0 + N) * NN + j] = C->Phixx[(size_t)i * NN + j] + Hp[j];
    double dV1 = 0, dV2 = 0;
    double Qx[NX], Qu[NX], Qxx[NN], Quu[NN], Qux[NN], HA[NN], HB[NN], Qinv[NN], Qinv2[NN], Gn[NX], T[NN];
    for (int k = N - 1; k >= 0; --k) {
        int s = s0 + k, kc = k0 + k;
        const double *Ak = C->A + (size_t)kc * NN, *Bk = C->B + (size_t)kc * NN;
        const double *Hn = H + (size_t)(s + 1) * NN;
        double Hd[NX];
        mat_vec(Hn, e->Defect + (s + 1) * NX, Hd);
        for (int j = 0; j < NX; ++j) Gn[j] = G[(s + 1) * NX + j] + Hd[j];
        double t[NX];
        matT_vec(Ak, Gn, t);
        for (int j = 0; j < NX; ++j) Qx[j] = C->lx[kc * NX + j] + t[j];
        matT_vec(Bk, Gn, t);
        for (int j = 0; j < NX; ++j) Qu[j] = C->lu[kc * NX + j] + t[j];
        mat_mul(Hn, Ak, HA);
        mat_mul(Hn, Bk, HB);
        matT_mul(Ak, HA, T);
        for (int j = 0; j < NN; ++j) Qxx[j] = C->lxx[(size_t)kc * NN + j] + T[j];
        matT_mul(Bk, HB, T);
        for (int j = 0; j < NN; ++j) Quu[j] = C->luu[(size_t)kc * NN + j] + T[j];
        matT_mul(Bk, HA, T);
        for (int j = 0; j < NN; ++j) Qux[j] = C->lux[(size_t)kc * NN + j] + T[j];
        for (int j = 0; j < NX; ++j) { Qxx[j * NX + j] += reg; Quu[j * NX + j] += reg; }
        double Qs[NN];
        memcpy(Qs, Quu, sizeof(Qs));
        for (int j = 0; j < NX; ++j) Qs[j * NX + j] -= 1e-9;
        if (!eigen_ldlt_is_positive(Qs)) { success = 0; break; }
        lu_inverse(Quu, Qinv);
        memcpy(Qinv2, Qinv, sizeof(Qinv2));
        for (int a = 0; a < NX; ++a)
            for (int b = 0; b < NX; ++b) T[a * NX + b] = (Qinv[a * NX + b] + Qinv2[b * NX + a]) / 2;
        memcpy(Qinv, T, sizeof(T));
        for (int a = 0; a < NX; ++a)
            for (int b = 0; b < NX; ++b) T[a * NX + b] = (Qxx[a * NX + b] + Qxx[b * NX + a]) / 2;
        memcpy(Qxx, T, sizeof(T));
        double *dU = e->dU + kc * NX, *Kk = e->K + (size_t)kc * NN;
        mat_vec(Qinv, Qu, t);
        for (int j = 0; j < NX; ++j) dU[j] = -t[j];
        mat_mul(Qinv, Qux, T);
        for (int j = 0; j < NN; ++j) Kk[j] = -T[j];
        /* G = Qx - Qux^T Quu_inv Qu;  H = Qxx - Qux^T Quu_inv Qux */
        double w[NX];
        matT_vec(Qux, t, w);
        for (int j = 0; j < NX; ++j) G[s * NX + j] = Qx[j] - w[j];
        double W[NN];
        matT_mul(Qux, T, W);
        for (int j = 0; j < NN; ++j) H[(size_t)s * NN + j] = Qxx[j] - W[j];
        double dVk = 0;
        for (int j = 0; j < NX; ++j) dVk += Qu[j] * dU[j];
        dVk = -dVk;
        dV1 -= dVk;
        dV2 += dVk;
    }
    double Hd[NX];
    mat_vec(H + (size_t)s0 * NN, e->Defect + s0 * NX, Hd);
    for (int j = 0; j < NX; ++j) G[s0 * NX + j] += Hd[j];
    C->dV1p[i] = dV1;
    C->dV2p[i] = dV2;
    return success;
}

/* SinglePhase::backward_sweep (SinglePhase.cpp:298-367) alone, on caller-supplied time-invariant LQ
 * data over one phase of N knots: A, B, lxx, luu (24 x 24, row-major), lx, lu, terminal Phix, Phixx,
 * regularisation reg, zero defects.  The known-answer entry for the outside Riccati pin (SURVEY.md
 * §4.3 item 1): as N grows, K[0] and H[0] converge to the discrete algebraic Riccati solution.
 * Outputs K0, H0 (24 x 24), dU0, G0 (24); returns the sweep's success flag (PSD test). */
int orc_riccati_lq(int N, const double *A, const double *B, const double *lxx, const double *luu, const double *lx,
                   const double *lu, const double *Phix, const double *Phixx, double reg, double *K0, double *dU0,
                   double *G0, double *H0)
{
    if (N < 1 || N > 100000) return 0;
    const int S = N + 1;
    ctx_t C;
    memset(&C, 0, sizeof C);
    orc_element e;
    memset(&e, 0, sizeof e);
    C.e = &e;
    C.P = 1; C.S = S; C.Kc = N;
    C.N[0] = N; C.s0[0] = 0; C.k0[0] = 0;
    double *buf = calloc((size_t)N * (2 * NN + 3 * NN + 2 * NX) + (size_t)S * (NN + NX + NX) + NX + NN + (size_t)N * (NN + NX), sizeof(double));
    if (!buf) return 0;
    double *q = buf;
    C.A = q; q += (size_t)N * NN; C.B = q; q += (size_t)N * NN;
    C.lxx = q; q += (size_t)N * NN; C.luu = q; q += (size_t)N * NN; C.lux = q; q += (size_t)N * NN;
    C.lx = q; q += (size_t)N * NX; C.lu = q; q += (size_t)N * NX;
    C.H = q; q += (size_t)S * NN; C.G = q; q += (size_t)S * NX; e.Defect = q; q += (size_t)S * NX;
    C.Phix = q; q += NX; C.Phixx = q; q += NN;
    e.K = q; q += (size_t)N * NN; e.dU = q;
    for (int k = 0; k < N; ++k) {
        memcpy(C.A + (size_t)k * NN, A, sizeof(double) * NN); memcpy(C.B + (size_t)k * NN, B, sizeof(double) * NN);
        memcpy(C.lxx + (size_t)k * NN, lxx, sizeof(double) * NN); memcpy(C.luu + (size_t)k * NN, luu, sizeof(double) * NN);
        memcpy(C.lx + (size_t)k * NX, lx, sizeof(double) * NX); memcpy(C.lu + (size_t)k * NX, lu, sizeof(double) * NX);
    }
    memcpy(C.Phix, Phix, sizeof(double) * NX);
    memcpy(C.Phixx, Phixx, sizeof(double) * NN);
    double Gp[NX] = {0}, Hp[NN] = {0};
    const int ok = phase_backward(&C, 0, reg, Gp, Hp);
    memcpy(K0, e.K, sizeof(double) * NN); memcpy(dU0, e.dU, sizeof(double) * NX);
    memcpy(G0, C.G, sizeof(double) * NX); memcpy(H0, C.H, sizeof(double) * NN);
    free(buf);
    return ok;
}

/* SinglePhase::linear_rollout (SinglePhase.cpp:144-178) */
static void phase_linear_rollout(ctx_t *C, int i, double eps, const double *dx_init)
{
    orc_element *e = C->e;
    const int N = C->N[i], s0 = C->s0[i], k0 = C->k0[i];
    double dV1 = 0, dV2 = 0;
    for (int j = 0; j < NX; ++j) e->dX[s0 * NX + j] = dx_init[j] + eps * e->Defect[s0 * NX + j];
    for (int k = 0; k < N; ++k) {
        int s = s0 + k, kc = k0 + k;
        const double *dx = e->dX + s * NX;
        double du[NX], t[NX], t2[NX];
        mat_vec(e->K + (size_t)kc * NN, dx, t);
        for (int j = 0; j < NX; ++j) du[j] = eps * e->dU[kc * NX + j] + t[j];
        mat_vec(C->A + (size_t)kc * NN, dx, t);
        mat_vec(C->B + (size_t)kc * NN, du, t2);
        for (int j = 0; j < NX; ++j) e->dX[(s + 1) * NX + j] = t[j] + t2[j] + eps * e->Defect[(s + 1) * NX + j];
        double a = 0, b = 0;
        for (int j = 0; j < NX; ++j) a += C->lx[kc * NX + j] * dx[j];
        for (int j = 0; j < NX; ++j) b += C->lu[kc * NX + j] * du[j];
        dV1 += a + b;
        mat_vec(C->lxx + (size_t)kc * NN, dx, t);
        a = 0;
        for (int j = 0; j < NX; ++j) a += dx[j] * t[j];
        dV2 += a;
        mat_vec(C->luu + (size_t)kc * NN, du, t);
        a = 0;
        for (int j = 0; j < NX; ++j) a += du[j] * t[j];
        dV2 += a;
        mat_vec(C->lux + (size_t)kc * NN, dx, t);
        a = 0;
        for (int j = 0; j < NX; ++j) a += du[j] * t[j];
        dV2 += a;
    }
    const double *dxN = e->dX + (s0 + N) * NX;
    double a = 0, t[NX];
    for (int j = 0; j < NX; ++j) a += C->Phix[i * NX + j] * dxN[j];
    dV1 += a;
    mat_vec(C->Phixx + (size_t)i * NN, dxN, t);
    a = 0;
    for (int j = 0; j < NX; ++j) a += dxN[j] * t[j];
    dV2 += a;
    C->dV1p[i] = dV1;
    C->dV2p[i] = dV2;
}

/* ---- multi-phase routines (MultiPhaseDDP.cpp) -------------------------------------------- */
static int mp_hybrid_rollout(ctx_t *C, double eps)
{
    C->actual_cost = 0; C->max_pconstr = 0; C->max_tconstr = 0;
    double xinit[NX];
    memcpy(xinit, C->e->x0, sizeof(xinit));
    int success = 1;
    for (int i = 0; i < C->P; ++i) {
        if (i > 0) {
            const double *xend = C->e->X + (size_t)(C->s0[i - 1] + C->N[i - 1]) * NX;
            orc_resetmap(xend, C->c[i - 1], C->c[i], xinit);
        }
        if (!phase_hybrid_rollout(C, i, eps, xinit)) { success = 0; break; }
        C->max_pconstr = fmin(C->max_pconstr, C->pviol[i]);
        C->max_tconstr = fmax(C->max_tconstr, C->tviol[i]);
    }
    return success;
}

static void mp_compute_cost(ctx_t *C)
{
    C->actual_cost = 0;
    for (int i = 0; i < C->P; ++i) { phase_compute_cost(C, i); C->actual_cost += C->phase_cost[i]; }
}

static double mp_feas(ctx_t *C)
{
    double f = 0;
    for (int i = 0; i < C->P; ++i) {
        double fi = 0;
        for (int k = 0; k <= C->N[i]; ++k)
            for (int j = 0; j < NX; ++j) { double d = C->e->Defect[(C->s0[i] + k) * NX + j]; fi += d * d; }
        f += fi;
    }
    return sqrt(f);
}

static int mp_backward(ctx_t *C, double reg)
{
    C->dV_1 = 0; C->dV_2 = 0;
    double Gp[NX], Hp[NN], Px[NN], T[NN], t[NX];
    for (int i = C->P - 1; i >= 0; --i) {
        memset(Gp, 0, sizeof(Gp)); memset(Hp, 0, sizeof(Hp));
        if (i <= C->P - 2) {
            const double *xend = C->e->X + (size_t)(C->s0[i] + C->N[i]) * NX;
            orc_resetmap_partial(xend, C->c[i], C->c[i + 1], Px);
            const int sn = C->s0[i + 1];
            memcpy(Gp, C->G + sn * NX, sizeof(Gp));
            memcpy(Hp, C->H + (size_t)sn * NN, sizeof(Hp));
            matT_vec(Px, Gp, t); memcpy(Gp, t, sizeof(t));
            matT_mul(Px, Hp, T); mat_mul(T, Px, Hp);
        }
        if (!phase_backward(C, i, reg, Gp, Hp)) return 0;
        C->dV_1 += C->dV1p[i];
        C->dV_2 += C->dV2p[i];
    }
    return 1;
}

static int mp_backward_regularized(ctx_t *C, double *reg)
{
    int success = 0;
    while (!success) {
        success = mp_backward(C, *reg);
        if (success) break;
        *reg = fmax(*reg * C->o->update_regularization, 1e-03);
        if (*reg > 1e2) break;
    }
    *reg = *reg / 20;
    if (*reg < 1e-06) *reg = 0;
    return success;
}

static void mp_linear_rollout(ctx_t *C, double eps)
{
    double dx_init[NX], Px[NN];
    memset(dx_init, 0, sizeof(dx_init));
    C->dV_1 = 0; C->dV_2 = 0;
    for (int i = 0; i < C->P; ++i) {
        if (i > 0) {
            const double *dxe = C->e->dX + (size_t)(C->s0[i - 1] + C->N[i - 1]) * NX;
            const double *xend = C->e->X + (size_t)(C->s0[i - 1] + C->N[i - 1]) * NX;
            orc_resetmap_partial(xend, C->c[i - 1], C->c[i], Px);
            mat_vec(Px, dxe, dx_init);
        }
        phase_linear_rollout(C, i, eps, dx_init);
        C->dV_1 += C->dV1p[i];
        C->dV_2 += C->dV2p[i];
    }
}

static void mp_update_nominal(ctx_t *C)
{
    orc_element *e = C->e;
    memcpy(e->Xbar, e->X, sizeof(double) * C->S * NX);
    memcpy(e->Ubar, e->U, sizeof(double) * C->Kc * NX);
    memcpy(e->Defect_bar, e->Defect, sizeof(double) * C->S * NX);
}

static int mp_line_search(ctx_t *C)
{
    const orc_options *o = C->o;
    double eps = 1, merit_prev = C->merit, feas_prev = C->feas;
    while (eps > 1e-3) {
        int ok = mp_hybrid_rollout(C, eps);
        C->n_ls++;
        C->e->n_diverged += !ok;
        mp_compute_cost(C);
        C->feas = mp_feas(C);
        C->merit = C->actual_cost + C->merit_rho * C->feas;
        double exp_cost_change = eps * C->dV_1 + 0.5 * eps * eps * C->dV_2;
        double exp_merit_change = exp_cost_change - eps * C->merit_rho * feas_prev;
        if ((C->merit <= merit_prev + o->gamma * exp_merit_change) && ok) return 1;
        eps *= o->alpha;
    }
    return 0;
}

static void mp_update_AL(ctx_t *C)
{
    orc_element *e = C->e;
    const orc_options *o = C->o;
    /* update_al_params of every touchdown constraint (ConstraintsBase.h:354-372) */
    for (int i = 0; i < C->P; ++i)
        for (int j = 0; j < ORC_MAX_TD; ++j) {
            const int m = e->td_mask[i * ORC_MAX_TD + j];
            for (int l = 0; l < 4; ++l) {
                if (!((m >> l) & 1)) continue;
                const int q = (i * ORC_MAX_TD + j) * 4 + l;
                double hh = C->td_h[q];
                if (fabs(hh) < o->tconstr_thresh) continue;
                double *sg = &e->al_sigma[q];
                if (fabs(hh) > 0.005) { *sg *= o->update_penalty; *sg = fmin(*sg, C->p->td_sigma_max); }
                else e->al_lambda[q] += hh * *sg;
            }
        }
}

static void mp_update_ReB(ctx_t *C)
{
    orc_element *e = C->e;
    const orc_options *o = C->o;
    for (int i = 0; i < C->P; ++i) {
        if (!n_stance(C->c[i])) continue;
        for (int k = 0; k < C->N[i]; ++k)
            for (int l = 0; l < 4; ++l) {
                if (!C->c[i][l]) continue;
                for (int r = 0; r < 5; ++r) {
                    int q = (C->k0[i] + k) * 20 + 5 * l + r;
                    if (C->g[q] > -o->pconstr_thresh) continue;
                    e->reb_eps[q] *= o->update_ReB;
                    e->reb_delta[q] *= o->update_relax;
                    e->reb_delta[q] = fmax(e->reb_delta[q], C->p->grf_delta_min);
                }
            }
    }
}

void orc_init_element(const orc_problem *p, orc_element *e)
{
    int P = p->n_phases, Kc = 0;
    for (int i = 0; i < P; ++i) Kc += p->horizons[i];
    /* create_data: zero constraint values (ConstraintsBase.h:26-34, 50-54, 133-139, 318-320) */
    if (e->grf_g) memset(e->grf_g, 0, sizeof(double) * (size_t)Kc * 20);
    if (e->td_h) memset(e->td_h, 0, sizeof(double) * (size_t)P * ORC_MAX_TD * 4);
    for (int q = 0; q < Kc * 20; ++q) { e->reb_delta[q] = p->grf_delta; e->reb_eps[q] = p->grf_eps; }
    for (int q = 0; q < P * ORC_MAX_TD * 4; ++q) { e->al_sigma[q] = p->td_sigma; e->al_lambda[q] = p->td_lambda; }
    for (int i = 0; i < P; ++i)
        for (int j = 0; j < ORC_MAX_TD; ++j) {
            int m = 0;
            if (j == 0)  /* add_tconstr_one_phase at initialization: legs with c = 0 -> cn = 1 */
                for (int l = 0; l < 4; ++l)
                    if (e->contacts[i * 4 + l] == 0 && e->contacts[(i + 1) * 4 + l] == 1) m |= 1 << l;
            e->td_mask[i * ORC_MAX_TD + j] = m;
        }
}

/* One knot and one phase end, evaluated alone (test infrastructure for the known-answer and
 * finite-difference tests): a one-phase, one-knot problem whose running slot holds (x, u) with
 * references (xr, ur, pf) and whose terminal slot holds x_end (references xr_end, pf_end), phase
 * contact c and next contact cn.  The constraint values come from GRFConstraint::compute_violation
 * (HKDConstraints.cpp:7-66) and TouchDownConstraint::compute_violation (:69-118), then
 * SinglePhase::compute_cost (SinglePhase.cpp:235-262) and LQ_approximation (:264-296) run as in the
 * solve.  out: l, Phi (2) | lx, lu (48) | lxx, luu, lux (3 x 576) | Phix (24) | Phixx (576) |
 * A, B (2 x 576). */
void orc_knot_eval(const orc_problem *p, const orc_options *o, const int *c, const int *cn, const double *x,
                   const double *u, const double *xr, const double *ur, const double *pf, const double *x_end,
                   const double *xr_end, const double *pf_end, const double *reb_delta, const double *reb_eps,
                   const double *sigma, const double *lambda, double *out)
{
    orc_problem p1 = *p;
    const int hz[1] = {1};
    p1.n_phases = 1;
    p1.horizons = hz;
    p1.shooting = NULL;
    double X[2 * NX], Xbar[2 * NX], U[NX], Ubar[NX], D[2 * NX], Db[2 * NX], dX[2 * NX], dU[NX], K[NN];
    double RX[2 * NX], RU[2 * NX], RF[24], rd[20], re[20], as[ORC_MAX_TD * 4], al[ORC_MAX_TD * 4];
    int cc[8], tdm[ORC_MAX_TD] = {0, 0, 0, 0};
    memcpy(X, x, sizeof(double) * NX); memcpy(X + NX, x_end, sizeof(double) * NX);
    memcpy(U, u, sizeof(double) * NX);
    memcpy(RX, xr, sizeof(double) * NX); memcpy(RX + NX, xr_end, sizeof(double) * NX);
    memcpy(RU, ur, sizeof(double) * NX); memset(RU + NX, 0, sizeof(double) * NX);
    memcpy(RF, pf, sizeof(double) * 12); memcpy(RF + 12, pf_end, sizeof(double) * 12);
    memcpy(rd, reb_delta, sizeof rd); memcpy(re, reb_eps, sizeof re);
    memset(as, 0, sizeof as); memset(al, 0, sizeof al);
    memcpy(as, sigma, 4 * sizeof(double)); memcpy(al, lambda, 4 * sizeof(double));
    for (int l = 0; l < 4; ++l) { cc[l] = c[l]; cc[4 + l] = cn[l]; tdm[0] |= (c[l] == 0 && cn[l] == 1) << l; }
    orc_element e;
    memset(&e, 0, sizeof e);
    e.contacts = cc; e.x0 = x; e.ref_x = RX; e.ref_u = RU; e.ref_foot = RF;
    e.X = X; e.Xbar = Xbar; e.U = U; e.Ubar = Ubar; e.Defect = D; e.Defect_bar = Db; e.dX = dX; e.dU = dU; e.K = K;
    e.reb_delta = rd; e.reb_eps = re; e.al_sigma = as; e.al_lambda = al; e.td_mask = tdm;
    ctx_t *C = (ctx_t *)calloc(1, sizeof(ctx_t));
    double *pool = (double *)calloc(8 * NN + 4 * NX + 64 + ORC_MAX_TD * 4, sizeof(double));
    C->p = &p1; C->o = o; C->e = &e; C->P = 1; C->S = 2; C->Kc = 1;
    C->N[0] = 1; C->s0[0] = 0; C->k0[0] = 0;
    for (int l = 0; l < 4; ++l) { C->c[0][l] = c[l]; C->c[1][l] = cn[l]; }
    setup_costs(C);
    double *q = pool;
    C->A = q; q += NN; C->B = q; q += NN; C->lxx = q; q += NN; C->luu = q; q += NN; C->lux = q; q += NN;
    C->l = q; q += 1; C->lx = q; q += NX; C->lu = q; q += NX;
    C->Phi = q; q += 1; C->Phix = q; q += NX; C->Phixx = q; q += NN; C->g = q; q += 20;
    C->td_h = q; q += ORC_MAX_TD * 4;
    for (int l = 0; l < 4; ++l)
        if (c[l]) grf_rows(p1.mu_fric, u + 3 * l, C->g + 5 * l);
    for (int l = 0; l < 4; ++l) {
        if (!(c[l] == 0 && cn[l] == 1)) continue;
        double pfz[3];
        orc_foot_position(l, x_end + 3, x_end, x_end + 12 + 3 * l, pfz);
        C->td_h[l] = pfz[2] - p1.ground_height;  /* constraint slot 0 */
    }
    phase_compute_cost(C, 0);
    phase_LQ(C, 0);
    out[0] = C->l[0]; out[1] = C->Phi[0];
    memcpy(out + 2, C->lx, sizeof(double) * NX); memcpy(out + 2 + NX, C->lu, sizeof(double) * NX);
    memcpy(out + 2 + 2 * NX, C->lxx, sizeof(double) * NN); memcpy(out + 2 + 2 * NX + NN, C->luu, sizeof(double) * NN);
    memcpy(out + 2 + 2 * NX + 2 * NN, C->lux, sizeof(double) * NN);
    memcpy(out + 2 + 2 * NX + 3 * NN, C->Phix, sizeof(double) * NX);
    memcpy(out + 2 + 3 * NX + 3 * NN, C->Phixx, sizeof(double) * NN);
    memcpy(out + 2 + 3 * NX + 4 * NN, C->A, sizeof(double) * NN);
    memcpy(out + 2 + 3 * NX + 5 * NN, C->B, sizeof(double) * NN);
    free(pool);
    free(C);
}

/* cost_buffer / dyn_feas_buffer / eqn_feas_buffer / ineq_feas_buffer .push_back (float vectors) */
static void push_info(ctx_t *C)
{
    orc_element *e = C->e;
    if (e->hist && e->hist_n < e->hist_cap) {
        float *h = e->hist + 4 * (size_t)e->hist_n;
        h[0] = (float)C->actual_cost; h[1] = (float)C->feas;
        h[2] = (float)C->max_tconstr; h[3] = (float)C->max_pconstr;
    }
    e->hist_n++;
}

/* MultiPhaseDDP::solve (MultiPhaseDDP.cpp:232-428) */
int orc_solve(const orc_problem *p, const orc_options *o, orc_element *e)
{
    ctx_t *C = (ctx_t *)calloc(1, sizeof(ctx_t));
    if (!C) return -1;
    C->p = p; C->o = o; C->e = e;
    C->P = p->n_phases;
    if (C->P > MAXP || C->P < 1) { free(C); return -2; }
    int s = 0, k = 0;
    for (int i = 0; i < C->P; ++i) {
        C->N[i] = p->horizons[i]; C->s0[i] = s; C->k0[i] = k;
        s += C->N[i] + 1; k += C->N[i];
        for (int l = 0; l < 4; ++l) C->c[i][l] = e->contacts[i * 4 + l];
    }
    for (int l = 0; l < 4; ++l) C->c[C->P][l] = e->contacts[C->P * 4 + l];
    C->S = s; C->Kc = k;
    setup_costs(C);
    size_t Kc = (size_t)C->Kc, S = (size_t)C->S;
    double *pool = (double *)calloc(Kc * NN * 5 + Kc * (1 + 2 * NX) + (size_t)C->P * (1 + NX + NN) +
                                        S * (NX + NN) + S * NX + Kc * 20 + (size_t)C->P * ORC_MAX_TD * 4,
                                    sizeof(double));
    if (!pool) { free(C); return -1; }
    double *q = pool;
    C->A = q; q += Kc * NN; C->B = q; q += Kc * NN;
    C->lxx = q; q += Kc * NN; C->luu = q; q += Kc * NN; C->lux = q; q += Kc * NN;
    C->l = q; q += Kc; C->lx = q; q += Kc * NX; C->lu = q; q += Kc * NX;
    C->Phi = q; q += C->P; C->Phix = q; q += (size_t)C->P * NX; C->Phixx = q; q += (size_t)C->P * NN;
    C->G = q; q += S * NX; C->H = q; q += S * NN; C->Xsim = q; q += S * NX; C->g = q; q += Kc * 20;
    C->td_h = q; q += (size_t)C->P * ORC_MAX_TD * 4;
    /* the constraint objects' data persists across solves (orc_element.grf_g / td_h) */
    if (e->grf_g) C->g = e->grf_g;
    if (e->td_h) C->td_h = e->td_h;

    int iter = 0, iter_ou = 0, iter_in = 0, success = 1;
    double cost_prev = 0, merit_prev = 0;
    e->status = 0;

    e->n_diverged = 0;
    e->diverged_init = !mp_hybrid_rollout(C, 0);
    mp_update_nominal(C);
    mp_compute_cost(C);
    C->feas = mp_feas(C);
    e->hist_n = 0;
    push_info(C);  /* the initial information (MultiPhaseDDP.cpp:277-280) */

    while (iter_ou < o->max_AL_iter) {
        iter_ou++;
        C->max_tconstr_prev = C->max_tconstr;
        C->max_pconstr_prev = C->max_pconstr;
        double reg = 0;
        iter_in = 0;
        while (iter_in < o->max_DDP_iter) {
            mp_compute_cost(C);
            C->feas = mp_feas(C);
            iter_in++;
            iter++;
            for (int i = 0; i < C->P; ++i) phase_LQ(C, i);
            success = mp_backward_regularized(C, &reg);
            if (!success) goto bad_solve;
            if (o->MS) mp_linear_rollout(C, 1.0);
            double dV_abs = fabs(C->dV_1 + 0.5 * C->dV_2);
            C->merit_rho = (C->feas > o->dynamics_feas_thresh)
                               ? dV_abs / ((1 - o->merit_scale) * C->feas) + o->merit_offset : 0;
            C->merit = C->actual_cost + C->merit_rho * C->feas;
            cost_prev = C->actual_cost;
            merit_prev = C->merit;
            if (!o->no_early_exit && (dV_abs < o->cost_thresh) && (C->feas <= o->dynamics_feas_thresh)) break;
            if (mp_line_search(C)) mp_update_nominal(C);
            else { C->actual_cost = cost_prev; C->merit = merit_prev; }
            if (!o->no_early_exit && (fabs((cost_prev - C->actual_cost) / cost_prev) < o->cost_thresh) &&
                (C->feas <= o->dynamics_feas_thresh))
                break;
            push_info(C);  /* MultiPhaseDDP.cpp:368-371 */
        }
        if (o->AL_active) mp_update_AL(C);
        if (o->ReB_active) mp_update_ReB(C);
        if (o->no_early_exit) continue;
        if (C->max_tconstr < o->tconstr_thresh && fabs(C->max_pconstr) < o->pconstr_thresh &&
            C->feas <= o->dynamics_feas_thresh)
            break;
        if (fabs(C->max_tconstr - C->max_tconstr_prev) < 0.0001 &&
            fabs(C->max_pconstr - C->max_pconstr_prev) < 0.0001 && C->feas <= o->dynamics_feas_thresh)
            break;
    }
bad_solve:
    if (!success) e->status = 1;
    e->cost = C->actual_cost; e->feas = C->feas; e->merit = C->merit;
    e->max_tconstr = C->max_tconstr; e->max_pconstr = C->max_pconstr;
    e->iters = iter; e->outer_iters = iter_ou; e->n_ls_trials = C->n_ls;
    free(pool);
    free(C);
    return 0;
}

/* ---- batch driver (CPU baseline) ---------------------------------------------------------- */
typedef struct { const orc_problem *p; const orc_options *o; orc_element *e; int n, next; pthread_mutex_t mu; } pool_t;

static void *worker(void *arg)
{
    pool_t *P = (pool_t *)arg;
    for (;;) {
        pthread_mutex_lock(&P->mu);
        int i = P->next++;
        pthread_mutex_unlock(&P->mu);
        if (i >= P->n) break;
        orc_solve(P->p, P->o, &P->e[i]);
    }
    return 0;
}

int orc_solve_batch(const orc_problem *p, const orc_options *o, orc_element *elems, int n, int n_threads)
{
    if (n_threads < 1) n_threads = 1;
    pool_t P = {p, o, elems, n, 0, PTHREAD_MUTEX_INITIALIZER};
    pthread_t th[256];
    if (n_threads > 256) n_threads = 256;
    for (int t = 0; t < n_threads; ++t) pthread_create(&th[t], 0, worker, &P);
    for (int t = 0; t < n_threads; ++t) pthread_join(th[t], 0);
    return 0;
}
