/*
 * hkd_model_ref.c — TEST INFRASTRUCTURE ONLY (see hkd_oracle.h).
 *
 * Hand restatement of the reference's CasADi-generated HKD model kernels:
 *   hkinodyn       HKDMPC/HKD-TrajOpt/CasadiGen/source/hkinodyn_casadi.cpp:177-658
 *   hkinodyn_par   .../hkinodyn_par_casadi.cpp:181-2800 (discrete Jacobians A = dx+/dx, B = dx+/du)
 *   compute_foot_position  .../comp_foot_pos_casadi.cpp:46-160
 *   comp_foot_jacob_{1..4} .../comp_foot_jacob_1_casadi.cpp:46-520
 * and the HKD reset map, HKDMPC/HKD-TrajOpt/HKDReset.h:41-136.
 * Pinned against the compiled reference kernels in tests/test_oracle_model.py.
 */
#include <math.h>
#include <string.h>
#include "hkd_oracle.h"

/* Model constants read off the generated expression graph (hkinodyn_casadi.cpp:257-578). */
static const double MASS = 8.9120000000000008e+00;     /* :559 */
static const double GRAV = -9.8100000000000005e+00;    /* :575 */
static const double INERTIA[3][3] = {                  /* :257-270, :409-411 */
    {2.7460779999999994e-02, 1.0842021724855044e-19, -1.2037062152420224e-35},
    {1.0842021724855044e-19, 2.4251579680000002e-01, 0.0},
    {-1.2037062152420224e-35, 0.0, 2.6519357680000000e-01}};
static const double INERTIA_INV[3][3] = {              /* :256, :405, :491, :534-546 */
    {3.6415571589736352e+01, -1.6280111378663628e-17, 1.6528925920107902e-33},
    {-1.6280111378663628e-17, 4.1234427331951844e+00, -7.3894969432494111e-52},
    {1.6528925920107902e-33, -7.3894969432494111e-52, 3.7708303951651367e+00}};

/* Mini Cheetah leg geometry (comp_foot_pos_casadi.cpp:53-102). */
static const double HIP_X = 0.19, SIDE_Y = 0.049, ABAD = 0.062, L_UP = -0.209, L_LOW = -0.195;
/* side = (-1)^id, front = (-1)^floor(id/3), id = leg+1 */
static const double LEG_SIDE[4] = {-1.0, 1.0, -1.0, 1.0};
static const double LEG_FRONT[4] = {1.0, 1.0, -1.0, -1.0};

/* R = Rz(yaw) Ry(pitch) Rx(roll) and its partials w.r.t. (yaw, pitch, roll). */
static void rot_zyx(const double *eul, double R[3][3], double dR[3][3][3])
{
    double cy = cos(eul[0]), sy = sin(eul[0]);
    double cp = cos(eul[1]), sp = sin(eul[1]);
    double cr = cos(eul[2]), sr = sin(eul[2]);
    R[0][0] = cy * cp; R[0][1] = cy * sp * sr - sy * cr; R[0][2] = sy * sr + cy * sp * cr;
    R[1][0] = sy * cp; R[1][1] = cy * cr + sy * sp * sr; R[1][2] = sy * sp * cr - cy * sr;
    R[2][0] = -sp;     R[2][1] = cp * sr;                R[2][2] = cp * cr;
    if (!dR) return;
    /* d/dyaw */
    dR[0][0][0] = -sy * cp; dR[0][0][1] = -sy * sp * sr - cy * cr; dR[0][0][2] = cy * sr - sy * sp * cr;
    dR[0][1][0] = cy * cp;  dR[0][1][1] = -sy * cr + cy * sp * sr; dR[0][1][2] = cy * sp * cr + sy * sr;
    dR[0][2][0] = 0;        dR[0][2][1] = 0;                       dR[0][2][2] = 0;
    /* d/dpitch */
    dR[1][0][0] = -cy * sp; dR[1][0][1] = cy * cp * sr; dR[1][0][2] = cy * cp * cr;
    dR[1][1][0] = -sy * sp; dR[1][1][1] = sy * cp * sr; dR[1][1][2] = sy * cp * cr;
    dR[1][2][0] = -cp;      dR[1][2][1] = -sp * sr;     dR[1][2][2] = -sp * cr;
    /* d/droll */
    dR[2][0][0] = 0; dR[2][0][1] = cy * sp * cr + sy * sr; dR[2][0][2] = sy * cr - cy * sp * sr;
    dR[2][1][0] = 0; dR[2][1][1] = -cy * sr + sy * sp * cr; dR[2][1][2] = -sy * sp * sr - cy * cr;
    dR[2][2][0] = 0; dR[2][2][1] = cp * cr;                 dR[2][2][2] = -cp * sr;
}

static void cross3(const double *a, const double *b, double *o)
{
    o[0] = a[1] * b[2] - a[2] * b[1];
    o[1] = a[2] * b[0] - a[0] * b[2];
    o[2] = a[0] * b[1] - a[1] * b[0];
}

/* skew(a) so that skew(a) b = a x b */
static void skew3(const double *a, double S[3][3])
{
    S[0][0] = 0;     S[0][1] = -a[2]; S[0][2] = a[1];
    S[1][0] = a[2];  S[1][1] = 0;     S[1][2] = -a[0];
    S[2][0] = -a[1]; S[2][1] = a[0];  S[2][2] = 0;
}

/* Lever arm used by the generated model: foot at (qx, qy, 0) in world, so r = (qx-px, qy-py, -pz)
 * (hkinodyn_casadi.cpp:272-289: the lever's z uses -x[5], never qdummy z). */
static void lever(const double *x, int l, double *r)
{
    r[0] = x[12 + 3 * l] - x[3];
    r[1] = x[12 + 3 * l + 1] - x[4];
    r[2] = -x[5];
}

/* World-frame contact torque sum w = sum_l c_l r_l x f_l;  body torque = R^T w. */
static void world_torque(const double *x, const double *u, const double *c, double *w)
{
    w[0] = w[1] = w[2] = 0;
    for (int l = 0; l < 4; ++l) {
        double r[3], t[3];
        lever(x, l, r);
        cross3(r, u + 3 * l, t);
        for (int i = 0; i < 3; ++i) w[i] += c[l] * t[i];
    }
}

void orc_hkd_step(const double *x, const double *u, double dt, const double *c, double *xn)
{
    const double *eul = x, *pos = x + 3, *om = x + 6, *v = x + 9;
    double cp = cos(eul[1]), sp = sin(eul[1]), cr = cos(eul[2]), sr = sin(eul[2]);
    /* ZYX Euler-rate map (hkinodyn_casadi.cpp:178-219) */
    double yaw_rate = (sr * om[1] + cr * om[2]) / cp;
    xn[0] = eul[0] + dt * yaw_rate;
    xn[1] = eul[1] + dt * (cr * om[1] - sr * om[2]);
    xn[2] = eul[2] + dt * (om[0] + sp * yaw_rate);
    for (int i = 0; i < 3; ++i) xn[3 + i] = pos[i] + dt * v[i];  /* :220-234 */
    /* angular momentum balance in body frame (:235-551) */
    double R[3][3], w[3], tau[3], Iw[3], gyro[3], rhs[3];
    rot_zyx(eul, R, 0);
    world_torque(x, u, c, w);
    for (int i = 0; i < 3; ++i) tau[i] = R[0][i] * w[0] + R[1][i] * w[1] + R[2][i] * w[2];
    for (int i = 0; i < 3; ++i) Iw[i] = INERTIA[i][0] * om[0] + INERTIA[i][1] * om[1] + INERTIA[i][2] * om[2];
    cross3(om, Iw, gyro);
    for (int i = 0; i < 3; ++i) rhs[i] = tau[i] - gyro[i];
    for (int i = 0; i < 3; ++i)
        xn[6 + i] = om[i] + dt * (INERTIA_INV[i][0] * rhs[0] + INERTIA_INV[i][1] * rhs[1] + INERTIA_INV[i][2] * rhs[2]);
    /* linear momentum (:553-587) */
    for (int i = 0; i < 3; ++i) {
        double f = c[0] * u[i] + c[1] * u[3 + i] + c[2] * u[6 + i] + c[3] * u[9 + i];
        double acc = f / MASS + (i == 2 ? GRAV : 0.0);
        xn[9 + i] = v[i] + dt * acc;
    }
    /* qdummy: swing legs integrate commanded joint velocity (:588-656) */
    for (int l = 0; l < 4; ++l)
        for (int j = 0; j < 3; ++j)
            xn[12 + 3 * l + j] = x[12 + 3 * l + j] + (1.0 - c[l]) * u[12 + 3 * l + j] * dt;
}

void orc_hkd_partial(const double *x, const double *u, double dt, const double *c, double *A, double *B)
{
    const double *eul = x, *om = x + 6;
    memset(A, 0, sizeof(double) * 576);
    memset(B, 0, sizeof(double) * 576);
    for (int i = 0; i < 24; ++i) A[i * 24 + i] = 1.0;
    double cp = cos(eul[1]), sp = sin(eul[1]), cr = cos(eul[2]), sr = sin(eul[2]);
    double a = sr * om[1] + cr * om[2]; /* cos(pitch) * yaw rate */
    double b = cr * om[1] - sr * om[2];
    /* Euler-rate rows */
    A[0 * 24 + 1] += dt * a * sp / (cp * cp);
    A[0 * 24 + 2] += dt * b / cp;
    A[0 * 24 + 7] += dt * sr / cp;
    A[0 * 24 + 8] += dt * cr / cp;
    A[1 * 24 + 2] += dt * (-a);
    A[1 * 24 + 7] += dt * cr;
    A[1 * 24 + 8] += dt * (-sr);
    A[2 * 24 + 1] += dt * a / (cp * cp);
    A[2 * 24 + 2] += dt * sp / cp * b;
    A[2 * 24 + 6] += dt;
    A[2 * 24 + 7] += dt * sr * sp / cp;
    A[2 * 24 + 8] += dt * cr * sp / cp;
    /* position rows */
    for (int i = 0; i < 3; ++i) A[(3 + i) * 24 + 9 + i] = dt;
    /* angular velocity rows: d omega+ = dt * Iinv * d(tau - omega x I omega) */
    double R[3][3], dR[3][3][3], w[3];
    rot_zyx(eul, R, dR);
    world_torque(x, u, c, w);
    double M[3][24]; /* d(rhs)/dx, rows omega, cols state */
    memset(M, 0, sizeof(M));
    for (int j = 0; j < 3; ++j)          /* d(R^T w)/d eul_j = dR_j^T w */
        for (int i = 0; i < 3; ++i)
            M[i][j] = dR[j][0][i] * w[0] + dR[j][1][i] * w[1] + dR[j][2][i] * w[2];
    for (int l = 0; l < 4; ++l) {
        double Sf[3][3];
        skew3(u + 3 * l, Sf);
        /* d w / d pos = sum c_l skew(f_l);  d w / d q_l(x,y) = -c_l skew(f_l)[:, 0:2] */
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k) {
                double Rt_Sf = R[0][i] * Sf[0][k] + R[1][i] * Sf[1][k] + R[2][i] * Sf[2][k];
                M[i][3 + k] += c[l] * Rt_Sf;
                if (k < 2) M[i][12 + 3 * l + k] += -c[l] * Rt_Sf;
            }
    }
    /* gyroscopic: d(-omega x I omega)/d omega = skew(I omega) - skew(omega) I */
    double Iw[3], SIw[3][3], So[3][3];
    for (int i = 0; i < 3; ++i) Iw[i] = INERTIA[i][0] * om[0] + INERTIA[i][1] * om[1] + INERTIA[i][2] * om[2];
    skew3(Iw, SIw);
    skew3(om, So);
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) {
            double SoI = So[i][0] * INERTIA[0][k] + So[i][1] * INERTIA[1][k] + So[i][2] * INERTIA[2][k];
            M[i][6 + k] += SIw[i][k] - SoI;
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 24; ++j) {
            double s = INERTIA_INV[i][0] * M[0][j] + INERTIA_INV[i][1] * M[1][j] + INERTIA_INV[i][2] * M[2][j];
            A[(6 + i) * 24 + j] += dt * s;
        }
    /* B: omega rows <- Iinv R^T c_l skew(r_l);  v rows <- c_l / m;  q rows <- (1 - c_l) */
    for (int l = 0; l < 4; ++l) {
        double r[3], Sr[3][3], T[3][3];
        lever(x, l, r);
        skew3(r, Sr);
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k)
                T[i][k] = c[l] * (R[0][i] * Sr[0][k] + R[1][i] * Sr[1][k] + R[2][i] * Sr[2][k]);
        for (int i = 0; i < 3; ++i)
            for (int k = 0; k < 3; ++k)
                B[(6 + i) * 24 + 3 * l + k] =
                    dt * (INERTIA_INV[i][0] * T[0][k] + INERTIA_INV[i][1] * T[1][k] + INERTIA_INV[i][2] * T[2][k]);
        for (int k = 0; k < 3; ++k) {
            B[(9 + k) * 24 + 3 * l + k] = dt * c[l] / MASS;
            B[(12 + 3 * l + k) * 24 + 12 + 3 * l + k] = dt * (1.0 - c[l]);
        }
    }
}

/* body-frame foot position relative to the trunk origin */
static void foot_body(int l, const double *q, double *pb, double dpb[3][3])
{
    double s = LEG_SIDE[l], f = LEG_FRONT[l];
    double c0 = cos(q[0]), s0 = sin(q[0]);
    double c1 = cos(q[1]), s1 = sin(q[1]);
    double c12 = cos(q[1] + q[2]), s12 = sin(q[1] + q[2]);
    pb[0] = HIP_X * f - L_LOW * s12 - L_UP * s1;
    pb[1] = SIDE_Y * s + ABAD * s * c0 - L_LOW * s0 * c12 - L_UP * s0 * c1;
    pb[2] = L_LOW * c0 * c12 + L_UP * c0 * c1 + ABAD * s * s0;
    if (!dpb) return;
    dpb[0][0] = 0;
    dpb[0][1] = -L_LOW * c12 - L_UP * c1;
    dpb[0][2] = -L_LOW * c12;
    dpb[1][0] = -ABAD * s * s0 - L_LOW * c0 * c12 - L_UP * c0 * c1;
    dpb[1][1] = L_LOW * s0 * s12 + L_UP * s0 * s1;
    dpb[1][2] = L_LOW * s0 * s12;
    dpb[2][0] = -L_LOW * s0 * c12 - L_UP * s0 * c1 + ABAD * s * c0;
    dpb[2][1] = -L_LOW * c0 * s12 - L_UP * c0 * s1;
    dpb[2][2] = -L_LOW * c0 * s12;
}

void orc_foot_position(int leg, const double *pos, const double *eul, const double *qleg, double *p)
{
    double R[3][3], pb[3];
    rot_zyx(eul, R, 0);
    foot_body(leg, qleg, pb, 0);
    for (int i = 0; i < 3; ++i) p[i] = pos[i] + R[i][0] * pb[0] + R[i][1] * pb[1] + R[i][2] * pb[2];
}

void orc_foot_jacobian(int leg, const double *pos, const double *eul, const double *qleg, double *J)
{
    (void)pos;
    double R[3][3], dR[3][3][3], pb[3], dpb[3][3];
    rot_zyx(eul, R, dR);
    foot_body(leg, qleg, pb, dpb);
    memset(J, 0, sizeof(double) * 54);
    for (int i = 0; i < 3; ++i) {
        J[i * 18 + i] = 1.0;
        for (int j = 0; j < 3; ++j)
            J[i * 18 + 3 + j] = dR[j][i][0] * pb[0] + dR[j][i][1] * pb[1] + dR[j][i][2] * pb[2];
        for (int k = 0; k < 3; ++k)
            J[i * 18 + 6 + 3 * leg + k] = R[i][0] * dpb[0][k] + R[i][1] * dpb[1][k] + R[i][2] * dpb[2][k];
    }
}

/* HKDReset::resetmap (HKDReset.h:41-75) */
void orc_resetmap(const double *x, const int *c, const int *cn, double *xn)
{
    static const double qleg_default[3] = {0.0, -0.8, 1.7}; /* HKDReset.h:37 */
    memcpy(xn, x, sizeof(double) * 24);
    for (int l = 0; l < 4; ++l) {
        if (c[l] && !cn[l])
            for (int j = 0; j < 3; ++j) xn[12 + 3 * l + j] = qleg_default[j];
        if (!c[l] && cn[l]) {
            double pf[3];
            orc_foot_position(l, x + 3, x, x + 12 + 3 * l, pf);
            xn[12 + 3 * l + 0] = pf[0];
            xn[12 + 3 * l + 1] = pf[1];
            xn[12 + 3 * l + 2] = 0.0 * pf[2];
        }
    }
}

/* HKDReset::resetmap_partial (HKDReset.h:78-136) */
void orc_resetmap_partial(const double *x, const int *c, const int *cn, double *Px)
{
    memset(Px, 0, sizeof(double) * 576);
    for (int i = 0; i < 24; ++i) Px[i * 24 + i] = 1.0;
    for (int l = 0; l < 4; ++l) {
        if (c[l] && !cn[l])
            for (int r = 0; r < 3; ++r)
                for (int j = 0; j < 24; ++j) Px[(12 + 3 * l + r) * 24 + j] = 0.0;
        if (!c[l] && cn[l]) {
            double J[54];
            orc_foot_jacobian(l, x + 3, x, x + 12 + 3 * l, J);
            for (int r = 0; r < 3; ++r) {
                double cm = (r < 2) ? 1.0 : 0.0;
                double *row = Px + (12 + 3 * l + r) * 24;
                for (int j = 0; j < 3; ++j) row[j] = cm * J[r * 18 + 3 + j];      /* eul <- J[:,3:6] */
                for (int j = 0; j < 3; ++j) row[3 + j] = cm * J[r * 18 + j];      /* pos <- J[:,0:3] */
                for (int j = 0; j < 12; ++j) row[12 + j] = cm * J[r * 18 + 6 + j]; /* q <- J[:,6:18] */
            }
        }
    }
}
