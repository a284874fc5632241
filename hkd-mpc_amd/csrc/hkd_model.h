// hkd_model.h — HKD quadruped model, __host__ __device__, fp64.
//
// Native replacement of the reference's CasADi-generated kernels (called through
// common/casadi_interface.cpp:5-80, which heap-allocates and scatters on every call):
//   hkd_step          <- hkinodyn      HKDMPC/HKD-TrajOpt/CasadiGen/source/hkinodyn_casadi.cpp:177-658
//   hkd_partial_*     <- hkinodyn_par  .../hkinodyn_par_casadi.cpp:181-2800
//   hkd_foot_position <- compute_foot_position  .../comp_foot_pos_casadi.cpp:46-160
//   hkd_foot_jacobian <- comp_foot_jacob_{1..4}  .../comp_foot_jacob_1_casadi.cpp:46-520
//   hkd_resetmap(_partial) <- HKDReset::resetmap(_partial)  HKDMPC/HKD-TrajOpt/HKDReset.h:41-136
//
// The discrete Jacobians are emitted in compact form (A = I + S):
//   Se[3][5]  : rows eul(0..2) x cols {pitch, roll, wx, wy, wz} = {1, 2, 6, 7, 8}
//   Sw[3][17] : rows omega(6..8) x cols {0..8, 12,13, 15,16, 18,19, 21,22}
//   Bw[3][12] : rows omega(6..8) x GRF cols 0..11
// constants (not stored): S[3+i][9+i] = dt; B[9+j][3l+j] = dt c_l / m; B[12+m][12+m] = dt (1 - c_leg(m)).
// Every other entry of S and B is structurally zero (checked against the reference's CasADi
// sparsity, hkinodyn_par_casadi.cpp:177-178, in tests/test_model_gpu.py).
#pragma once

#ifndef __HIPCC__
#ifndef __host__
#define __host__
#define __device__
#endif
#endif
#include <math.h>

#define HKD_FN __host__ __device__ inline

namespace hkd {

constexpr int NX = 24;
constexpr int NU = 24;
constexpr int SE_N = 15;
constexpr int SW_N = 51;
constexpr int BW_N = 36;

// Model constants (read off the generated expression graph, hkinodyn_casadi.cpp:256-578).
constexpr double kMass = 8.9120000000000008e+00;
constexpr double kGravity = -9.8100000000000005e+00;
constexpr double kI00 = 2.7460779999999994e-02, kI01 = 1.0842021724855044e-19, kI02 = -1.2037062152420224e-35;
constexpr double kI11 = 2.4251579680000002e-01, kI22 = 2.6519357680000000e-01;
constexpr double kJ00 = 3.6415571589736352e+01, kJ01 = -1.6280111378663628e-17, kJ02 = 1.6528925920107902e-33;
constexpr double kJ11 = 4.1234427331951844e+00, kJ12 = -7.3894969432494111e-52, kJ22 = 3.7708303951651367e+00;

// Mini Cheetah leg (comp_foot_pos_casadi.cpp:53-102)
constexpr double kHipX = 0.19, kSideY = 0.049, kAbad = 0.062, kUpper = -0.209, kLower = -0.195;

__host__ __device__ constexpr int se_col(int q) { return q < 2 ? 1 + q : 4 + q; }          // {1,2,6,7,8}
__host__ __device__ constexpr int sw_col(int q) { return q < 9 ? q : 12 + 3 * ((q - 9) >> 1) + ((q - 9) & 1); }
// inverse maps (-1 when the column carries no entry of that block)
__host__ __device__ constexpr int se_index(int c) { return c == 1 ? 0 : c == 2 ? 1 : (c >= 6 && c <= 8) ? c - 4 : -1; }
__host__ __device__ constexpr int sw_index(int c)
{
    return c < 9 ? c : (c >= 12 && ((c - 12) % 3) < 2) ? 9 + 2 * ((c - 12) / 3) + ((c - 12) % 3) : -1;
}

HKD_FN double leg_side(int l) { return (l & 1) ? 1.0 : -1.0; }   // (-1)^(l+1)
HKD_FN double leg_front(int l) { return l < 2 ? 1.0 : -1.0; }    // (-1)^floor((l+1)/3)

struct Rot {
    double r[3][3];
};

// sin / cos of the three Euler angles, each pair from one sincos (one argument reduction): the
// model's rotation, its derivatives and the Euler-rate terms share them
struct EulTrig {
    double cy, sy, cp, sp, cr, sr;
};
HKD_FN EulTrig eul_trig(const double *eul)
{
    EulTrig t;
    sincos(eul[0], &t.sy, &t.cy);
    sincos(eul[1], &t.sp, &t.cp);
    sincos(eul[2], &t.sr, &t.cr);
    return t;
}

HKD_FN void rot_zyx(const EulTrig &t, Rot &R)
{
    const double cy = t.cy, sy = t.sy, cp = t.cp, sp = t.sp, cr = t.cr, sr = t.sr;
    R.r[0][0] = cy * cp; R.r[0][1] = cy * sp * sr - sy * cr; R.r[0][2] = sy * sr + cy * sp * cr;
    R.r[1][0] = sy * cp; R.r[1][1] = cy * cr + sy * sp * sr; R.r[1][2] = sy * sp * cr - cy * sr;
    R.r[2][0] = -sp;     R.r[2][1] = cp * sr;                R.r[2][2] = cp * cr;
}

// dR/d(yaw), dR/d(pitch), dR/d(roll)
HKD_FN void rot_zyx_grad(const EulTrig &t, Rot &Dy, Rot &Dp, Rot &Dr)
{
    const double cy = t.cy, sy = t.sy, cp = t.cp, sp = t.sp, cr = t.cr, sr = t.sr;
    Dy.r[0][0] = -sy * cp; Dy.r[0][1] = -sy * sp * sr - cy * cr; Dy.r[0][2] = cy * sr - sy * sp * cr;
    Dy.r[1][0] = cy * cp;  Dy.r[1][1] = cy * sp * sr - sy * cr;  Dy.r[1][2] = sy * sr + cy * sp * cr;
    Dy.r[2][0] = 0.0;      Dy.r[2][1] = 0.0;                     Dy.r[2][2] = 0.0;
    Dp.r[0][0] = -cy * sp; Dp.r[0][1] = cy * cp * sr; Dp.r[0][2] = cy * cp * cr;
    Dp.r[1][0] = -sy * sp; Dp.r[1][1] = sy * cp * sr; Dp.r[1][2] = sy * cp * cr;
    Dp.r[2][0] = -cp;      Dp.r[2][1] = -sp * sr;     Dp.r[2][2] = -sp * cr;
    Dr.r[0][0] = 0.0; Dr.r[0][1] = cy * sp * cr + sy * sr; Dr.r[0][2] = sy * cr - cy * sp * sr;
    Dr.r[1][0] = 0.0; Dr.r[1][1] = sy * sp * cr - cy * sr; Dr.r[1][2] = -cy * cr - sy * sp * sr;
    Dr.r[2][0] = 0.0; Dr.r[2][1] = cp * cr;                Dr.r[2][2] = -cp * sr;
}

HKD_FN void rot_zyx(const double *eul, Rot &R) { rot_zyx(eul_trig(eul), R); }
HKD_FN void rot_zyx_grad(const double *eul, Rot &Dy, Rot &Dp, Rot &Dr) { rot_zyx_grad(eul_trig(eul), Dy, Dp, Dr); }

// sum_l c_l (r_l x f_l), lever r_l = (q_lx - px, q_ly - py, -pz): the generated model places
// the stance foot on the ground plane (hkinodyn_casadi.cpp:272-289 never reads qdummy z).
HKD_FN void contact_moment(const double *x, const double *u, const double *c, double *w)
{
    w[0] = w[1] = w[2] = 0.0;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        double rx = x[12 + 3 * l] - x[3], ry = x[13 + 3 * l] - x[4], rz = -x[5];
        const double *f = u + 3 * l;
        w[0] += c[l] * (ry * f[2] - rz * f[1]);
        w[1] += c[l] * (rz * f[0] - rx * f[2]);
        w[2] += c[l] * (rx * f[1] - ry * f[0]);
    }
}

HKD_FN void inertia_apply(const double *v, double *o)
{
    o[0] = kI00 * v[0] + kI01 * v[1] + kI02 * v[2];
    o[1] = kI01 * v[0] + kI11 * v[1];
    o[2] = kI02 * v[0] + kI22 * v[2];
}
HKD_FN void inertia_inv_apply(const double *v, double *o)
{
    o[0] = kJ00 * v[0] + kJ01 * v[1] + kJ02 * v[2];
    o[1] = kJ01 * v[0] + kJ11 * v[1] + kJ12 * v[2];
    o[2] = kJ02 * v[0] + kJ12 * v[1] + kJ22 * v[2];
}

// x+ = x + dt f(x, u; c), explicit Euler (hkinodyn)
HKD_FN void hkd_step(const double *x, const double *u, const double *c, double dt, double *xn)
{
    const double *om = x + 6;
    const EulTrig tr = eul_trig(x);
    const double cp = tr.cp, sp = tr.sp, cr = tr.cr, sr = tr.sr;
    double ydot = (sr * om[1] + cr * om[2]) / cp;
    xn[0] = x[0] + dt * ydot;
    xn[1] = x[1] + dt * (cr * om[1] - sr * om[2]);
    xn[2] = x[2] + dt * (om[0] + sp * ydot);
#pragma unroll
    for (int i = 0; i < 3; ++i) xn[3 + i] = x[3 + i] + dt * x[9 + i];
    Rot R;
    rot_zyx(tr, R);
    double w[3], tau[3], Iw[3], rhs[3], acc[3];
    contact_moment(x, u, c, w);
#pragma unroll
    for (int i = 0; i < 3; ++i) tau[i] = R.r[0][i] * w[0] + R.r[1][i] * w[1] + R.r[2][i] * w[2];
    inertia_apply(om, Iw);
    rhs[0] = tau[0] - (om[1] * Iw[2] - om[2] * Iw[1]);
    rhs[1] = tau[1] - (om[2] * Iw[0] - om[0] * Iw[2]);
    rhs[2] = tau[2] - (om[0] * Iw[1] - om[1] * Iw[0]);
    inertia_inv_apply(rhs, acc);
#pragma unroll
    for (int i = 0; i < 3; ++i) xn[6 + i] = om[i] + dt * acc[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        double f = c[0] * u[i] + c[1] * u[3 + i] + c[2] * u[6 + i] + c[3] * u[9 + i];
        xn[9 + i] = x[9 + i] + dt * (f / kMass + (i == 2 ? kGravity : 0.0));
    }
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
        for (int j = 0; j < 3; ++j) xn[12 + 3 * l + j] = x[12 + 3 * l + j] + (1.0 - c[l]) * u[12 + 3 * l + j] * dt;
}

// Compact discrete Jacobians (see header comment).
HKD_FN void hkd_partial_compact(const double *x, const double *u, const double *c, double dt, double *Se,
                                double *Sw, double *Bw)
{
    const double *om = x + 6;
    const EulTrig tr = eul_trig(x);
    const double cp = tr.cp, sp = tr.sp, cr = tr.cr, sr = tr.sr;
    double a = sr * om[1] + cr * om[2], b = cr * om[1] - sr * om[2];
    const double icp = 1.0 / cp, tp = sp * icp;  // one reciprocal for the Euler-rate rows
    // eul rows, cols {1, 2, 6, 7, 8}
    Se[0] = dt * a * sp * (icp * icp); Se[1] = dt * b * icp; Se[2] = 0.0; Se[3] = dt * sr * icp; Se[4] = dt * cr * icp;
    Se[5] = 0.0;                     Se[6] = -dt * a;     Se[7] = 0.0;     Se[8] = dt * cr;      Se[9] = -dt * sr;
    Se[10] = dt * a * icp * icp;     Se[11] = dt * tp * b; Se[12] = dt;    Se[13] = dt * sr * tp; Se[14] = dt * cr * tp;
    // omega rows: dt * Iinv * d(tau - omega x I omega)/dx
    Rot R, Dy, Dp, Dr;
    rot_zyx(tr, R);
    rot_zyx_grad(tr, Dy, Dp, Dr);
    double w[3];
    contact_moment(x, u, c, w);
    double M[3][17];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        M[i][0] = Dy.r[0][i] * w[0] + Dy.r[1][i] * w[1] + Dy.r[2][i] * w[2];
        M[i][1] = Dp.r[0][i] * w[0] + Dp.r[1][i] * w[1] + Dp.r[2][i] * w[2];
        M[i][2] = Dr.r[0][i] * w[0] + Dr.r[1][i] * w[1] + Dr.r[2][i] * w[2];
#pragma unroll
        for (int q = 3; q < 17; ++q) M[i][q] = 0.0;
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const double *f = u + 3 * l;
        // R^T skew(f): (R^T [f]x)[i][k] = sum_m R[m][i] [f]x[m][k]
        double Sf[3][3] = {{0.0, -f[2], f[1]}, {f[2], 0.0, -f[0]}, {-f[1], f[0], 0.0}};
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                double t = c[l] * (R.r[0][i] * Sf[0][k] + R.r[1][i] * Sf[1][k] + R.r[2][i] * Sf[2][k]);
                M[i][3 + k] += t;                       // d/d pos
                if (k < 2) M[i][9 + 2 * l + k] = -t;    // d/d q_l(x, y)
            }
    }
    // gyroscopic: skew(I w) - skew(w) I
    double Iw[3];
    inertia_apply(om, Iw);
    const double Ssk[3][3] = {{0.0, -Iw[2], Iw[1]}, {Iw[2], 0.0, -Iw[0]}, {-Iw[1], Iw[0], 0.0}};
    const double So[3][3] = {{0.0, -om[2], om[1]}, {om[2], 0.0, -om[0]}, {-om[1], om[0], 0.0}};
    const double In[3][3] = {{kI00, kI01, kI02}, {kI01, kI11, 0.0}, {kI02, 0.0, kI22}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int k = 0; k < 3; ++k)
            M[i][6 + k] = Ssk[i][k] - (So[i][0] * In[0][k] + So[i][1] * In[1][k] + So[i][2] * In[2][k]);
#pragma unroll
    for (int q = 0; q < 17; ++q) {
        double v[3] = {M[0][q], M[1][q], M[2][q]}, o[3];
        inertia_inv_apply(v, o);
        Sw[q] = dt * o[0]; Sw[17 + q] = dt * o[1]; Sw[34 + q] = dt * o[2];
    }
    // B omega rows: dt Iinv R^T c_l skew(r_l)
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        double r0 = x[12 + 3 * l] - x[3], r1 = x[13 + 3 * l] - x[4], r2 = -x[5];
        double Sr[3][3] = {{0.0, -r2, r1}, {r2, 0.0, -r0}, {-r1, r0, 0.0}};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            double v[3], o[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) v[i] = c[l] * (R.r[0][i] * Sr[0][k] + R.r[1][i] * Sr[1][k] + R.r[2][i] * Sr[2][k]);
            inertia_inv_apply(v, o);
            Bw[3 * l + k] = dt * o[0]; Bw[12 + 3 * l + k] = dt * o[1]; Bw[24 + 3 * l + k] = dt * o[2];
        }
    }
}

// hkd_partial_compact's values, each handed to emit(piece, index, value) as soon as it is computed
// (piece 0: Se[index], 1: Sw[index], 2: Bw[index]) — the same expression per value, but a column
// of the omega rows at a time, columns in increasing order (the record's column-major positions,
// sw_at / bw_at), so a caller that stores each value right away never holds the 102 outputs (or
// the 3 x 17 moment Jacobian) at once.
template <typename Emit>
HKD_FN void hkd_partial_emit(const double *x, const double *u, const double *c, double dt, Emit emit)
{
    const double *om = x + 6;
    const EulTrig tr = eul_trig(x);
    const double cp = tr.cp, sp = tr.sp, cr = tr.cr, sr = tr.sr;
    double a = sr * om[1] + cr * om[2], b = cr * om[1] - sr * om[2];
    const double icp = 1.0 / cp, tp = sp * icp;  // one reciprocal for the Euler-rate rows
    emit(0, 0, dt * a * sp * (icp * icp)); emit(0, 1, dt * b * icp); emit(0, 2, 0.0); emit(0, 3, dt * sr * icp);
    emit(0, 4, dt * cr * icp); emit(0, 5, 0.0); emit(0, 6, -dt * a); emit(0, 7, 0.0); emit(0, 8, dt * cr);
    emit(0, 9, -dt * sr); emit(0, 10, dt * a * icp * icp); emit(0, 11, dt * tp * b); emit(0, 12, dt);
    emit(0, 13, dt * sr * tp); emit(0, 14, dt * cr * tp);
    Rot R, Dy, Dp, Dr;
    rot_zyx(tr, R);
    rot_zyx_grad(tr, Dy, Dp, Dr);
    // omega rows: column q of M = d(tau - omega x I omega)/dx, then dt Iinv M[:, q]
    auto col = [&](const double (&v)[3], int q) {
        double o[3];
        inertia_inv_apply(v, o);
        emit(1, q, dt * o[0]); emit(1, 17 + q, dt * o[1]); emit(1, 34 + q, dt * o[2]);
    };
    {   // columns 0..2: the contact moment rotated by the Euler-angle derivatives of R
        double w[3];
        contact_moment(x, u, c, w);
        double v[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) v[i] = Dy.r[0][i] * w[0] + Dy.r[1][i] * w[1] + Dy.r[2][i] * w[2];
        col(v, 0);
#pragma unroll
        for (int i = 0; i < 3; ++i) v[i] = Dp.r[0][i] * w[0] + Dp.r[1][i] * w[1] + Dp.r[2][i] * w[2];
        col(v, 1);
#pragma unroll
        for (int i = 0; i < 3; ++i) v[i] = Dr.r[0][i] * w[0] + Dr.r[1][i] * w[1] + Dr.r[2][i] * w[2];
        col(v, 2);
    }
    // R^T skew(f_l) terms: columns 3 + k (summed over the legs in leg order) and 9 + 2 l + k (k < 2)
    auto tl = [&](int l, int i, int k) {
        const double *f = u + 3 * l;
        const double Sf[3][3] = {{0.0, -f[2], f[1]}, {f[2], 0.0, -f[0]}, {-f[1], f[0], 0.0}};
        return c[l] * (R.r[0][i] * Sf[0][k] + R.r[1][i] * Sf[1][k] + R.r[2][i] * Sf[2][k]);
    };
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        double v[3] = {0.0, 0.0, 0.0};
#pragma unroll
        for (int l = 0; l < 4; ++l)
#pragma unroll
            for (int i = 0; i < 3; ++i) v[i] += tl(l, i, k);
        col(v, 3 + k);
    }
    {   // columns 6..8, gyroscopic: skew(I w) - skew(w) I
        double Iw[3];
        inertia_apply(om, Iw);
        const double Ssk[3][3] = {{0.0, -Iw[2], Iw[1]}, {Iw[2], 0.0, -Iw[0]}, {-Iw[1], Iw[0], 0.0}};
        const double So[3][3] = {{0.0, -om[2], om[1]}, {om[2], 0.0, -om[0]}, {-om[1], om[0], 0.0}};
        const double In[3][3] = {{kI00, kI01, kI02}, {kI01, kI11, 0.0}, {kI02, 0.0, kI22}};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            double v[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) v[i] = Ssk[i][k] - (So[i][0] * In[0][k] + So[i][1] * In[1][k] + So[i][2] * In[2][k]);
            col(v, 6 + k);
        }
    }
#pragma unroll
    for (int l = 0; l < 4; ++l)
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            double v[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) v[i] = -tl(l, i, k);
            col(v, 9 + 2 * l + k);
        }
    // B omega rows: dt Iinv R^T c_l skew(r_l), GRF column 3 l + k
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        double r0 = x[12 + 3 * l] - x[3], r1 = x[13 + 3 * l] - x[4], r2 = -x[5];
        double Sr[3][3] = {{0.0, -r2, r1}, {r2, 0.0, -r0}, {-r1, r0, 0.0}};
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            double v[3], o[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) v[i] = c[l] * (R.r[0][i] * Sr[0][k] + R.r[1][i] * Sr[1][k] + R.r[2][i] * Sr[2][k]);
            inertia_inv_apply(v, o);
            emit(2, 3 * l + k, dt * o[0]); emit(2, 12 + 3 * l + k, dt * o[1]); emit(2, 24 + 3 * l + k, dt * o[2]);
        }
    }
}

// dense column-major expansion (Eigen layout of the reference's StateMap / ContrlMap)
HKD_FN void hkd_expand_colmajor(const double *Se, const double *Sw, const double *Bw, const double *c, double dt,
                                double *A, double *B)
{
    for (int i = 0; i < NX * NX; ++i) { A[i] = 0.0; B[i] = 0.0; }
    for (int i = 0; i < NX; ++i) A[i + NX * i] = 1.0;
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 5; ++q) A[r + NX * se_col(q)] += Se[5 * r + q];
    for (int i = 0; i < 3; ++i) A[(3 + i) + NX * (9 + i)] = dt;
    for (int r = 0; r < 3; ++r)
        for (int q = 0; q < 17; ++q) A[(6 + r) + NX * sw_col(q)] += Sw[17 * r + q];
    for (int r = 0; r < 3; ++r)
        for (int k = 0; k < 12; ++k) B[(6 + r) + NX * k] = Bw[12 * r + k];
    for (int l = 0; l < 4; ++l)
        for (int j = 0; j < 3; ++j) {
            B[(9 + j) + NX * (3 * l + j)] = dt * c[l] / kMass;
            B[(12 + 3 * l + j) + NX * (12 + 3 * l + j)] = dt * (1.0 - c[l]);
        }
}

// ---- kinematics ------------------------------------------------------------------------
// from the sines / cosines of q0, q1 and q1 + q2 (tr: s0, c0, s1, c1, s12, c12)
HKD_FN void foot_body_trig(int l, const double *tr, double *pb, double (*dpb)[3])
{
    double s = leg_side(l), f = leg_front(l);
    const double s0 = tr[0], c0 = tr[1], s1 = tr[2], c1 = tr[3], s12 = tr[4], c12 = tr[5];
    pb[0] = kHipX * f - kLower * s12 - kUpper * s1;
    pb[1] = kSideY * s + kAbad * s * c0 - kLower * s0 * c12 - kUpper * s0 * c1;
    pb[2] = kLower * c0 * c12 + kUpper * c0 * c1 + kAbad * s * s0;
    if (dpb) {
        dpb[0][0] = 0.0; dpb[0][1] = -kLower * c12 - kUpper * c1; dpb[0][2] = -kLower * c12;
        dpb[1][0] = -kAbad * s * s0 - kLower * c0 * c12 - kUpper * c0 * c1;
        dpb[1][1] = kLower * s0 * s12 + kUpper * s0 * s1; dpb[1][2] = kLower * s0 * s12;
        dpb[2][0] = -kLower * s0 * c12 - kUpper * s0 * c1 + kAbad * s * c0;
        dpb[2][1] = -kLower * c0 * s12 - kUpper * c0 * s1; dpb[2][2] = -kLower * c0 * s12;
    }
}

HKD_FN void foot_body(int l, const double *q, double *pb, double (*dpb)[3])
{
    double tr[6];
    sincos(q[0], &tr[0], &tr[1]);
    sincos(q[1], &tr[2], &tr[3]);
    sincos(q[1] + q[2], &tr[4], &tr[5]);
    foot_body_trig(l, tr, pb, dpb);
}

// foot position in world of leg l, joint angles taken from q (3)
HKD_FN void hkd_foot_position(int l, const double *pos, const double *eul, const double *q, double *p)
{
    Rot R;
    rot_zyx(eul, R);
    double pb[3];
    foot_body(l, q, pb, nullptr);
    for (int i = 0; i < 3; ++i) p[i] = pos[i] + R.r[i][0] * pb[0] + R.r[i][1] * pb[1] + R.r[i][2] * pb[2];
}

// J row-major [3][18], columns [pos | eul | qJ(12)] (only leg l's three joint columns non-zero)
HKD_FN void hkd_foot_jacobian(int l, const double *eul, const double *q, double *J)
{
    Rot R, Dy, Dp, Dr;
    const EulTrig tr = eul_trig(eul);
    rot_zyx(tr, R);
    rot_zyx_grad(tr, Dy, Dp, Dr);
    double pb[3], dpb[3][3];
    foot_body(l, q, pb, dpb);
    for (int i = 0; i < 54; ++i) J[i] = 0.0;
    for (int i = 0; i < 3; ++i) {
        J[18 * i + i] = 1.0;
        J[18 * i + 3] = Dy.r[i][0] * pb[0] + Dy.r[i][1] * pb[1] + Dy.r[i][2] * pb[2];
        J[18 * i + 4] = Dp.r[i][0] * pb[0] + Dp.r[i][1] * pb[1] + Dp.r[i][2] * pb[2];
        J[18 * i + 5] = Dr.r[i][0] * pb[0] + Dr.r[i][1] * pb[1] + Dr.r[i][2] * pb[2];
        for (int k = 0; k < 3; ++k)
            J[18 * i + 6 + 3 * l + k] = R.r[i][0] * dpb[0][k] + R.r[i][1] * dpb[1][k] + R.r[i][2] * dpb[2][k];
    }
}

// foot height h and dh/dx in state order (TouchDownConstraint, HKDConstraints.cpp:69-171)
HKD_FN double hkd_foot_height_grad(int l, const double *x, double *hx)
{
    Rot R, Dy, Dp, Dr;
    const EulTrig tr = eul_trig(x);
    rot_zyx(tr, R);
    rot_zyx_grad(tr, Dy, Dp, Dr);
    double pb[3], dpb[3][3];
    foot_body(l, x + 12 + 3 * l, pb, dpb);
    if (hx) {
        for (int j = 0; j < NX; ++j) hx[j] = 0.0;
        hx[0] = Dy.r[2][0] * pb[0] + Dy.r[2][1] * pb[1] + Dy.r[2][2] * pb[2];
        hx[1] = Dp.r[2][0] * pb[0] + Dp.r[2][1] * pb[1] + Dp.r[2][2] * pb[2];
        hx[2] = Dr.r[2][0] * pb[0] + Dr.r[2][1] * pb[1] + Dr.r[2][2] * pb[2];
        hx[5] = 1.0;
        for (int k = 0; k < 3; ++k)
            hx[12 + 3 * l + k] = R.r[2][0] * dpb[0][k] + R.r[2][1] * dpb[1][k] + R.r[2][2] * dpb[2][k];
    }
    return x[5] + R.r[2][0] * pb[0] + R.r[2][1] * pb[1] + R.r[2][2] * pb[2];
}

// hkd_foot_height_grad's non-zeros only (no runtime-indexed local array): ge = d h / d eul (state
// 0..2), gq = d h / d foot position of leg l (states 12 + 3 l + k); d h / d state 5 is 1
HKD_FN double hkd_foot_height_grad_sparse(int l, const double *x, double *ge, double *gq)
{
    Rot R, Dy, Dp, Dr;
    const EulTrig tr = eul_trig(x);
    rot_zyx(tr, R);
    rot_zyx_grad(tr, Dy, Dp, Dr);
    double pb[3], dpb[3][3];
    foot_body(l, x + 12 + 3 * l, pb, dpb);
    ge[0] = Dy.r[2][0] * pb[0] + Dy.r[2][1] * pb[1] + Dy.r[2][2] * pb[2];
    ge[1] = Dp.r[2][0] * pb[0] + Dp.r[2][1] * pb[1] + Dp.r[2][2] * pb[2];
    ge[2] = Dr.r[2][0] * pb[0] + Dr.r[2][1] * pb[1] + Dr.r[2][2] * pb[2];
    for (int k = 0; k < 3; ++k) gq[k] = R.r[2][0] * dpb[0][k] + R.r[2][1] * dpb[1][k] + R.r[2][2] * dpb[2][k];
    return x[5] + R.r[2][0] * pb[0] + R.r[2][1] * pb[1] + R.r[2][2] * pb[2];
}

// HKDReset::resetmap
HKD_FN void hkd_resetmap(const double *x, const int *c, const int *cn, double *xn)
{
    for (int j = 0; j < NX; ++j) xn[j] = x[j];
#pragma unroll  // compile-time leg index keeps xn in registers on the device
    for (int l = 0; l < 4; ++l) {
        if (c[l] && !cn[l]) { xn[12 + 3 * l] = 0.0; xn[13 + 3 * l] = -0.8; xn[14 + 3 * l] = 1.7; }
        if (!c[l] && cn[l]) {
            double p[3];
            hkd_foot_position(l, x + 3, x, x + 12 + 3 * l, p);
            xn[12 + 3 * l] = p[0]; xn[13 + 3 * l] = p[1]; xn[14 + 3 * l] = 0.0 * p[2];
        }
    }
}

// HKDReset::resetmap_partial, one row of Px (row-major row r), for use row-parallel on the device
HKD_FN void hkd_resetmap_partial_row(const double *x, const int *c, const int *cn, int r, double *row)
{
    for (int j = 0; j < NX; ++j) row[j] = (j == r) ? 1.0 : 0.0;
    if (r < 12) return;
    int l = (r - 12) / 3, k = (r - 12) % 3;
    if (c[l] && !cn[l]) { row[r] = 0.0; return; }
    if (!c[l] && cn[l]) {
        row[r] = 0.0;
        if (k == 2) return;
        double J[54];
        hkd_foot_jacobian(l, x, x + 12 + 3 * l, J);
        for (int j = 0; j < 3; ++j) { row[j] = J[18 * k + 3 + j]; row[3 + j] = J[18 * k + j]; }
        for (int j = 0; j < 12; ++j) row[12 + j] = J[18 * k + 6 + j];
    }
}

}  // namespace hkd
