/*
 * ref_shim.c — TEST INFRASTRUCTURE ONLY (oracle side; never linked into the product).
 *
 * Dense-output C entry points over the reference's own CasADi-generated HKD kernels,
 * compiled in place from /root/reference by oracle/Makefile into oracle/_ref/.
 * Used only to pin oracle/hkd_model_ref.c (the CPU restatement) and to emit the golden
 * fixtures under tests/golden/.  The scatter from CasADi's column-compressed output into a
 * dense column-major buffer mirrors what the reference does at
 * common/casadi_interface.cpp:46-68 (row index + nrow*col).
 *
 * Reference kernels wrapped (signatures from CasadiGen/header/*.h):
 *   hkinodyn(x[24], u[24], dt, c[4]) -> x+[24]          hkinodyn_casadi.cpp:177-658
 *   hkinodyn_par(x, u, dt, c)        -> A[24x24], B[24x24]  hkinodyn_par_casadi.cpp:181-2800
 *   compute_foot_position(pos, eul, qleg, id) -> p[3]     comp_foot_pos_casadi.cpp:46-160
 *   comp_foot_jacob_{1..4}(pos, eul, qleg) -> J[3x18]      comp_foot_jacob_1_casadi.cpp:46-520
 */
#include <string.h>

typedef long long int casadi_int;
typedef int (*cas_fn)(const double **, double **, casadi_int *, double *, int);
typedef const casadi_int *(*cas_sp)(casadi_int);

#define DECL(name)                                                                     \
    int name(const double **arg, double **res, casadi_int *iw, double *w, int mem);    \
    const casadi_int *name##_sparsity_out(casadi_int i);

DECL(hkinodyn)
DECL(hkinodyn_par)
DECL(compute_foot_position)
DECL(comp_foot_jacob_1)
DECL(comp_foot_jacob_2)
DECL(comp_foot_jacob_3)
DECL(comp_foot_jacob_4)

/* Scatter CCS output `nz` (pattern sp) into dense column-major `dense` (zero-filled first). */
static void scatter(const casadi_int *sp, const double *nz, double *dense)
{
    casadi_int nrow = sp[0], ncol = sp[1];
    const casadi_int *colptr = sp + 2;
    const casadi_int *row = colptr + ncol + 1;
    memset(dense, 0, sizeof(double) * (size_t)(nrow * ncol));
    for (casadi_int c = 0; c < ncol; ++c)
        for (casadi_int p = colptr[c]; p < colptr[c + 1]; ++p)
            dense[row[p] + nrow * c] = nz[p];
}

static void call_dense(cas_fn f, cas_sp sp, int nout, const double **arg, double **out)
{
    double buf[2][1024];
    double *res[2] = {buf[0], buf[1]};
    f(arg, res, 0, 0, 0);
    for (int i = 0; i < nout; ++i)
        scatter(sp(i), buf[i], out[i]);
}

/* x_next[24] = hkinodyn(x, u, dt, c) */
void ref_hkinodyn(const double *x, const double *u, double dt, const double *c, double *x_next)
{
    const double *arg[4] = {x, u, &dt, c};
    double *out[1] = {x_next};
    call_dense(hkinodyn, hkinodyn_sparsity_out, 1, arg, out);
}

/* A[24*24], B[24*24] column-major = hkinodyn_par(x, u, dt, c) */
void ref_hkinodyn_par(const double *x, const double *u, double dt, const double *c, double *A, double *B)
{
    const double *arg[4] = {x, u, &dt, c};
    double *out[2] = {A, B};
    call_dense(hkinodyn_par, hkinodyn_par_sparsity_out, 2, arg, out);
}

/* p[3] = compute_foot_position(pos, eul, qleg, foot_id)   foot_id in 1..4 (FR, FL, HR, HL) */
void ref_foot_position(const double *pos, const double *eul, const double *qleg, double foot_id, double *p)
{
    const double *arg[4] = {pos, eul, qleg, &foot_id};
    double *out[1] = {p};
    call_dense(compute_foot_position, compute_foot_position_sparsity_out, 1, arg, out);
}

/* J[3*18] column-major = comp_foot_jacob_{leg+1}(pos, eul, qleg)   leg in 0..3 */
void ref_foot_jacobian(int leg, const double *pos, const double *eul, const double *qleg, double *J)
{
    static const cas_fn fns[4] = {comp_foot_jacob_1, comp_foot_jacob_2, comp_foot_jacob_3, comp_foot_jacob_4};
    static const cas_sp sps[4] = {comp_foot_jacob_1_sparsity_out, comp_foot_jacob_2_sparsity_out,
                                  comp_foot_jacob_3_sparsity_out, comp_foot_jacob_4_sparsity_out};
    const double *arg[3] = {pos, eul, qleg};
    double *out[1] = {J};
    call_dense(fns[leg], sps[leg], 1, arg, out);
}
