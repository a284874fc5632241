// hsddp_device.h — device-side cost/constraint helpers shared by the solver kernels.
// HKD costs: HKDCost.h:8-99, HKDCost.cpp:5-63; SinglePhaseInterface.cpp:55-118.
// ReB / GRF: ConstraintsBase.h:204-263, HKDConstraints.cpp:7-66.  AL / touchdown: ConstraintsBase.h:374-399,
// HKDConstraints.cpp:69-171.
#pragma once
#include <type_traits>

#include "hsddp_internal.h"

namespace hsddp {
using namespace hkd;

#define DEV __device__ __forceinline__

// Register pin: the values must exist in VGPRs at this point.  Placed at the end of a stage, it
// stops LLVM from sinking the stage's arithmetic into a later one (which keeps the stage's
// operands live and spills).
template <typename T, int N>
DEV void pin(T (&a)[N])
{
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(a[i]));
}
// scheduling fence between stages: keeps the scheduler from hoisting a later stage's loads (and
// their registers) into an earlier one
#define SFENCE() __builtin_amdgcn_sched_barrier(0)

// ---------------------------------------------------------------------------------------------
// cost model helpers (HKDCost.h / HKDCost.cpp / SinglePhaseInterface.cpp:55-118)
// Params read in place from the kernel-argument segment (scalar loads).  Every kernel takes Params
// first, so it sits at offset 0; indexing the by-value copy with a runtime index makes the compiler
// copy the whole struct to scratch, per lane.
typedef const __attribute__((address_space(4))) Params KParams;
DEV KParams *kparams() { return (KParams *)__builtin_amdgcn_kernarg_segment_ptr(); }

// PT: Params (compile-time indices) or KParams (runtime indices)
template <typename PT>
DEV double q_diag(const PT &p, const int *c, int j) { return j < 12 ? p.qbase[j] : p.q_qJ * (1 - c[(j - 12) / 3]); }
DEV double r_diag(const Params &p, int j) { return j < 12 ? p.r_grf : p.r_qJd; }
template <typename PT>
DEV double foot_weight(const PT &p, const int *c, int j) { return p.foot_gain * p.foot_w[j % 3] * c[j / 3]; }
DEV bool touchdown(const int *c, const int *cn, int l) { return c[l] == 0 && cn[l] == 1; }

// ---- the phase layout of element b ----------------------------------------------------------
// The handle's layout (Params, read in place: runtime phase indices never index the by-value copy)
// or, with per-element layouts (Params::elem_layout, hsddp_set_element_layouts), element b's own
// (Bufs::lay).  The kernels are instantiated for both (EL), so the shared-layout path carries no
// per-access selection.
template <bool EL>
struct LayT {
    const Layout *l;
    DEV int P() const { if constexpr (EL) return l->P; else return kparams()->P; }
    DEV int S() const { if constexpr (EL) return l->S; else return kparams()->S; }
    DEV int N(int i) const { if constexpr (EL) return l->N[i]; else return kparams()->N[i]; }
    DEV int s0(int i) const { if constexpr (EL) return l->s0[i]; else return kparams()->s0[i]; }
    DEV int k0(int i) const { if constexpr (EL) return l->k0[i]; else return kparams()->k0[i]; }
    DEV int ss(int i) const { if constexpr (EL) return l->ss[i]; else return kparams()->ss[i]; }
};
template <bool EL>
DEV LayT<EL> layout_of(const Bufs &d, int b) { return LayT<EL>{EL ? d.lay + b : nullptr}; }

// phase i and knot k of state slot s
template <typename L_>
DEV void slot_phase(const L_ &L, int s, int &i, int &k)
{
    i = 0;
    const int P = L.P();
    for (int j = 1; j < P; ++j)
        if (s >= L.s0(j)) i = j;
    k = s - L.s0(i);
}

// phase i and knot k of control knot kc (kc = k0(i) + k)
template <typename L_>
DEV void knot_phase(const L_ &L, int kc, int &i, int &k)
{
    i = 0;
    const int P = L.P();
    for (int j = 1; j < P; ++j)
        if (kc >= L.k0(j)) i = j;
    k = kc - L.k0(i);
}

// element b's nominal (Xbar / Ubar), working (X / U / Defect) and trial-target buffers (Bufs::sel)
DEV int nom_buf(const Bufs &d, int b) { return d.sel[b] & 3; }
DEV int work_buf(const Bufs &d, int b) { return (d.sel[b] >> 2) & 3; }
DEV int trial_of(int nb, int wb) { return nb == wb ? (nb == 2 ? 0 : nb + 1) : 3 - nb - wb; }
DEV int trial_buf(const Bufs &d, int b) { const int q = d.sel[b]; return trial_of(q & 3, (q >> 2) & 3); }
DEV int sel_code(int nb, int wb) { return nb | (wb << 2); }
// Bufs read in place from the kernel-argument segment, for kernels whose first two arguments are
// (Params, Bufs): loads the compiler can repeat where a value is used, instead of keeping the
// pointers live in scalar registers across the kernel (it spilled them to VGPR lanes)
typedef const __attribute__((address_space(4))) Bufs KBufs;
DEV KBufs *kbufs()
{
    constexpr size_t off = (sizeof(Params) + alignof(Bufs) - 1) / alignof(Bufs) * alignof(Bufs);
    return (KBufs *)((const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr() + off);
}
DEV double *kxbuf(int q) { return kbufs()->X3 + (size_t)q * kbufs()->xs3; }
DEV double *kdbuf(int q) { return kbufs()->D3 + (size_t)q * kbufs()->xs3; }
DEV double *kubuf(int q) { return kbufs()->U3 + (size_t)q * kbufs()->us3; }

// buffer q of the three-buffer sets (one allocation each: base + q x stride)
DEV double *xbuf(const Bufs &d, int q) { return d.X3 + (size_t)q * d.xs3; }
DEV double *dbuf(const Bufs &d, int q) { return d.D3 + (size_t)q * d.xs3; }
DEV double *ubuf(const Bufs &d, int q) { return d.U3 + (size_t)q * d.us3; }

// the control forces element b's stored GRF constraint values at control knot kc come from: the
// knot's own entry of Bufs::cf_u where its cf_flag is set, or nullptr — the working control row's.
// (A pointer, not a copy: the callers read a leg's three forces where they use them, so the
// common case keeps no second force vector in registers.)
DEV const double *constraint_forces(const Bufs &d, const ElemState &E, int b, int kc)
{
    if (!E.ovr) return nullptr;
    const size_t q = (size_t)b * kparams()->Kc + kc;
    return d.cf_flag[q] ? d.cf_u + q * 12 : nullptr;
}
// force a of leg lg for the GRF constraint rows: the control row's, or the older ones (ovr)
DEV double grf_force(const double *u, const double *ovr, int i) { return ovr ? ovr[i] : u[i]; }

DEV void load_contacts(const Bufs &d, const Params &p, int b, int i, int *c, int *cn)
{
    const int *cc = d.contacts + ((size_t)b * (p.P + 1) + i) * 4;
#pragma unroll
    for (int l = 0; l < 4; ++l) { c[l] = cc[l]; cn[l] = cc[4 + l]; }
}

DEV const double *ref_ptr(const Params &p, const double *base, int b, int s, int width)
{
    return base + ((size_t)(p.ref_per_element ? b : 0) * p.S + s) * width;
}

// The reference of state slot s from the entry-major copy (Bufs::ref_t) into rows xr[24], ur[24],
// pf[12]: 30 16-byte loads in flight at once, and lanes on consecutive slots read one contiguous
// piece per entry pair (the rows would be 64 lines per load instruction)
DEV void ref_from_cols(const Params &p, const Bufs &d, int b, int s, double *xr, double *ur, double *pf)
{
    typedef double d2 __attribute__((ext_vector_type(2)));
    const size_t r = (size_t)(p.ref_per_element ? b : 0) * p.S + s, w = d.ref_tw;
    const d2 *col = (const d2 *)d.ref_t + r;
    d2 v[REF_COLS / 2];
#pragma unroll
    for (int j = 0; j < REF_COLS / 2; ++j) v[j] = col[j * w];
#pragma unroll
    for (int j = 0; j < NX / 2; ++j) { xr[2 * j] = v[j].x; xr[2 * j + 1] = v[j].y; }
#pragma unroll
    for (int j = 0; j < NU / 2; ++j) { ur[2 * j] = v[NX / 2 + j].x; ur[2 * j + 1] = v[NX / 2 + j].y; }
#pragma unroll
    for (int j = 0; j < 6; ++j) { pf[2 * j] = v[(NX + NU) / 2 + j].x; pf[2 * j + 1] = v[(NX + NU) / 2 + j].y; }
}

// ReB barrier (ConstraintsBase.h:204-263)
DEV double reb_cost(double g, double delta, double log_delta)
{
    if (g > delta) return -log(g);
    double t = (g - 2 * delta) / delta;
    return .5 * (t * t - 1) - log_delta;
}
// first and second derivative of reb_cost in g; inv_delta = 1 / delta.  One reciprocal per row
// (the branches are selects across lanes, so both sides always execute)
DEV void reb_derivs(double g, double delta, double inv_delta, double &d1, double &d2)
{
    const double r = 1.0 / g, q = inv_delta * inv_delta;
    d1 = g > delta ? -r : (g - 2 * delta) * q;
    d2 = g > delta ? r * r : q;
}

// GRF friction pyramid (HKDConstraints.cpp:7-66): rows of A_leg applied to one leg's force
DEV void grf_row(double mu, int r, double *row)
{
    row[0] = (r == 1) ? -1.0 : (r == 2) ? 1.0 : 0.0;
    row[1] = (r == 3) ? -1.0 : (r == 4) ? 1.0 : 0.0;
    row[2] = (r == 0) ? 1.0 : mu;
}
DEV double grf_value(double mu, int r, const double *f)
{
    double row[3];
    grf_row(mu, r, row);
    return row[0] * f[0] + row[1] * f[1] + row[2] * f[2];
}

// The running cost's terms (running_cost below): the tracking, control and foot sums over their
// entries in order, the dt * ReB sum with min(0, min g), and their combination.  Split so that a
// caller can bring the reference in pieces (k_rollout's slot waves), every term computed as
// running_cost computes it.
DEV double cost_tracking(const Params &p, const int *c, const double *x, const double *xrv)
{
    double lt = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) { double e = x[j] - xrv[j]; lt += e * q_diag(p, c, j) * e; }
    return lt;
}
DEV double cost_control(const Params &p, const double *u, const double *urv)
{
    double lu = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) { double e = u[j] - urv[j]; lu += e * r_diag(p, j) * e; }
    return lu;
}
DEV double cost_foot(const Params &p, const int *c, const double *x, const double *xrv, const double *pfv)
{
    double lf = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        double e = (x[12 + j] - x[3 + j % 3]) - (pfv[j] - xrv[3 + j % 3]);
        lf += e * foot_weight(p, c, j) * e;
    }
    return lf;
}
// ovr: older control forces of the stored GRF constraint values (constraint_forces), else u's
DEV double cost_reb(const Params &p, const int *c, const double *u, const double *delta, const double *eps, double &mk,
                    const double *ovr)
{
    double rc = 0.0;
    mk = 0.0;
    // unrolled: a runtime leg index into u would put the control vector in scratch.  Uniform ReB
    // parameters (the default schedule): one log(delta) for the 20 rows, the value each would compute
    auto reb_sum = [&](auto uniform) {
        if constexpr (decltype(uniform)::value) {
            // uniform parameters (the default schedule): the rows with g > delta of one leg share one
            // log of their product (sum of -log g = -log of the product), the others the quadratic branch
            const double dl = p.grf_delta, e = p.grf_eps, log_du = p.grf_log_delta, inv_dl = p.grf_inv_delta;
#pragma unroll
            for (int lg = 0; lg < 4; ++lg) {
                if (!c[lg]) continue;
                double prod = 1.0, quad = 0.0;
                const double f[3] = {grf_force(u, ovr, 3 * lg), grf_force(u, ovr, 3 * lg + 1), grf_force(u, ovr, 3 * lg + 2)};
#pragma unroll
                for (int r = 0; r < 5; ++r) {
                    const double g = grf_value(p.mu, r, f);
                    mk = fmin(mk, g);
                    const double t = (g - 2 * dl) * inv_dl;
                    prod *= g > dl ? g : 1.0;
                    quad += g > dl ? 0.0 : .5 * (t * t - 1) - log_du;
                }
                rc += e * (quad - log(prod));
            }
        } else {
#pragma unroll
            for (int lg = 0; lg < 4; ++lg) {
                if (!c[lg]) continue;
                const double f[3] = {grf_force(u, ovr, 3 * lg), grf_force(u, ovr, 3 * lg + 1), grf_force(u, ovr, 3 * lg + 2)};
#pragma unroll
                for (int r = 0; r < 5; ++r) {
                    double g = grf_value(p.mu, r, f);
                    mk = fmin(mk, g);
                    rc += eps[5 * lg + r] * reb_cost(g, delta[5 * lg + r], log(delta[5 * lg + r]));
                }
            }
        }
    };
    if (p.reb_uniform) reb_sum(std::true_type{});
    else reb_sum(std::false_type{});
    return rc;
}
DEV double cost_combine(const Params &p, const int *c, double lt, double lu, double lf, double rc)
{
    lt = 0.5 * lt;
    lt += 0.5 * lu;
    lt *= p.dt;
    lf = .5 * lf;
    lf *= p.dt;
    double l = lt + lf;
    if (p.ReB_active && (c[0] + c[1] + c[2] + c[3]) > 0) l += p.dt * rc;
    return l;
}

// running cost l_k (tracking + foot regularisation + dt * ReB), and min(0, min g)
DEV double running_cost(const Params &p, const int *c, const double *x, const double *u, const double *xr,
                        const double *ur, const double *pf, const double *delta, const double *eps, double &viol,
                        const double *ovr = nullptr)
{
    // The reference rows (16-byte aligned: rows of 24 / 12 doubles) as 16-byte loads, all issued
    // before the first use (a lane reads its own slot's rows: each instruction touches up to 64
    // lines, and the vector L1 serves the later pieces of a row — read past it (nt), the forward
    // line search took twice as long)
    typedef double d2v __attribute__((ext_vector_type(2)));
    double xrv[NX], urv[NU], pfv[12];
#pragma unroll
    for (int j = 0; j < NX / 2; ++j) {
        const d2v a = ((const d2v *)xr)[j], b = ((const d2v *)ur)[j];
        xrv[2 * j] = a.x; xrv[2 * j + 1] = a.y;
        urv[2 * j] = b.x; urv[2 * j + 1] = b.y;
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const d2v a = ((const d2v *)pf)[j];
        pfv[2 * j] = a.x; pfv[2 * j + 1] = a.y;
    }
    const double lt = cost_tracking(p, c, x, xrv), lu = cost_control(p, u, urv), lf = cost_foot(p, c, x, xrv, pfv);
    double mk;
    const double rc = cost_reb(p, c, u, delta, eps, mk, ovr);
    viol = mk;
    return cost_combine(p, c, lt, lu, lf, rc);
}

// The step after the sweep / linear rollout of MultiPhaseDDP::solve (MultiPhaseDDP.cpp:331-343):
// merit weight rho from the expected cost change (w1, w2) = (dV_1, dV_2), the merit, the values
// the line search compares against, and the early termination before the line search.
DEV void merit_step(const Params &p, ElemState &E, double w1, double w2)
{
    const double cost = E.cost, feas = E.feas;
    const double dV_abs = fabs(w1 + 0.5 * w2);
    const double rho = (feas > p.feas_thresh) ? dV_abs / ((1 - p.merit_scale) * feas) + p.merit_offset : 0;
    const double merit = cost + rho * feas;
    E.dV1 = w1; E.dV2 = w2; E.merit_rho = rho; E.merit = merit;
    E.cost_prev = cost; E.merit_prev = merit; E.feas_prev = feas;
    if (!p.no_early_exit && dV_abs < p.cost_thresh && feas <= p.feas_thresh) { E.inner_done = 1; E.ls_active = 0; }
    else E.ls_active = 1;
}

// the legs of the phase's touchdown constraints (union of the slot masks; TD_PENDING slots are
// resolved before any solve; TD_STALE is not a leg)
DEV unsigned td_union(const int *mask)
{
    unsigned u = 0;
#pragma unroll
    for (int j = 0; j < MTD; ++j) u |= (unsigned)mask[j];
    return u & 15u;
}
// the touchdown legs from contact c to cn as a mask (add_tconstr_one_phase, HKDProblem.cpp:270-276)
DEV int td_bits(const int *c, const int *cn)
{
    int m = 0;
#pragma unroll
    for (int l = 0; l < 4; ++l) m |= touchdown(c, cn, l) ? 1 << l : 0;
    return m;
}

// terminal cost Phi (tracking Qf + 10 * foot + AL) from the constraint legs' foot heights h[l]
// (hkd_foot_height_grad - ground; any value for other legs), and max |h|.  The AL terms are
// summed per touchdown constraint (slot j: legs mask[j], parameters sig / lam [j][4]) and added
// constraint by constraint, as update_terminal_cost_with_tconstr (SinglePhase.cpp:402-411).
// stored: the constraints' stored residuals (a TD_STALE constraint's is 0), as compute_cost reads
// them; else h as a rollout that completes the phase computes it for every constraint.
DEV double terminal_cost_h(const Params &p, const int *c, const double *x, const double *xr, const double *pf,
                           const int *mask, const double *sig, const double *lam, const double *hl, double &tviol,
                           bool stored = true)
{
    double phi = 0.0, fc = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
        double e = x[j] - xr[j];
        phi += e * (p.qf_gain * p.qf_scale[j] * q_diag(p, c, j)) * e;
    }
    phi *= 0.5;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        double e = (x[12 + j] - x[3 + j % 3]) - (pf[j] - xr[3 + j % 3]);
        fc += e * foot_weight(p, c, j) * e;
    }
    phi = phi + p.foot_term_cost * fc;
    double tv = 0.0;
    for (int q = 0; q < MTD; ++q) {
        const int m = mask[q];
        if (!(m & 15)) continue;
        const bool zero = stored && (m & TD_STALE);
        double al = 0.0;
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            if (!((m >> l) & 1)) continue;
            const double h = zero ? 0.0 : hl[l];
            tv = fmax(tv, fabs(h));
            al += 0.5 * sig[4 * q + l] * h * h;
            al += lam[4 * q + l] * h;
        }
        if (p.AL_active) phi += al;
    }
    tviol = tv;
    return phi;
}

// terminal cost Phi (tracking Qf + 10 * foot + AL), max |h| and h per constraint leg (stored:
// terminal_cost_h)
DEV double terminal_cost(const Params &p, const int *c, const double *x, const double *xr, const double *pf,
                         const int *mask, const double *sig, const double *lam, double &tviol, double *h_out,
                         bool stored)
{
    const unsigned u = td_union(mask);
#pragma unroll
    for (int l = 0; l < 4; ++l) h_out[l] = ((u >> l) & 1) ? hkd_foot_height_grad(l, x, nullptr) - p.ground : 0.0;
    return terminal_cost_h(p, c, x, xr, pf, mask, sig, lam, h_out, tviol, stored);
}



}  // namespace hsddp
