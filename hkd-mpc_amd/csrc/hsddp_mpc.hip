// hsddp_mpc.hip — the MPC caller's steps on either side of the solve, batched
// over the B elements of a handle.
//
//   k_extract_commands   HKDMPCSolver::update_foot_placement + publish_mpc_cmd (HKDMPC.cpp:207-298):
//                        the first N_mpcsteps control knots of the solved trajectory into the
//                        hkd_command_lcmt layout (lcmtypes/hkd_command_lcmt.lcm:1-11), one
//                        workgroup per element, threads striding over the record's fields.
//   k_build_refs         HKDSinglePhaseReference::get_reference_at_t at every slot of every element
//                        from a device-resident sample table (HKDReference.cpp:8-57).
//   k_shift_gather       HKDProblem::update's trajectory edits (HKDProblem.cpp:117-222): the
//                        warm start (Xbar, Ubar, K) re-laid for the shifted phases — dropped
//                        front knots / phases, pushed-back copies of X.back(), zero new phases —
//                        as one gather over (element, new slot, entry) from host-built slot maps;
//                        k_shift_gather_work then the working rows (X, U, Defect) alike.
#include <cstddef>
#include "../../include/hsddp.h"
#include "hsddp_device.h"
#include "hsddp_mpc.h"

namespace hsddp {

// One element per workgroup.  The knot walk of publish_mpc_cmd (phase i, knot s; HKDMPC.cpp:
// 239-246) depends only on the horizons: with the handle's shared layout the host passes it
// resolved (a.kc[k], a.xs[k], a.ph[k]); with per-element layouts (EL) the workgroup walks its
// element's own layout first.
template <bool EL>
__global__ __launch_bounds__(256) void k_extract_commands(Params p, Bufs d, CmdArgs a, hsddp_mpc_command *out)
{
    const int b = blockIdx.x, t = threadIdx.x;
    hsddp_mpc_command &o = out[b];
    const auto L = layout_of<EL>(d, b);
    __shared__ int wkc[HSDDP_CMD_STEPS], wxs[HSDDP_CMD_STEPS], wph[HSDDP_CMD_STEPS];
    if (t == 0) {
        if constexpr (EL) {
            for (int k = 0, i = 0, s = 0; k < a.n; ++k, ++s) {
                if (s >= L.N(i)) { s = 0; ++i; }
                wkc[k] = L.k0(i) + s;
                wxs[k] = L.s0(i) + s;
                wph[k] = i;
            }
        } else {
#pragma unroll
            for (int k = 0; k < HSDDP_CMD_STEPS; ++k) { wkc[k] = a.kc[k]; wxs[k] = a.xs[k]; wph[k] = a.ph[k]; }
        }
    }
    __syncthreads();
    const int *cb = d.contacts + (size_t)b * (p.P + 1) * 4;
    const double *Xbar = xbuf(d, nom_buf(d, b)), *Ubar = ubuf(d, nom_buf(d, b));
    // controls, body states, feedback rows (zero past N_mpcsteps, as a fresh message)
    for (int e = t; e < HSDDP_CMD_STEPS * 24; e += blockDim.x) {
        const int k = e / 24, j = e % 24;
        o.hkd_controls[k][j] = k < a.n ? (float)Ubar[((size_t)b * p.Kc + wkc[k]) * NX + j] : 0.f;
    }
    for (int e = t; e < HSDDP_CMD_STEPS * 12; e += blockDim.x) {
        const int k = e / 12, j = e % 12;
        o.des_body_state[k][j] = k < a.n ? (float)Xbar[((size_t)b * p.S + wxs[k]) * NX + j] : 0.f;
    }
    // K(m, n), m, n < 12: control m is leg m/3's GRF; its gain row is compact row m when the leg
    // is in stance and exactly zero when it swings (KCW layout, hsddp_internal.h)
    for (int e = t; e < HSDDP_CMD_STEPS * 144; e += blockDim.x) {
        const int k = e / 144, m = (e / 12) % 12, n = e % 12;
        float v = 0.f;
        if (k < a.n && cb[wph[k] * 4 + m / 3]) {
            const size_t idx = ((size_t)b * p.Kc + wkc[k]) * KCW + m * NX + n;
            v = p.fp32 ? d.K32[idx] : (float)d.K[idx];
        }
        o.feedback[k][m][n] = v;
    }
    for (int e = t; e < HSDDP_CMD_STEPS * 4; e += blockDim.x) {
        const int k = e / 4, l = e % 4;
        const bool on = k < a.n;
        o.contacts[k][l] = on ? cb[wph[k] * 4 + l] : 0;
        const double *dur = a.durations ? a.durations + ((size_t)(a.dur_per_elem ? b : 0) * p.P + wph[k]) * 4 : nullptr;
        o.statusTimes[k][l] = (on && dur) ? dur[l] : 0.0;
    }
    // mpc_time + k dt_mpc rounded twice, as written (no fused multiply-add)
    if (t < HSDDP_CMD_STEPS) o.mpc_times[t] = t < a.n ? __dadd_rn(a.mpc_time, __dmul_rn((double)t, a.dt_mpc)) : 0.0;
    // update_foot_placement (HKDMPC.cpp:207-230): the first swing -> stance transition of leg l
    // among phase pairs (i, i + 1), i = 0 .. 4, gives the foot position stored in the next phase's
    // first state (qdummy, states 12 + 3 l ..); otherwise the current foot position
    if (t < 12) {
        const int l = t / 3, ax = t % 3;
        float pf = a.feet ? a.feet[(size_t)(a.feet_per_elem ? b : 0) * 12 + t] : 0.f;
        for (int i = 0; i < L.P() - 1 && i <= 4; ++i) {
            if (cb[i * 4 + l] == 0 && cb[(i + 1) * 4 + l] == 1) {
                pf = (float)Xbar[((size_t)b * p.S + L.s0(i + 1)) * NX + 12 + 3 * l + ax];
                break;
            }
        }
        o.foot_placement[t] = pf;
    }
    if (t == 0) {
        o.N_mpcsteps = a.n;
        o.solve_time = a.solve_time;
    }
    // the struct's padding bytes (after N_mpcsteps, after solve_time) zero too: a record is the same
    // bytes wherever it is extracted (device buffers are not cleared; the multi-GPU gather sends bytes)
    constexpr size_t p0 = offsetof(hsddp_mpc_command, N_mpcsteps) + sizeof(int), p1 = offsetof(hsddp_mpc_command, mpc_times);
    constexpr size_t p2 = offsetof(hsddp_mpc_command, solve_time) + sizeof(float), p3 = sizeof(hsddp_mpc_command);
    char *ob = reinterpret_cast<char *>(&o);
    if (t < (int)(p1 - p0)) ob[p0 + t] = 0;
    if (t < (int)(p3 - p2)) ob[p2 + t] = 0;
}

// One thread per 16 bytes (two doubles / four floats, never straddling a row: NX and KCW are
// multiples of 4) of the new Xbar / Ubar rows and compact K rows of every element; gathered reads,
// contiguous writes.  The new rows go to the element's third buffer (neither its nominal nor its
// working one, which the gather reads); k_shift_sel then makes it both.
// element b's old state rows (stride S_old): nominal X (q = 0), working X (1), working Defect (2),
// in place or from the staging copy
DEV const double *old_rows(const ShiftArgs &a, const Bufs &d, long b, int q)
{
    if (a.stage) return a.stage + ((size_t)q * d.rows3 + b * a.S_old) * NX;
    const int buf = q == 0 ? nom_buf(d, (int)b) : work_buf(d, (int)b);
    return (q == 2 ? dbuf(d, buf) : xbuf(d, buf)) + b * a.S_old * NX;
}

// the staging copy (ShiftArgs::stage): one thread per 16 bytes of an element's old rows
__global__ __launch_bounds__(256) void k_shift_stage(int B, ShiftArgs a, Bufs d)
{
    const long per = (long)a.S_old * NX / 2, gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= 3L * B * per) return;
    const int q = (int)(gid / ((long)B * per));
    const long r = gid % ((long)B * per), b = r / per;
    const int nb = nom_buf(d, (int)b), wb = work_buf(d, (int)b);
    if (q == 1 && nb == wb) return;  // (read from the nominal copy)
    const double *src = (q == 2 ? dbuf(d, wb) : xbuf(d, q == 0 ? nb : wb)) + b * a.S_old * NX;
    reinterpret_cast<double2 *>(a.stage + ((size_t)q * d.rows3 + b * a.S_old) * NX)[r % per] =
        reinterpret_cast<const double2 *>(src)[r % per];
}

template <typename KT>
__global__ __launch_bounds__(256) void k_shift_gather(int B, ShiftArgs a, Bufs d, const KT *K, KT *Kn)
{
    constexpr int KV = 16 / sizeof(KT);  // K values per thread
    const long nx = (long)a.S_new * NX / 2, nu = (long)a.Kc * NX / 2, nk = (long)a.Kc * KCW / KV, per = nx + nu + nk;
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)B * per) return;
    const long b = gid / per;
    long e = gid % per;
    const int m = a.map_id ? a.map_id[b] : 0;
    const bool same = nom_buf(d, (int)b) == work_buf(d, (int)b);
    const double *Xbar = old_rows(a, d, b, 0), *X = old_rows(a, d, b, same ? 0 : 1),
                 *Ubar = ubuf(d, nom_buf(d, (int)b));
    double *Xn = xbuf(d, trial_buf(d, (int)b)), *Un = ubuf(d, trial_buf(d, (int)b));
    const int *smap = a.smap + (size_t)m * a.S_new, *cmap = a.cmap + (size_t)m * a.Kc;
    if (e < nx) {
        const int s = (int)(2 * e / NX), j = (int)(2 * e % NX), lab = smap[s];
        double2 v = {0.0, 0.0};
        if (lab >= 0) v = *(const double2 *)&Xbar[lab * NX + j];
        else if (lab <= -2) v = *(const double2 *)&X[(-2 - lab) * NX + j];
        *(double2 *)&Xn[(b * nx + e) * 2] = v;
        return;
    }
    e -= nx;
    if (e < nu) {
        const int k = (int)(2 * e / NX), j = (int)(2 * e % NX), lab = cmap[k];
        double2 v = {0.0, 0.0};
        if (lab >= 0 && !(a.zero_u0 && k == 0)) v = *(const double2 *)&Ubar[(b * a.Kc + lab) * NX + j];
        *(double2 *)&Un[(b * nu + e) * 2] = v;
        return;
    }
    e -= nu;
    const int k = (int)(KV * e / KCW), j = (int)(KV * e % KCW), lab = cmap[k];
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (lab >= 0) v = *(const float4 *)&K[((long)b * a.Kc + lab) * KCW + j];
    *(float4 *)&Kn[(b * nk + e) * KV] = v;
}

// The working trajectory through the same update (Trajectory::pop_front / push_back_state,
// TrajectoryManagement.cpp:118-207; a new phase's rows are zero): X rows by the state map (a
// pushed-back state is X.back() either way), U rows by the control map (a new knot's are zero;
// Ubar[0]'s zeroing is the nominal's only), Defect rows by the state map with a pushed-back state's
// zero.  After k_shift_gather: an element whose working rows are its nominal ones (no failed last
// line search, sel nominal == working) gathers only its Defect, into the third buffer beside the
// new nominal rows; any other gathers X, U and Defect into its old nominal buffer, which
// k_shift_gather has finished reading.
__global__ __launch_bounds__(256) void k_shift_gather_work(int B, ShiftArgs a, Bufs d)
{
    const long nx = (long)a.S_new * NX / 2, nu = (long)a.Kc * NX / 2, per = 2 * nx + nu;
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)B * per) return;
    const long b = gid / per;
    long e = gid % per;
    const int nb = nom_buf(d, (int)b), wb = work_buf(d, (int)b), same = nb == wb;
    const int m = a.map_id ? a.map_id[b] : 0, dst = same ? trial_of(nb, wb) : nb;
    const int *smap = a.smap + (size_t)m * a.S_new, *cmap = a.cmap + (size_t)m * a.Kc;
    if (e < nx) {  // Defect
        const int s = (int)(2 * e / NX), j = (int)(2 * e % NX), lab = smap[s];
        double2 v = {0.0, 0.0};
        if (lab >= 0) v = *(const double2 *)&old_rows(a, d, b, 2)[lab * NX + j];
        *(double2 *)&dbuf(d, dst)[(b * nx + e) * 2] = v;
        return;
    }
    if (same) return;
    e -= nx;
    if (e < nx) {  // X
        const int s = (int)(2 * e / NX), j = (int)(2 * e % NX), lab = smap[s];
        const int src = lab >= 0 ? lab : -2 - lab;
        double2 v = {0.0, 0.0};
        if (lab != -1) v = *(const double2 *)&old_rows(a, d, b, 1)[src * NX + j];
        *(double2 *)&xbuf(d, dst)[(b * nx + e) * 2] = v;
        return;
    }
    e -= nx;
    const int k = (int)(2 * e / NX), j = (int)(2 * e % NX), lab = cmap[k];
    double2 v = {0.0, 0.0};
    if (lab >= 0) v = *(const double2 *)&ubuf(d, wb)[(b * a.Kc + lab) * NX + j];
    *(double2 *)&ubuf(d, dst)[(b * nu + e) * 2] = v;
}

// new selection: nominal = the third buffer; working = the same, or the old nominal buffer
__global__ void k_shift_sel(int B, Bufs d)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const int nb = nom_buf(d, b), wb = work_buf(d, b), t = trial_of(nb, wb);
    d.sel[b] = sel_code(t, nb == wb ? t : nb);
}

void launch_shift_gather(int B, const ShiftArgs &a, const Bufs &d, void *K_new, hipStream_t st)
{
    static_assert(NX % 4 == 0 && KCW % 4 == 0, "16-byte pieces within rows");
    const int KV = a.fp32 ? 4 : 2;
    const long n = (long)B * ((long)a.S_new * NX / 2 + (long)a.Kc * NX / 2 + (long)a.Kc * KCW / KV);
    const dim3 g((unsigned)((n + 255) / 256));
    if (a.stage) {
        const long ns = 3L * B * a.S_old * NX / 2;
        hipLaunchKernelGGL(k_shift_stage, dim3((unsigned)((ns + 255) / 256)), dim3(256), 0, st, B, a, d);
    }
    if (a.fp32)
        hipLaunchKernelGGL(k_shift_gather<float>, g, dim3(256), 0, st, B, a, d, d.K32, (float *)K_new);
    else
        hipLaunchKernelGGL(k_shift_gather<double>, g, dim3(256), 0, st, B, a, d, d.K, (double *)K_new);
    const long nw = (long)B * ((long)a.S_new * NX + (long)a.Kc * NX / 2);
    hipLaunchKernelGGL(k_shift_gather_work, dim3((unsigned)((nw + 255) / 256)), dim3(256), 0, st, B, a, d);
    hipLaunchKernelGGL(k_shift_sel, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, st, B, d);
}

// The constraint objects the phases carry through HKDProblem::update (HKDProblem.cpp:117-222):
// per-knot ReB (delta, eps) follow their knots (PathConstraintBase::pop_front / push_back,
// ConstraintsBase.h:147-158, 271-291: a pushed knot copies the last one's; a new phase starts from
// the initial values), and so do the stored GRF values (a pushed knot's are zero, as its working
// control row: no table entry); each phase keeps its touchdown constraints with their AL
// parameters and stored residuals; the update's add_tconstr_one_phase appends one more (initial
// parameters, zero residual, legs resolved from the next contact rows: TD_PENDING | TD_STALE) at
// every step its last phase has reached its end.  One thread per (element, control slot, row) and
// per (element, new phase).
__global__ __launch_bounds__(256) void k_shift_params(int B, ShiftParamArgs a, Bufs d, ShiftParamOut o)
{
    const long nr = (long)B * a.Kc * 20, gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < nr) {
        const long b = gid / ((long)a.Kc * 20);
        const int k = (int)(gid / 20 % a.Kc), r = (int)(gid % 20);
        const int m = a.map_id ? a.map_id[b] : 0, lab = a.rmap[(size_t)m * a.Kc + k];
        o.reb_delta[gid] = lab >= 0 ? d.reb_delta[(b * a.Kc + lab) * 20 + r] : a.reb_delta0;
        o.reb_eps[gid] = lab >= 0 ? d.reb_eps[(b * a.Kc + lab) * 20 + r] : a.reb_eps0;
        if (d.el[b].ovr && r < 12) {  // (an element's table is read only while its ovr is set)
            const int src = a.cmap[(size_t)m * a.Kc + k];
            o.cf_u[(b * a.Kc + k) * 12 + r] = src >= 0 ? d.cf_u[(b * a.Kc + src) * 12 + r] : 0.0;
            if (r == 0) o.cf_flag[b * a.Kc + k] = src >= 0 ? d.cf_flag[b * a.Kc + src] : 0;
        }
        return;
    }
    const long g = gid - nr;
    if (g >= (long)B * a.P_new) return;
    const long b = g / a.P_new;
    const int i = (int)(g % a.P_new), m = a.map_id ? a.map_id[b] : 0;
    const int src = a.pmap[m * MAXP + i], add = a.nadd[m * MAXP + i];
    const size_t w = ((size_t)b * a.P_new + i) * MTD, q = ((size_t)b * a.P_old + src) * MTD;
    int mask[MTD];
    for (int j = 0; j < MTD; ++j) {
        mask[j] = src >= 0 ? d.td_mask[q + j] : 0;
        for (int l = 0; l < 4; ++l) {
            o.al_sigma[(w + j) * 4 + l] = src >= 0 ? d.al_sigma[(q + j) * 4 + l] : a.td_sigma0;
            o.al_lambda[(w + j) * 4 + l] = src >= 0 ? d.al_lambda[(q + j) * 4 + l] : a.td_lambda0;
        }
    }
    for (int n = 0; n < add; ++n) {  // appended constraints take the first free slots
        int j = 0;
        while (j < MTD && mask[j]) ++j;
        if (j == MTD) {
            atomicAdd(a.overflow, 1);
            break;
        }
        mask[j] = TD_PENDING | TD_STALE;
        d.el[b].td_stale = 1;
        for (int l = 0; l < 4; ++l) {
            o.al_sigma[(w + j) * 4 + l] = a.td_sigma0;
            o.al_lambda[(w + j) * 4 + l] = a.td_lambda0;
        }
    }
    for (int j = 0; j < MTD; ++j) o.td_mask[w + j] = mask[j];
}

void launch_shift_params(int B, const ShiftParamArgs &a, const Bufs &d, const ShiftParamOut &o, hipStream_t st)
{
    const long n = (long)B * a.Kc * 20 + (long)B * a.P_new;
    hipLaunchKernelGGL(k_shift_params, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, B, a, d, o);
}

// HKDSinglePhaseReference::get_reference_at_t (HKDReference.cpp:8-57) at state slot s of reference
// element b: one thread per (b, s); the slot -> sample offset map is shared (host-built with the
// reference's float time rounding), the window start is per element.
__global__ __launch_bounds__(256) void k_build_refs(Params p, Bufs d, int Bref, RefArgs a)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)Bref * p.S) return;
    const int b = (int)(gid / p.S), s = (int)(gid % p.S);
    int k = a.start[b] + a.slot_idx[(size_t)(a.map_id ? a.map_id[b] : 0) * p.S + s];
    k = k < a.n ? k : a.n - 1;  // past the loaded data: its last sample
    const double *q = a.table + (size_t)k * RT_W;
    double *rx = (double *)d.ref_x + gid * NX, *ru = (double *)d.ref_u + gid * NX, *rf = (double *)d.ref_foot + gid * 12;
    for (int j = 0; j < 12; ++j) rx[j] = q[RT_BODY + j];
    for (int l = 0; l < 4; ++l)
        for (int c = 0; c < 3; ++c)
            rx[12 + 3 * l + c] = q[RT_C + l] > 0 ? q[RT_FOOT + 3 * l + c] : q[RT_QJ + 3 * l + c];
    for (int j = 0; j < 12; ++j) {
        ru[j] = q[RT_GRF + j];
        ru[12 + j] = q[RT_QJD + j];
        rf[j] = q[RT_FOOT + j];
    }
    // the entry-major copy (Bufs::ref_t, column gid) from the rows just written: no separate pass
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 *col = (d2 *)d.ref_t + gid;
    for (int j = 0; j < NX / 2; ++j) col[(size_t)j * d.ref_tw] = d2{rx[2 * j], rx[2 * j + 1]};
    for (int j = 0; j < NU / 2; ++j) col[(size_t)(NX / 2 + j) * d.ref_tw] = d2{ru[2 * j], ru[2 * j + 1]};
    for (int j = 0; j < 6; ++j) col[(size_t)((NX + NU) / 2 + j) * d.ref_tw] = d2{rf[2 * j], rf[2 * j + 1]};
}

void launch_build_refs(const Params &p, const Bufs &d, int Bref, const RefArgs &a, hipStream_t st)
{
    const long n = (long)Bref * p.S;
    hipLaunchKernelGGL(k_build_refs, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, p, d, Bref, a);
}

void launch_extract_commands(const Params &p, const Bufs &d, const CmdArgs &a, hsddp_mpc_command *out,
                             hipStream_t st)
{
    if (p.elem_layout) hipLaunchKernelGGL(k_extract_commands<true>, dim3(p.B), dim3(256), 0, st, p, d, a, out);
    else hipLaunchKernelGGL(k_extract_commands<false>, dim3(p.B), dim3(256), 0, st, p, d, a, out);
}

}  // namespace hsddp
