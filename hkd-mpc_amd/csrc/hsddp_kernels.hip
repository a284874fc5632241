// hsddp_kernels.hip — CDNA4 (gfx950) kernels of the batched HS-DDP solver, fp64.
//
// One DDP inner iteration of MultiPhaseDDP::solve (HSDDPSolver/source/MultiPhaseDDP.cpp:304-381)
// for B trajectories is:
//   k_lq        knot-parallel  cost at (X, U) + compact LQ model   SinglePhase::compute_cost/LQ_approximation
//   (terminal)  (elem, phase)  Phix, Phixx (+AL), reset Jacobian   SinglePhase.cpp:286-295; HKDReset.h:78-136
//                              one wave per task, the last blocks of the k_lq launch
//   k_riccati   one wave/2 elems regularised Riccati sweep over all phases   (hsddp_sweep.hip)
//                              MultiPhaseDDP.cpp:141-229; SinglePhase.cpp:298-367
//   k_lin_rollout one wave/2 elems  MS linear rollout + merit                (hsddp_linear.hip)
//                              MultiPhaseDDP.cpp:20-50, 309-318; SinglePhase.cpp:144-178
//   k_rollout   knot-parallel  one line-search trial (all knots are shooting states)  SinglePhase.cpp:181-233
//   k_decide    per element    merit acceptance (MultiPhaseDDP.cpp:113-133) + inner-loop exit tests;
//                              Trajectory::update_nominal_vals (TrajectoryManagement.cpp:110-115)
//                              is its flip of the element's nominal buffer (no copies)
// plus the outer AL/ReB updates (ConstraintsBase.h:168-183, 349-365; MultiPhaseDDP.cpp:383-408).
//
// Every element carries its own control-flow state (ElemState): regularisation retries, line-search
// acceptance, early exits and AL/ReB updates are per-element masks, never lockstep.
#include <cstdlib>

#include "hsddp_device.h"

namespace hsddp {

using namespace hkd;

#ifndef HSDDP_RO_EXP
#define HSDDP_RO_EXP 0  // timing experiments only: 1 no Defect row stores, 2 no trial U row stores (k_rollout),
                        // 3 no running cost, 4 running cost without reference loads, 5 no control-row loads or stores
#endif
#ifndef HSDDP_STAMPS
#define HSDDP_STAMPS 0
#endif
// Diagnostic build (make stamps): s_memtime at the stage boundaries of a k_rollout slot wave (each
// after an LDS drain only: a stage's own loads are waited where they are used), the differences of
// every full slot wave added into Bufs::dbg — element 0's slots 12 .. 15 and element 1's slots 0 .. 3
// (the sweep and the linear rollout use the others) — tools/stamps.py
#if HSDDP_STAMPS
#define RSTAMP(n)                                                                             \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        unsigned long long t_;                                                                \
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        rst[n] = t_;                                                                          \
    } while (0)
#else
#define RSTAMP(n) \
    do {          \
    } while (0)
#endif
#ifndef HSDDP_LQ_EXP
#define HSDDP_LQ_EXP 0  // timing experiment only: 1 no terminal tasks
#endif
#ifndef FWD_MINB
#define FWD_MINB 2  // 256-thread blocks per CU for the knot-parallel kernels (k_lq, k_rollout)
#endif

// ---------------------------------------------------------------------------------------------
// Record stores of k_lq.  One lane computes one knot's record, so direct stores from the lanes hit
// 64 records (64 cache lines) per instruction.  For the gradient pieces (lx, lu, ReB Hessian) each
// wave instead stages the piece of its records in LDS (lane-major, odd stride) and the lanes still
// active write it back record by record: consecutive lanes write consecutive 2-value pairs of one
// record, so an instruction covers ~1 KB of contiguous records.  Pieces are even-sized at even
// offsets, so every pair is aligned in HBM.  Lanes that returned early (past the batch, finished
// element, phase-end slot) left ridx = -1 and their records are skipped.
// LDS stride per lane: one 128-byte line of a record (16 fp64 / 32 fp32 values) + 1
template <typename T> constexpr int LQ_STG = 128 / (int)sizeof(T) + 1;

// the wave's staged values (record positions OFF .. OFF + N - 1 at stage columns 0 .. N - 1) to the
// records, pair by pair, by the still-active lanes
template <typename T>
DEV void lq_flush(T *wl, const long *ridx, T *lq, int ldw, int lane, int OFF, int N)
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    using T2 = std::conditional_t<std::is_same_v<T, float>, float2, double2>;
    const unsigned long long m = __ballot(1);
    const int na = __popcll(m), rank = __popcll(m & ((1ull << lane) - 1));
    for (int q = rank; q < 64 * (N / 2); q += na) {
        const int r = q / (N / 2), jp = q % (N / 2);
        const long rr = ridx[r];
        if (rr >= 0) {
            T2 w;
            w.x = wl[r * LQ_STG<T> + 2 * jp];
            w.y = wl[r * LQ_STG<T> + 2 * jp + 1];
            *reinterpret_cast<T2 *>(lq + rr * ldw + OFF + 2 * jp) = w;
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}


// The terminal task of one (element, phase): Phix, Phixx (+AL, quirk A4) and the reset-map
// Jacobian Px, on TERM_TL lanes — TERM_TPW tasks share a wave (the per-task work is mostly serial:
// the leg kinematics on four lanes, the cost on one), so the LDS per task, not the wave count,
// bounds how many run at once.
#ifndef HSDDP_TERM_TPW
#define HSDDP_TERM_TPW 2
#endif
constexpr int TERM_TPW = HSDDP_TERM_TPW, TERM_TL = 64 / TERM_TPW;
struct TermLds {
    double sx[NX], shx[4][NX], scoef[4][2], sh[4], sxr[NX], spf[12], ssl[2 * MTD * 4];
    double sdw[NX + 12];  // the foot Hessian's diagonal, then its cross weights; first the 15 angles' sin / cos
    double spx[12 * (NX + 1)];  // Px rows 12 .. 23 (rows 0 .. 11 are the identity's)
    int sc[4], scn[4], smask[MTD];
};
static_assert(TERM_TL >= NX && TERM_TL >= 2 * MTD * 4 && TERM_TL >= 16, "terminal lane roles");

// LDS hand-over between the lanes of one wave (its LDS accesses complete in order)
DEV void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool EL>
DEV void terminal_task(const Params &p, const Bufs &d, TermLds &S, int task, int t)
{
    const int b = task / p.P, i = task % p.P;
    const ElemState &E = d.el[b];
    if (E.done || E.inner_done) return;
    const auto L = layout_of<EL>(d, b);
    const int P = L.P();
    if (i >= P) return;
    double *sx = S.sx, (*shx)[NX] = S.shx, (*scoef)[2] = S.scoef, *sh = S.sh, *sxr = S.sxr, *spf = S.spf, *ssl = S.ssl;
    int *sc = S.sc, *scn = S.scn, *smask = S.smask;
    const int s = L.s0(i) + L.N(i);
    const double *xr = ref_ptr(p, d.ref_x, b, s, NX), *pf = ref_ptr(p, d.ref_foot, b, s, 12);
    // X[N] and the terminal cost's other inputs, staged together (no memory round trip at the end)
    if (t < NX) {
        sx[t] = xbuf(d, work_buf(d, b))[((size_t)b * p.S + s) * NX + t];
        sxr[t] = xr[t];
    }
    // the phase's touchdown constraints: AL parameters [slot][leg] (sigma, then lambda) and leg masks
    if (t < 2 * MTD * 4) ssl[t] = (t < MTD * 4 ? d.al_sigma : d.al_lambda)[((size_t)b * p.P + i) * MTD * 4 + (t & (MTD * 4 - 1))];
    constexpr int MK = TERM_TL - MTD;
    if (t >= MK) smask[t - MK] = d.td_mask[((size_t)b * p.P + i) * MTD + t - MK];
    if (t >= 4 && t < 16) spf[t - 4] = pf[t - 4];
    if (t < 4) {
        const int *cc = d.contacts + ((size_t)b * (p.P + 1) + i) * 4;
        sc[t] = cc[t]; scn[t] = cc[4 + t];
    }
    wave_sync();
    // Px at X_i[N] (HKDReset.h:78-136) is built in LDS from the identity (phase boundaries only)
    double *spx = S.spx;
    const bool bnd = i < P - 1;
    for (int e = t; e < 4 * NX; e += TERM_TL) (&shx[0][0])[e] = 0.0;
    if (bnd)
        for (int e = t; e < 12 * (NX + 1); e += TERM_TL) spx[e] = (e / (NX + 1) + 12 == e % (NX + 1)) ? 1.0 : 0.0;
    // the kinematics' 15 angles, one sincos per lane: yaw, pitch, roll, then per leg q0, q1, q1 + q2
    double *strig = S.sdw;
    unsigned need = td_union(smask);
#pragma unroll
    for (int l = 0; l < 4; ++l) need |= (bnd && touchdown(sc, scn, l)) ? 1u << l : 0u;
    if (need && t < 15) {
        const int m = t - 3;
        const double a = t < 3 ? sx[t] : m % 3 == 2 ? sx[11 + m] + sx[12 + m] : sx[12 + m];
        sincos(a, &strig[2 * t], &strig[2 * t + 1]);
    }
    wave_sync();
#ifndef HSDDP_TERM_EXP
#define HSDDP_TERM_EXP 0
#endif
    if ((HSDDP_TERM_EXP & 2) == 0 && t < 4) {
        // legs of the touchdown constraints: foot height h and its gradient (non-zeros at 0..2, 5,
        // 12 + 3 l + k); legs touching down at a phase boundary: the reset map's foot-Jacobian rows
        // — from one evaluation of the leg's kinematics (hkd_foot_height_grad_sparse's and
        // hkd_foot_jacobian's expressions)
        const int l = t;
        const bool tdc = (td_union(smask) >> l) & 1, tdr = touchdown(sc, scn, l);
        double h = 0.0;
        if (tdc || (bnd && tdr)) {
            Rot R, Dy, Dp, Dr;
            const EulTrig tr{strig[1], strig[0], strig[3], strig[2], strig[5], strig[4]};
            rot_zyx(tr, R);
            rot_zyx_grad(tr, Dy, Dp, Dr);
            double pb[3], dpb[3][3];
            foot_body_trig(l, strig + 6 + 6 * l, pb, dpb);
            shx[l][0] = Dy.r[2][0] * pb[0] + Dy.r[2][1] * pb[1] + Dy.r[2][2] * pb[2];
            shx[l][1] = Dp.r[2][0] * pb[0] + Dp.r[2][1] * pb[1] + Dp.r[2][2] * pb[2];
            shx[l][2] = Dr.r[2][0] * pb[0] + Dr.r[2][1] * pb[1] + Dr.r[2][2] * pb[2];
#pragma unroll
            for (int k = 0; k < 3; ++k) shx[l][12 + 3 * l + k] = R.r[2][0] * dpb[0][k] + R.r[2][1] * dpb[1][k] + R.r[2][2] * dpb[2][k];
            shx[l][5] = 1.0;
            h = (sx[5] + R.r[2][0] * pb[0] + R.r[2][1] * pb[1] + R.r[2][2] * pb[2]) - p.ground;
            if (!tdc) {  // a reset-map leg without a constraint: no AL gradient
                h = 0.0;
#pragma unroll
                for (int j = 0; j < NX; ++j) shx[l][j] = 0.0;
            }
            if (bnd && tdr) {  // rows 12 + 3 l + k, k < 2: the foot Jacobian's rows; the k = 2 row is zero
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    double *row = spx + (3 * l + k) * (NX + 1);
                    row[12 + 3 * l + k] = 0.0;
                    if (k == 2) continue;
                    row[0] = Dy.r[k][0] * pb[0] + Dy.r[k][1] * pb[1] + Dy.r[k][2] * pb[2];
                    row[1] = Dp.r[k][0] * pb[0] + Dp.r[k][1] * pb[1] + Dp.r[k][2] * pb[2];
                    row[2] = Dr.r[k][0] * pb[0] + Dr.r[k][1] * pb[1] + Dr.r[k][2] * pb[2];
                    row[3 + k] = 1.0;
#pragma unroll
                    for (int m = 0; m < 3; ++m)
                        row[12 + 3 * l + m] = R.r[k][0] * dpb[0][m] + R.r[k][1] * dpb[1][m] + R.r[k][2] * dpb[2][m];
                }
            }
        } else if (bnd && sc[l] && !scn[l]) {  // lift-off: rows 12 + 3 l + k zero
#pragma unroll
            for (int k = 0; k < 3; ++k) spx[(3 * l + k) * (NX + 2) + 12] = 0.0;
        }
        // AL gradient / Hessian coefficients of the leg, summed over the constraints holding it
        // (quirk A4: (sigma (1 + h) + lambda) hx hx^T, ConstraintsBase.h:374-399)
        double c0 = 0.0, c1 = 0.0;
        if (tdc && p.AL_active)
            for (int q = 0; q < MTD; ++q)
                if ((smask[q] >> l) & 1) {
                    const double sg = ssl[4 * q + l], lm = ssl[MTD * 4 + 4 * q + l];
                    const double hq = (smask[q] & TD_STALE) ? 0.0 : h;  // the constraint's stored h
                    c0 += sg * hq + lm;
                    c1 += sg * (1 + hq) + lm;
                }
        scoef[l][0] = c0;
        scoef[l][1] = c1;
        sh[l] = h;
    }
    wave_sync();
    KParams &kp = *kparams();  // runtime-indexed weights
    double *rec = d.term + ((size_t)b * p.P + i) * TW;
    if ((HSDDP_TERM_EXP & 1) == 0 && t == 0) {  // the phase's terminal cost at X[N] (SinglePhase::compute_cost's last term) for k_lq's slot sums
        double tv;
        d.slot_cost[(size_t)b * p.S + s] = terminal_cost_h(p, sc, sx, sxr, spf, smask, ssl, ssl + MTD * 4, sh, tv);
    }
    if ((HSDDP_TERM_EXP & 8) == 0 && t < NX) { // Phix
        const int j = t;
        double v = kp.qf_gain * kp.qf_scale[j] * q_diag(kp, sc, j) * (sx[j] - sxr[j]);
        if (j >= 3 && j < 6) {
            for (int l = 0; l < 4; ++l) {
                int m = 3 * l + (j - 3);
                double e = (sx[12 + m] - sx[j]) - (spf[m] - sxr[j]);
                v += -(p.foot_term_grad * sc[l] * foot_weight(kp, sc, m) * e);
            }
        } else if (j >= 12) {
            int m = j - 12, l = m / 3;
            double e = (sx[j] - sx[3 + m % 3]) - (spf[m] - sxr[3 + m % 3]);
            v += p.foot_term_grad * sc[l] * foot_weight(kp, sc, m) * e;
        }
        for (int l = 0; l < 4; ++l) v += scoef[l][0] * shx[l][j];
        rec[TM_PHIX + j] = v;
    }
    // foot Hessian 20 D^T Qfoot D: weight of (leg l, axis j), entries (3 + j, 3 + j) (summed over
    // the legs in leg order), (12 + 3 l + j, 12 + 3 l + j) and, negated, the two cross entries.
    // Lane r < 24 forms diagonal entry r, lane m < 12 also the weight of joint column 12 + m
    // (runtime-indexed weights read once per phase, not once per entry); the 576 entries then
    // combine them.
    auto fw = [&](int l, int j) { return p.foot_term_grad * sc[l] * sc[l] * foot_weight(kp, sc, 3 * l + j); };
    double *sdd = S.sdw, *scw = S.sdw + NX;  // (the trig is dead: read before the last wave_sync)
    if (t < NX) {
        const int r = t;
        double v = kp.qf_gain * kp.qf_scale[r] * q_diag(kp, sc, r);
        if (r >= 3 && r < 6) {
            for (int l = 0; l < 4; ++l) v += fw(l, r - 3);
        } else if (r >= 12) {
            v += fw((r - 12) / 3, (r - 12) % 3);
        }
        sdd[r] = v;
    }
    if (t < 12) scw[t] = fw(t / 3, t % 3);
    wave_sync();
    // the AL terms of the touchdown legs only (a leg's coefficient is the same on every lane; the
    // others add exact zeros)
    bool use[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) use[l] = scoef[l][1] != 0.0;
    int r = t / NX, cidx = t % NX;  // entry e = t + TERM_TL j: (r, cidx) advance per step
    for (int e = t; e < ((HSDDP_TERM_EXP & 4) ? 0 : NN); e += TERM_TL) { // Phixx
        double v = 0.0;
        if (r == cidx)
            v = sdd[r];
        else if (r >= 3 && r < 6 && cidx >= 12 && (cidx - 12) % 3 == r - 3)
            v = -scw[cidx - 12];
        else if (cidx >= 3 && cidx < 6 && r >= 12 && (r - 12) % 3 == cidx - 3)
            v = -scw[r - 12];
#pragma unroll
        for (int l = 0; l < 4; ++l)
            if (use[l]) v += scoef[l][1] * (shx[l][r] * shx[l][cidx]);
        rec[TM_PHIXX + e] = v;
        // Px rows 12 .. 23 from LDS, stored coalesced (rows 0 .. 11 are the identity's, written once
        // for every record at create: launch_init_params)
        if (bnd && r >= 12) rec[TM_PX + e] = spx[(r - 12) * (NX + 1) + cidx];
        r += TERM_TL / NX;
        cidx += TERM_TL % NX;
        if (cidx >= NX) {
            cidx -= NX;
            r += 1;
        }
    }
}

// lu + ReB gradient / Hessian of one knot (SinglePhase.cpp:380-394); the GRF constraint values from
// the control row's forces, or the older ones ovr (constraint_forces)
DEV void lq_lu_reb(const Params &p, const int *c, const double *u, const double *ovr, const double *ur, const double *dl,
                   const double *ep, double *lu, double *rb)
{
#pragma unroll
    for (int j = 0; j < NU; ++j) lu[j] = p.dt * r_diag(p, j) * (u[j] - ur[j]);
#pragma unroll
    for (int j = 0; j < 24; ++j) rb[j] = 0.0;
    // uniform ReB parameters (the default schedule) and per-knot ones as separate code: in the
    // uniform case no per-row (delta, eps) load and no per-row 1 / delta division is issued
    auto reb = [&](auto uniform) {
        constexpr bool U = decltype(uniform)::value;
        const double inv_du = p.grf_inv_delta;
#pragma unroll
        for (int lg = 0; lg < 4; ++lg) {
            if (!c[lg]) continue;
            double gu[3] = {0, 0, 0}, hu[6] = {0, 0, 0, 0, 0, 0};
            const double f0 = grf_force(u, ovr, 3 * lg), f1 = grf_force(u, ovr, 3 * lg + 1), f2 = grf_force(u, ovr, 3 * lg + 2);
#pragma unroll
            for (int r = 0; r < 5; ++r) {
                double row[3], d1, d2;
                grf_row(p.mu, r, row);
                double g = row[0] * f0 + row[1] * f1 + row[2] * f2;
                const double dlr = U ? p.grf_delta : dl[5 * lg + r];
                reb_derivs(g, dlr, U ? inv_du : 1.0 / dlr, d1, d2);
                double e = U ? p.grf_eps : ep[5 * lg + r];
                for (int a = 0; a < 3; ++a) gu[a] += e * d1 * row[a];
                hu[0] += e * (d2 * row[0] * row[0]); hu[1] += e * (d2 * row[0] * row[1]);
                hu[2] += e * (d2 * row[0] * row[2]); hu[3] += e * (d2 * row[1] * row[1]);
                hu[4] += e * (d2 * row[1] * row[2]); hu[5] += e * (d2 * row[2] * row[2]);
            }
            for (int a = 0; a < 3; ++a) lu[3 * lg + a] += p.dt * gu[a];
            for (int a = 0; a < 6; ++a) rb[6 * lg + a] = p.dt * hu[a];
        }
    };
    if (p.ReB_active) {
        if (p.reb_uniform) reb(std::true_type{});
        else reb(std::false_type{});
    }
}

// One terminal wave: tasks (element, phase) TERM_TPW wave .. + TERM_TPW - 1 on S[0 ..]; the first
// wave also resets the iteration's counters (k_terminal's comment)
template <bool EL>
DEV void terminal_wave(const Params &p, const Bufs &d, TermLds *S, long wave, int lane)
{
    if (p.retry_cap > 0 && wave == 0 && lane == 0) *d.retry_count = 0;
    if (wave == 0)
        for (int t = lane; t < LS_LIVE; t += 64) d.ls_live[t] = 0;
    if (wave == 0 && lane < 4) d.counter[lane] = 0;
#if HSDDP_LQ_EXP == 1
    return;
#endif
    const int h = lane / TERM_TL;
    const long task = wave * TERM_TPW + h;
    if (task < (long)p.B * p.P) terminal_task<EL>(p, d, S[h], (int)task, lane % TERM_TL);
}

// ---------------------------------------------------------------------------------------------
// k_lq: per (element, state slot): cost and |Defect|^2 at the current (X, U); compact LQ model at
// control slots (SinglePhase::compute_cost + LQ_approximation, SinglePhase.cpp:235-296).
// F32: config C5's fp32 Riccati mode (records in fp32 plus an fp32 copy of Defect for the sweep)
// The A - I / B pieces go out by direct stores (staging them would keep all 102 values live).
// SLOTS: the slot costs and |Defect|^2 are recomputed (Params::lq_slots; instantiated apart so the
// common path keeps the registers the cost code would take)
template <bool F32, bool EL, bool SLOTS>
__global__ __launch_bounds__(256, FWD_MINB) void k_lq(Params p, Bufs d)
{
    using T = std::conditional_t<F32, float, double>;
    // the record stage of the knot waves, or the LDS of the terminal waves (blocks after them: small
    // batches, launch_lq)
    constexpr size_t STG = sizeof(T) * 4 * 64 * LQ_STG<T>, TRM = 4 * TERM_TPW * sizeof(TermLds);
    __shared__ __attribute__((aligned(16))) char lds[STG > TRM ? STG : TRM];
    T (*stage)[64 * LQ_STG<T>] = reinterpret_cast<T (*)[64 * LQ_STG<T>]>(lds);
    __shared__ long sridx[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // one thread per control knot (the records' own order); the modes that also have work at the
    // phase-end slots — |Defect|^2 (SLOTS), the fp32 Defect copy (F32) — one per state slot
    constexpr bool BY_KNOT = !SLOTS && !F32;
    const long nunit = (long)p.B * (BY_KNOT ? p.Kc : p.S);
    const long nknot = (nunit + 255) / 256;
    if ((long)blockIdx.x >= nknot) {
        terminal_wave<EL>(p, d, reinterpret_cast<TermLds *>(lds) + w * TERM_TPW, ((long)blockIdx.x - nknot) * 4 + w, lane);
        return;
    }
    sridx[w][lane] = -1; // before any early return: lanes without a record stay -1
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= nunit) return;
    const int b = (int)(gid / (BY_KNOT ? p.Kc : p.S));
    const ElemState &E = d.el[b];
    if (E.done || E.inner_done) return;
    const auto L = layout_of<EL>(d, b);
    int i, k, s;
    if constexpr (BY_KNOT) {
        const int kc0 = (int)(gid % p.Kc);
        knot_phase(L, kc0, i, k);
        if (k >= L.N(i)) return;  // (every layout has Kc knots: none past the last phase)
        s = L.s0(i) + k;
    } else {
        s = (int)(gid % p.S);
        if (s >= L.S()) return;
        slot_phase(L, s, i, k);
    }
    int c[4], cn[4];
    load_contacts(d, p, b, i, c, cn);
    double x[NX];
    const int wb = work_buf(d, b);
    const double *xg = xbuf(d, wb) + ((size_t)b * p.S + s) * NX;
#pragma unroll
    for (int j = 0; j < NX; ++j) x[j] = xg[j];
    const double *dg = dbuf(d, wb) + ((size_t)b * p.S + s) * NX;
    if (SLOTS) {  // |Defect|^2 (else the last rollout's, of this working trajectory)
        double fs = 0.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) fs += dg[j] * dg[j];
        d.slot_feas[(size_t)b * p.S + s] = fs;
    }
    if constexpr (F32) { // the sweep's and linear rollout's fp32 copy of Defect
        float *d32 = d.def32 + ((size_t)b * p.S + s) * NX;
#pragma unroll
        for (int j = 0; j < NX; ++j) d32[j] = (float)dg[j];
    }
    const double *xr = ref_ptr(p, d.ref_x, b, s, NX), *pf = ref_ptr(p, d.ref_foot, b, s, 12);
    if (k == L.N(i)) return;  // the terminal cost: the terminal task (the same function, from its foot heights)
    const int kc = L.k0(i) + k;
    sridx[w][lane] = (long)b * p.Kc + kc;
    double u[NU];
    const double *ug = ubuf(d, wb) + ((size_t)b * p.Kc + kc) * NU;
#pragma unroll
    for (int j = 0; j < NU; ++j) u[j] = ug[j];
    // the forces of the knot's stored GRF constraint values (older ones after a diverged trial)
    const double *ovr = constraint_forces(d, E, b, kc);
    const double *ur = ref_ptr(p, d.ref_u, b, s, NU);
    const double *dl = d.reb_delta + ((size_t)b * p.Kc + kc) * 20, *ep = d.reb_eps + ((size_t)b * p.Kc + kc) * 20;
    if (SLOTS) {  // the running cost (else the last rollout's: same trajectory, same parameters)
        double viol;
        d.slot_cost[(size_t)b * p.S + s] = running_cost(p, c, x, u, xr, ur, pf, dl, ep, viol, ovr);
    }

    // the record in the solver's Riccati precision (fp64, or fp32 in config C5's mode)
    T *lqT = F32 ? (T *)d.lq32 : (T *)d.lq;
    const int ldw = F32 ? LQW32 : LQW;
    double cd[4] = {(double)c[0], (double)c[1], (double)c[2], (double)c[3]};
    // A - I and B pieces (record positions 0 .. 103) in position order (hkd_partial_emit): each
    // value goes to this wave's LDS stage as it is computed and the stage is stored coalesced;
    // positions 15 and 67 are the record's zero slots.
    T *wl = stage[w];
    // The record leaves in 128-byte lines (W values): every line of a record is written once,
    // whole — a line written in two pieces at different times costs a second line write (PMC:
    // 7-11 % more WRITE_SIZE than the records; 0.47 -> 0.40 ms for lq + terminal when aligned).
    // Positions 0 .. 95 (A - I and B) in emission order, a line leaving with its last value;
    // positions 96 .. 103 (the last B values) then wait in the stage for lx, lu, the ReB Hessian
    // and (fp32: the record is 192 values, 6 lines) zero padding, put in position order.
    constexpr int W = 128 / (int)sizeof(T);
    auto col = [&](int pos) -> T & { return wl[lane * LQ_STG<T> + (pos & (W - 1))]; };
    auto put = [&](int pos, double v) {  // positions >= 96, in order
        col(pos) = (T)v;
        if ((pos & (W - 1)) == W - 1) lq_flush(wl, sridx[w], lqT, ldw, lane, pos - (W - 1), W);
    };
    col(15) = 0;
    hkd_partial_emit(x, u, cd, p.dt, [&](int piece, int j, double v) {
        const int pos = piece == 0 ? LQ_SE + j : piece == 1 ? sw_at(j / 17, j % 17) : bw_at(j / 12, j % 12);
        col(pos) = (T)v;
        // a line's last value (position 15 of the first fp64 line is a zero slot; 96 .. 103 wait)
        if (pos < 96 && ((pos & (W - 1)) == W - 1 || (W == 16 && pos == 14))) {
            lq_flush(wl, sridx[w], lqT, ldw, lane, pos & ~(W - 1), W);
            if (pos == 63) col(67) = 0;  // the line holding the second zero slot starts
        }
    });
    // lx: tracking + foot regularisation (HKDCost.cpp:22-37)
    {
        double lx[NX];
#pragma unroll
        for (int j = 0; j < NX; ++j) lx[j] = p.dt * q_diag(p, c, j) * (x[j] - xr[j]);
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            double e = (x[12 + j] - x[3 + j % 3]) - (pf[j] - xr[3 + j % 3]);
            double v = p.dt * c[j / 3] * foot_weight(p, c, j) * e;
            lx[3 + j % 3] += -v;
            lx[12 + j] += v;
        }
#pragma unroll
        for (int j = 0; j < NX; ++j) put(LQ_LX + j, lx[j]);
    }
    // lu + ReB gradient / Hessian (SinglePhase.cpp:380-394)
    double lu[NU], rb[24];
    lq_lu_reb(p, c, u, ovr, ur, dl, ep, lu, rb);
#pragma unroll
    for (int j = 0; j < NU; ++j) put(LQ_LU + j, lu[j]);
#pragma unroll
    for (int j = 0; j < 24; ++j) put(LQ_RB + j, rb[j]);
    if constexpr (F32)
#pragma unroll
        for (int j = LQW; j < LQW32; ++j) put(j, 0.0);
}

// ---------------------------------------------------------------------------------------------
// Per-slot outputs of one rollout trial from the slot's state x = X[k], simulated state xs =
// Xsim[k] and control u = U[k] (k < N): Defect, |Defect|^2, divergence flag, running or terminal
// cost with its constraint violation and touchdown residuals (SinglePhase.cpp:196-232).
// Defect = Xsim - X, its squared norm and the divergence flag of slot s
DEV void finish_defect(const Params &p, const Bufs &d, int b, int s, int k, const double *x, const double *xs)
{
    const size_t sb = (size_t)b * p.S;
    double nrm = 0.0, fs = 0.0;
    double *Dg = dbuf(d, trial_buf(d, b)) + (sb + s) * NX;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
        nrm += xs[j] * xs[j];
        const double df = xs[j] - x[j];
        fs += df * df;
#if HSDDP_RO_EXP == 1
        if (df == 12345.678) Dg[j] = df;
#else
        Dg[j] = df;
#endif
    }
    d.slot_feas[sb + s] = fs;
    d.slot_div[sb + s] = (k > 0 && sqrt(nrm) > 1e6) ? 1 : 0;
}

// the terminal cost of phase i at its last slot s (x = X[N]) with its violation and touchdown
// residuals; stored: with the constraints' stored residuals (a phase the rollout did not complete),
// else as a rollout completing the phase computes them
DEV void finish_terminal(const Params &p, const Bufs &d, int b, int s, int i, const int *c, const int *cn, const double *x,
                         bool stored = false)
{
    const size_t sb = (size_t)b * p.S;
    const double *xr = ref_ptr(p, d.ref_x, b, s, NX), *pf = ref_ptr(p, d.ref_foot, b, s, 12);
    double tv, h[4];
    const size_t q = ((size_t)b * p.P + i) * MTD;
    (void)cn;
    d.slot_cost[sb + s] = terminal_cost(p, c, x, xr, pf, d.td_mask + q, d.al_sigma + q * 4, d.al_lambda + q * 4, tv, h,
                                        stored);
    d.slot_viol[sb + s] = tv;
#pragma unroll
    for (int l = 0; l < 4; ++l) d.term_h[((size_t)b * p.P + i) * 4 + l] = h[l];
}

// the running cost of control slot kc = k0(i) + k at state slot s; COLS: the reference from the
// entry-major copy (Bufs::ref_t: lanes on consecutive slots read contiguous pieces)
template <bool COLS = false>
DEV void finish_running(const Params &p, const Bufs &d, int b, int s, int kc, const int *c, const double *x, const double *u)
{
    if constexpr (COLS) {
        const double *dl = d.reb_delta + ((size_t)b * p.Kc + kc) * 20, *ep = d.reb_eps + ((size_t)b * p.Kc + kc) * 20;
#if HSDDP_RO_STAGED
        // the reference in two pieces, so that the 60 values are never live at once: the control
        // reference first (the ReB term, which needs none, covers its loads), then the state and
        // foot references
        typedef double d2 __attribute__((ext_vector_type(2)));
        const size_t r = (size_t)(p.ref_per_element ? b : 0) * p.S + s, w = d.ref_tw;
        const d2 *col = (const d2 *)d.ref_t + r;
        double lu, mk, rc;
        {
            d2 v[NU / 2];
#pragma unroll
            for (int j = 0; j < NU / 2; ++j) v[j] = col[(NX / 2 + j) * w];
            rc = cost_reb(p, c, u, dl, ep, mk, nullptr);
            double urv[NU];
#pragma unroll
            for (int j = 0; j < NU / 2; ++j) { urv[2 * j] = v[j].x; urv[2 * j + 1] = v[j].y; }
            lu = cost_control(p, u, urv);
        }
        __builtin_amdgcn_sched_barrier(0);
        double lt, lf;
        {
            d2 v[(NX + 12) / 2];
#pragma unroll
            for (int j = 0; j < NX / 2; ++j) v[j] = col[j * w];
#pragma unroll
            for (int j = 0; j < 6; ++j) v[NX / 2 + j] = col[((NX + NU) / 2 + j) * w];
            double xrv[NX], pfv[12];
#pragma unroll
            for (int j = 0; j < NX / 2; ++j) { xrv[2 * j] = v[j].x; xrv[2 * j + 1] = v[j].y; }
#pragma unroll
            for (int j = 0; j < 6; ++j) { pfv[2 * j] = v[NX / 2 + j].x; pfv[2 * j + 1] = v[NX / 2 + j].y; }
            lt = cost_tracking(p, c, x, xrv);
            lf = cost_foot(p, c, x, xrv, pfv);
        }
        d.slot_cost[(size_t)b * p.S + s] = cost_combine(p, c, lt, lu, lf, rc);
        d.slot_viol[(size_t)b * p.S + s] = mk;
#else
        alignas(16) double xr[NX], ur[NU], pf[12];
        ref_from_cols(p, d, b, s, xr, ur, pf);
        double viol;
        d.slot_cost[(size_t)b * p.S + s] = running_cost(p, c, x, u, xr, ur, pf, dl, ep, viol);
        d.slot_viol[(size_t)b * p.S + s] = viol;
#endif
        return;
    }
    const size_t sb = (size_t)b * p.S;
#if HSDDP_RO_EXP == 3
    d.slot_cost[sb + s] = x[0];  // timing only: no running cost
    d.slot_viol[sb + s] = u[0];
    return;
#endif
#if HSDDP_RO_EXP == 4
    const double *xr = x, *pf = x + 12, *ur = u;  // timing only: the cost without its reference loads
#else
    const double *xr = ref_ptr(p, d.ref_x, b, s, NX), *pf = ref_ptr(p, d.ref_foot, b, s, 12);
    const double *ur = ref_ptr(p, d.ref_u, b, s, NU);
#endif
    const double *dl = d.reb_delta + ((size_t)b * p.Kc + kc) * 20, *ep = d.reb_eps + ((size_t)b * p.Kc + kc) * 20;
    double viol;
    d.slot_cost[sb + s] = running_cost(p, c, x, u, xr, ur, pf, dl, ep, viol);
    d.slot_viol[sb + s] = viol;
}

template <typename L_>
DEV void finish_slot(const Params &p, const Bufs &d, const L_ &L, int b, int s, int i, int k, const int *c,
                     const int *cn, const double *x, const double *xs, const double *u)
{
    finish_defect(p, d, b, s, k, x, xs);
    if (k == L.N(i))
        finish_terminal(p, d, b, s, i, c, cn, x);
    else
        finish_running(p, d, b, s, L.k0(i) + k, c, x, u);
}

// trial tix > 0 of an inner iteration runs only when an element is still searching after trial
// tix - 1 (Bufs::ls_live, written by the previous launch; a batch with none left returns at once)
DEV bool ls_skip(const Bufs &d, int tix)
{
    if (tix <= 0 || tix > LS_LIVE) return false;
    return __builtin_amdgcn_readfirstlane(d.ls_live[tix - 1]) == 0;
}

// k_rollout: one line-search trial (eps) per (element, state slot).  All knots are shooting states
// (HKDProblem.cpp:104), so X[k] = Xbar[k] + eps dX[k] and the simulated state at k depends only on
// knot k-1: the nonlinear rollout is knot-parallel.  U = Ubar + eps du with du = dU + K dX from the
// linear rollout (equal to the reference's Ubar + eps dU + K (X - Xbar) up to rounding of X - Xbar).
//
// One wave per 64 consecutive slots.  The trial state rows it needs (its slots and the one before)
// are formed with coalesced 16-byte loads (lanes over row entries, not rows) into LDS — the output
// X rows are stored from the same pass — and each lane then reads its rows from LDS.
constexpr int RS = NX + 1;  // LDS row stride (doubles): conflict-free row-per-lane reads

// The trial's steps b + eps v.  dX, du and dU are not reset between solves (hsddp_update_problem),
// as the reference keeps its own from tick to tick: the initial rollout (eps = 0) multiplies them
// by 0 as the reference does (SinglePhase.cpp:189, 200, 216).  (A select that skipped them at
// eps = 0 cost the metric's trials 7 %: k_rollout 148.8 -> 159.7 us.)
DEV double fma_step(double eps, double v, double b) { return __builtin_fma(eps, v, b); }
DEV double add_step(double b, double eps, double v) { return b + eps * v; }
constexpr int RW = 65;      // rows per wave: 64 slots and the one before

// X_t = Xbar + eps dX for rows r0 .. r0 + RW - 1 of the [rows][24] state buffers into LDS; rows
// of inactive elements are skipped, own rows (own(r)) are stored to the element's trial buffer
// (selof(element): the element's Bufs::sel, nominal and working buffer indices)
template <typename Act, typename Own, typename Sel>
DEV void stage_trial(double *L, const Bufs &d, const double *del, long r0, long nrows, int per, double eps,
                     int lane, Act active, Own own, Sel selof)
{
    constexpr int CH = NX / 2;  // 16-byte chunks per row
#pragma unroll 1
    for (int f = lane; f < RW * CH; f += 64) {
        const int row = f / CH, cc = 2 * (f % CH);
        const long r = r0 + row;
        if (r < 0 || r >= nrows || !active((int)(r / per))) continue;
        const int q = selof((int)(r / per));
        const double *bar = xbuf(d, q & 3);
        double *out = xbuf(d, trial_of(q & 3, (q >> 2) & 3));
        typedef double d2 __attribute__((ext_vector_type(2)));
        const d2 xb = *(const d2 *)(bar + r * NX + cc), dx = *(const d2 *)(del + r * NX + cc);
        d2 v;
        v.x = fma_step(eps, dx.x, xb.x);
        v.y = fma_step(eps, dx.y, xb.y);
        L[row * RS + cc] = v.x;
        L[row * RS + cc + 1] = v.y;
        if (own(r)) *(d2 *)(out + r * NX + cc) = v;
    }
}

// The same for per >= RW: the wave's 64 slots belong to its elements bA and bB, whose activity and
// nominal buffers are known (no per-row lookups), and the loads of all chunks are issued before any
// is used.  Row r0 may be the previous element's last slot: no slot of this wave reads it (slot 0
// of an element starts from x0 or a reset map of its own rows), so it is skipped.  Rows of
// inactive elements are read (in range, harmless) but neither staged nor stored.
DEV void stage_trial2(double *L, const Bufs &d, long r0, long nrows, int per, double eps, int lane, long g0, int bA,
                      bool aA, int nA, int tA, int bB, bool aB, int nB, int tB)
{
    constexpr int CH = NX / 2, NIT = (RW * CH + 63) / 64;
    typedef double d2 __attribute__((ext_vector_type(2)));
    // the elements' nominal (read) and trial (written) buffers
    const double *barA = kxbuf(nA), *barB = kxbuf(nB), *del = d.dX;
    double *outA = kxbuf(tA), *outB = kxbuf(tB);
    d2 xb[NIT], dx[NIT];
    long rr[NIT];
    bool use[NIT];
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        const int f = lane + 64 * it, row = f / CH, cc = 2 * (f % CH);
        const long r = r0 + row;
        const bool in = f < RW * CH && r >= 0 && r < nrows;
        const long rc = in ? r : (r0 + 1 > 0 ? r0 + 1 : 0);  // a valid row for out-of-range chunks
        const long eb = rc / per;
        const bool first = eb == bA;
        use[it] = in && (first ? aA : eb == bB && aB);
        rr[it] = rc;
        xb[it] = *(const d2 *)((first ? barA : barB) + rc * NX + cc);
        dx[it] = *(const d2 *)(del + rc * NX + cc);
    }
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
        if (!use[it]) continue;
        const int f = lane + 64 * it, row = f / CH, cc = 2 * (f % CH);
        const long r = rr[it];
        d2 v;  // Xbar + eps dX as one rounding (rollout_boundary forms the same rows)
        v.x = fma_step(eps, dx[it].x, xb[it].x);
        v.y = fma_step(eps, dx[it].y, xb[it].y);
        L[row * RS + cc] = v.x;
        L[row * RS + cc + 1] = v.y;
        const bool first = r / per == bA;
        if (r >= g0) *(d2 *)((first ? outA : outB) + r * NX + cc) = v;
    }
}

#ifndef HSDDP_RO_REVERSE
#define HSDDP_RO_REVERSE 1
#endif
#ifndef HSDDP_RO_STAGED
#define HSDDP_RO_STAGED 1  // the slot waves' reference loaded in two pieces (0: all 30 pairs at once)
#endif
#ifndef HSDDP_RO_COLS
#define HSDDP_RO_COLS 1  // the slot waves' reference reads from Bufs::ref_t (0: from the rows)
#endif

#ifndef HSDDP_ROLLOUT_WAVES
#define HSDDP_ROLLOUT_WAVES 2  // measured: 2 (256 VGPRs, no spills) 0.93 ms/step forward vs 3: 1.23, 4: 1.07
#endif

// trial control row r: U = Ubar + eps du, straight from global memory (the wave's 64 rows are one
// contiguous 12 KB range, so the row-per-lane loads are served by the vector L1 / L2)
DEV void trial_row(const Bufs &d, const double *Ubar, long r, double eps, double *u)
{
    typedef double d2 __attribute__((ext_vector_type(2)));
    const d2 *ub = (const d2 *)(Ubar + r * NU), *du = (const d2 *)(d.du + r * NU);
#pragma unroll
    for (int j = 0; j < NU / 2; ++j) {
        const d2 a = ub[j], e = du[j];
        u[2 * j] = add_step(a.x, eps, e.x);
        u[2 * j + 1] = add_step(a.y, eps, e.y);
    }
}

// v of the previous lane of the wave (DPP wave_shr:1; lane 0 gets 0).  Every lane must be active.
DEV double from_prev_lane(double v)
{
    const unsigned lo = __builtin_amdgcn_update_dpp(0u, (unsigned)__double2loint(v), 0x138, 0xf, 0xf, false);
    const unsigned hi = __builtin_amdgcn_update_dpp(0u, (unsigned)__double2hiint(v), 0x138, 0xf, 0xf, false);
    return __hiloint2double((int)hi, (int)lo);
}

// Only the state rows go through LDS (13 KB per wave); the control rows are read per lane
// (trial_row), the slot's own control row stored from registers.  With both row sets in LDS
// (26 KB per wave) only 6 waves fit a CU: 1.25 ms/step of line search vs 0.93 here.
// The phase-boundary work of one trial, one thread per (phase i, element b), i-major so that a
// wave's threads share a phase (and, in a shared-gait batch, its contacts: no divergence): the
// reset map into the phase's first slot (MultiPhaseDDP.cpp:73-81) with that slot's Defect, and the
// terminal cost at its last slot.  These run in waves of their own: inside the slot waves, a
// lane's reset map or terminal cost (foot kinematics) stalled its 63 neighbours.
template <bool EL>
DEV void rollout_boundary(const Params &p, const Bufs &d, double eps, int init, long t)
{
    if (t >= (long)p.B * p.P) return;
    const int i = (int)(t / p.B), b = (int)(t % p.B);
    const ElemState &E = d.el[b];
    if (!(init ? !E.done : E.ls_active != 0)) return;
    const auto L = layout_of<EL>(d, b);
    if (i >= L.P()) return;
    const int nb = nom_buf(d, b), s0 = L.s0(i), sN = s0 + L.N(i);
    const double *Xbar = xbuf(d, nb);
    const size_t sb = (size_t)b * p.S;
    // trial rows X = Xbar + eps dX (the slot waves' expression: the same values)
    auto trial = [&](int s, double *x) {
        const double *xb = Xbar + (sb + s) * NX, *dx = d.dX + (sb + s) * NX;
#pragma unroll
        for (int j = 0; j < NX; ++j) x[j] = fma_step(eps, dx[j], xb[j]);
    };
    int c[4], cn[4];
    load_contacts(d, p, b, i, c, cn);
    double x[NX];
    if (i > 0) {
        double xp[NX], xs[NX];
        int cp_[4], cpn[4];
        load_contacts(d, p, b, i - 1, cp_, cpn);
        trial(s0 - 1, xp);
        trial(s0, x);
        hkd_resetmap(xp, cp_, cpn, xs);
        finish_defect(p, d, b, s0, 0, x, xs);
    }
    trial(sN, x);
    finish_terminal(p, d, b, sN, i, c, cn, x);
}

// WIDE: p.S >= RW (instantiated apart: a wave's 64 slots then belong to at most two elements, and
// the kernel carries only that staging path)
template <bool EL, bool WIDE>
DEV void rollout_block(const Params &p, const Bufs &d, double eps, int init, int tix)
{
    __shared__ double Xt[RW * RS];
    const int lane = threadIdx.x;
    const long total = (long)p.B * p.S;
    const long nslot = (total + 63) / 64;
    if ((long)blockIdx.x >= nslot) {  // the phase-boundary waves (after the slot waves)
        rollout_boundary<EL>(p, d, eps, init, ((long)blockIdx.x - nslot) * 64 + lane);
        return;
    }
    // (HSDDP_RO_REVERSE: every second trial walks the slot blocks from the batch's end, where the
    // trial before's last reads of the same rows may still sit in the memory-side cache)
    const long blk = (HSDDP_RO_REVERSE && tix > 0 && (tix & 1)) ? nslot - 1 - (long)blockIdx.x : (long)blockIdx.x;
#if HSDDP_STAMPS
    unsigned long long rst[8];
#endif
    RSTAMP(0);
    const long g0 = blk * 64, gid = g0 + lane;
    const long gl = min(g0 + 63, total - 1);
    const int bA = (int)(g0 / p.S), bB = (int)(gl / p.S);
    auto act = [&](int b) { const ElemState &E = d.el[b]; return init ? !E.done : E.ls_active != 0; };
    const bool aA = act(bA), aB = act(bB);
    bool any = aA || aB;
    for (int b = bA + 1; b < bB && !any; ++b) any = act(b);
    if (!any) return;
    auto active = [&](int b) { return b == bA ? aA : b == bB ? aB : act(b); };
    const int qA = d.sel[bA], qB = d.sel[bB];
    const int nA = qA & 3, nB = qB & 3, tA = trial_of(nA, (qA >> 2) & 3), tB = trial_of(nB, (qB >> 2) & 3);
    auto selof = [&](int b) { return b == bA ? qA : b == bB ? qB : d.sel[b]; };
    auto nomof = [&](int b) { return selof(b) & 3; };
    auto trialof = [&](int b) { const int q = selof(b); return trial_of(q & 3, (q >> 2) & 3); };
    // the control row before the wave's first slot (that slot's u_prev; every other slot takes its
    // u_prev from the previous lane): lanes 0..11 load it with the state rows, stage it after them
    typedef double d2 __attribute__((ext_vector_type(2)));
    __shared__ double Up0[NU];
    d2 ua = {0, 0}, ue = {0, 0};
    bool up0 = false;
    {
        const int s0 = (int)(g0 % p.S);
        const auto L0 = layout_of<EL>(d, bA);
        int i0, k0;
        slot_phase(L0, s0, i0, k0);
        up0 = aA && s0 < L0.S() && k0 > 0 && lane < NU / 2;
        if (up0) {
            const long r = (long)bA * p.Kc + s0 - i0 - 1;
            ua = ((const d2 *)(kubuf(nA) + r * NU))[lane];
            ue = ((const d2 *)(d.du + r * NU))[lane];
        }
    }
    // every lane stays active up to the u_prev exchange: lanes without a slot of their own work on a
    // valid one (clamped) and write nothing
    const long gc = gid < total ? gid : total - 1;
    const int b = (int)(gc / p.S), s = (int)(gc % p.S);
    const auto L = layout_of<EL>(d, b);
    const bool mine = gid < total && active(b) && s < L.S();
    int i, k;
    slot_phase(L, s < L.S() ? s : L.S() - 1, i, k);
    const int nb = nomof(b), tb = trialof(b);
    const long kq = (long)b * p.Kc + s - i;  // the slot's control row (k < N)
    const long kqmax = (long)p.B * p.Kc - 1;
    const long kqr = kq < kqmax ? kq : kqmax;  // (the terminal slot's row index is clamped and unused)
    RSTAMP(1);
    const long xr0 = g0 - 1;
    if constexpr (WIDE)
        stage_trial2(Xt, d, xr0, total, p.S, eps, lane, g0, bA, aA, nA, tA, bB, aB, nB, tB);
    else
        stage_trial(Xt, d, d.dX, xr0, total, p.S, eps, lane, active, [&](long r) { return r >= g0; }, selof);
    if (up0) {
        Up0[2 * lane] = add_step(ua.x, eps, ue.x);
        Up0[2 * lane + 1] = add_step(ua.y, eps, ue.y);
    }
    __syncthreads();
    RSTAMP(2);
    int c[4], cn[4];
    load_contacts(d, p, b, i, c, cn);
    const double *x = Xt + (gc - xr0) * RS;
    // the trial control row of the slot, U = Ubar + eps du (k < N)
    double u[NU];
#if HSDDP_RO_EXP == 5
    for (int j = 0; j < NU; ++j) u[j] = x[j] * eps;  // timing only: no control-row loads
#else
    trial_row(d, kubuf(nb), kqr, eps, u);
#endif
#if HSDDP_STAMPS
    asm volatile("" : "+v"(u[0]), "+v"(u[NU - 1]));
#endif
    RSTAMP(3);
    // the running cost of a control slot (the terminal cost at k = N: the boundary waves)
    if (mine && k < L.N(i)) {
        d2 *ug = (d2 *)(kubuf(tb) + kq * NU);
#if HSDDP_RO_EXP == 2 || HSDDP_RO_EXP == 5
        if (u[0] == 12345.678)
#endif
#pragma unroll
        for (int j = 0; j < NU / 2; ++j) ug[j] = d2{u[2 * j], u[2 * j + 1]};
        finish_running<HSDDP_RO_COLS>(p, d, b, s, L.k0(i) + k, c, x, u);
    }
    RSTAMP(4);
    // u_prev: the previous slot's control row is the previous lane's (k > 0: slot s - 1 is a
    // control slot of the same phase), lane 0's was staged
    double up[NU];
#pragma unroll
    for (int j = 0; j < NU; ++j) up[j] = from_prev_lane(u[j]);
    if (lane == 0)
#pragma unroll
        for (int j = 0; j < NU; ++j) up[j] = Up0[j];
    // Defect rows through LDS: each slot's row replaces its own staged state row once every lane's
    // dynamics have read theirs, then the wave stores the 64 rows as one contiguous range (16-byte
    // pieces over lanes) instead of one row per lane
    __shared__ int wflag[64];
    const bool wr = mine && (k > 0 || i == 0);
    if (wr) {
        double xs[NX];
        if (k == 0) {
#pragma unroll
            for (int j = 0; j < NX; ++j) xs[j] = d.x0[(size_t)b * NX + j];
        } else {
            double cd[4] = {(double)c[0], (double)c[1], (double)c[2], (double)c[3]};
            hkd_step(x - RS, up, cd, p.dt, xs);
        }
        wave_sync();  // (no lane writes a row before every lane's dynamics have read the previous one)
        double *xw = Xt + (gc - xr0) * RS;
        double nrm = 0.0, fs = 0.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            nrm += xs[j] * xs[j];
            const double df = xs[j] - xw[j];
            fs += df * df;
            xw[j] = df;
        }
        const size_t q = (size_t)b * p.S + s;
        d.slot_feas[q] = fs;
        d.slot_div[q] = (k > 0 && sqrt(nrm) > 1e6) ? 1 : 0;
    } else {
        wave_sync();
    }
    RSTAMP(5);
    wflag[lane] = wr;
    const int rsplit = (int)((long)bB * p.S - g0);  // (WIDE) rows from here on are element bB's
    double *const DtA = kdbuf(tA), *const DtB = kdbuf(tB);
    wave_sync();
    typedef double d2 __attribute__((ext_vector_type(2)));
    constexpr int CH = NX / 2;
#pragma unroll 4
    for (int f = lane; f < 64 * CH; f += 64) {
        const int row = f / CH, cc = 2 * (f % CH);
        if (wflag[row]) {
            const double *src = Xt + (row + 1) * RS + cc;
            // the row's element's trial buffer (bA below rsplit, bB from it; horizons shorter than a
            // wave: the row's own element)
            double *Dt;
            if constexpr (WIDE) Dt = row >= rsplit ? DtB : DtA;
            else Dt = kdbuf(trialof((int)((g0 + row) / p.S)));
            *(d2 *)(Dt + (g0 + row) * NX + cc) = d2{src[0], src[1]};
        }
    }
#if HSDDP_STAMPS
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    RSTAMP(6);
    if (lane == 0) {
        unsigned long long *acc = (unsigned long long *)d.dbg;
        const int slot[7] = {12, 13, 14, 15, 16, 17, 18};  // element 0: 12 .. 15, element 1: 0 .. 2
#pragma unroll
        for (int n = 1; n <= 6; ++n) atomicAdd(acc + slot[n - 1], rst[n] - rst[n - 1]);
        atomicAdd(acc + 19, 1ull);  // waves
    }
#endif
}

// k_rollout_tail: the non-shooting states of a phase (k >= ss; HKDProblem::update leaves a new
// last phase of horizon <= 2 without shooting states) after k_rollout has handled the rest:
// SinglePhase::hybrid_rollout's sequential branch (SinglePhase.cpp:185-222), X[k] = Xsim[k]
// (X[0] = x_init when the set is empty) and U[k] = Ubar[k] + eps dU[k] + K[k] (X[k] - Xbar[k]),
// then the slot outputs of those states.  One thread per element; rare (a few states per element).
template <bool EL>
__global__ __launch_bounds__(64) void k_rollout_tail(Params p, Bufs d, double eps, int init, int tix)
{
    if (ls_skip(d, tix)) return;
    const int b = blockIdx.x * 64 + threadIdx.x;
    if (b >= p.B) return;
    const ElemState &E = d.el[b];
    if (!(init ? !E.done : E.ls_active != 0)) return;
    const size_t sb = (size_t)b * p.S, kb = (size_t)b * p.Kc;
    const auto L = layout_of<EL>(d, b);
    const int nb = nom_buf(d, b), tb = trial_buf(d, b);
    const double *Xbar = xbuf(d, nb), *Ubar = ubuf(d, nb);
    double *X = xbuf(d, tb), *U = ubuf(d, tb);  // the trial's rows (k_rollout wrote the shooting ones)
    for (int i = 0; i < L.P(); ++i) {
        const int N = L.N(i), ss = L.ss(i), s0 = L.s0(i), k0 = L.k0(i);
        if (ss >= N + 1) continue;
        int c[4], cn[4];
        load_contacts(d, p, b, i, c, cn);
        const double cd[4] = {(double)c[0], (double)c[1], (double)c[2], (double)c[3]};
        double x[NX], xs[NX], u[NU];
        if (ss == 0) { // X[0] = Xsim[0] = x_init (MultiPhaseDDP.cpp:73-81)
            if (i == 0) {
                for (int j = 0; j < NX; ++j) xs[j] = d.x0[(size_t)b * NX + j];
            } else {
                int cp_[4], cpn[4];
                load_contacts(d, p, b, i - 1, cp_, cpn);
                hkd_resetmap(X + (sb + s0 - 1) * NX, cp_, cpn, xs);
            }
        } else { // Xsim[ss] from the last shooting state and its control (written by k_rollout)
            const double *xg = X + (sb + s0 + ss - 1) * NX, *ug = U + (kb + k0 + ss - 1) * NU;
            for (int j = 0; j < NX; ++j) x[j] = xg[j];
            for (int j = 0; j < NU; ++j) u[j] = ug[j];
            hkd_step(x, u, cd, p.dt, xs);
        }
        for (int k = ss; k <= N; ++k) {
            const int s = s0 + k;
            double *xg = X + (sb + s) * NX;
            for (int j = 0; j < NX; ++j) { x[j] = xs[j]; xg[j] = xs[j]; }
            const double *up = nullptr;
            if (k < N) {
                const int kc = k0 + k;
                const double *xb = Xbar + (sb + s) * NX, *ub = Ubar + (kb + kc) * NU, *du = d.dU + (kb + kc) * NU;
                double dx[NX];
                for (int j = 0; j < NX; ++j) dx[j] = x[j] - xb[j];
                for (int j = 0; j < NU; ++j) u[j] = 0.0;
                // K (X - Xbar) from the 12 coupled gain rows (KCW layout; the other rows are zero)
                for (int q = 0; q < 12; ++q) {
                    const size_t kr = ((kb + kc) * 12 + q) * NX;
                    double acc = 0.0;
                    for (int j = 0; j < NX; ++j) acc += (p.fp32 ? (double)d.K32[kr + j] : d.K[kr + j]) * dx[j];
                    u[c[q / 3] ? q : 12 + q] = acc;
                }
                double *ug = U + (kb + kc) * NU;
                for (int j = 0; j < NU; ++j) { u[j] = add_step(ub[j], eps, du[j]) + u[j]; ug[j] = u[j]; }
                up = u;
            }
            finish_slot(p, d, L, b, s, i, k, c, cn, x, xs, up);
            if (k < N) hkd_step(x, u, cd, p.dt, xs);
        }
    }
}

// k_rollout_ss: one trial with single shooting (HSDDP_OPTION::MS = false).  SinglePhase::
// hybrid_rollout (SinglePhase.cpp:181-233) then takes X[k+1] = Xsim[k+1] at every knot whatever
// SS_set says (:214-220); only a phase's first state stays a shooting state when its set holds 0
// (:187-193): X[0] = Xbar[0] + eps dX[0] (dX is not written without the linear rollout,
// MultiPhaseDDP.cpp:326-329, so it keeps its last values), else X[0] = x_init.  So phases that start
// from a shooting state are independent: one thread per (element, phase), 16 per element (four
// elements per 64-thread block), each simulating its phase's knots one after another.  Then, after
// the block's barrier, the phase-start Defects (Xsim[0] = x_init: x0 or the reset map of the
// previous phase's X[N], MultiPhaseDDP.cpp:73-81) and the phases without shooting states (a new
// last phase of <= 2 knots after a receding-horizon shift), which start from that reset map.
template <bool EL>
DEV void ss_phase(const Params &p, const Bufs &d, int b, int i, double eps, const double *x_init)
{
    const auto L = layout_of<EL>(d, b);
    const size_t sb = (size_t)b * p.S, kb = (size_t)b * p.Kc;
    const int nb = nom_buf(d, b), tb = trial_buf(d, b);
    const double *Xbar = xbuf(d, nb), *Ubar = ubuf(d, nb);
    double *X = xbuf(d, tb), *U = ubuf(d, tb);
    const int N = L.N(i), s0 = L.s0(i), k0 = L.k0(i);
    int c[4], cn[4];
    load_contacts(d, p, b, i, c, cn);
    const double cd[4] = {(double)c[0], (double)c[1], (double)c[2], (double)c[3]};
    double x[NX], xs[NX], u[NU];
    if (x_init) {  // no shooting state: X[0] = x_init (Defect[0] = 0)
        for (int j = 0; j < NX; ++j) x[j] = x_init[j];
    } else {       // X[0] = Xbar[0] + eps dX[0] (k_rollout's expression)
        const double *xb = Xbar + (sb + s0) * NX, *dx = d.dX + (sb + s0) * NX;
        for (int j = 0; j < NX; ++j) x[j] = fma_step(eps, dx[j], xb[j]);
    }
    for (int k = 0; k <= N; ++k) {
        const int s = s0 + k;
        double *xg = X + (sb + s) * NX;
        if (k > 0)
            for (int j = 0; j < NX; ++j) x[j] = xs[j];
        for (int j = 0; j < NX; ++j) xg[j] = x[j];
        if (k > 0 || x_init) finish_defect(p, d, b, s, k, x, k > 0 ? xs : x);
        if (k == N) {
            finish_terminal(p, d, b, s, i, c, cn, x);
            break;
        }
        // U = Ubar + eps dU + K (X - Xbar) (SinglePhase.cpp:200), K from the 12 coupled gain rows
        const int kc = k0 + k;
        const double *xb = Xbar + (sb + s) * NX, *ub = Ubar + (kb + kc) * NU, *du = d.dU + (kb + kc) * NU;
        double dx[NX];
        for (int j = 0; j < NX; ++j) dx[j] = x[j] - xb[j];
        for (int j = 0; j < NU; ++j) u[j] = 0.0;
        for (int q = 0; q < 12; ++q) {
            const size_t kr = ((kb + kc) * 12 + q) * NX;
            double acc = 0.0;
            for (int j = 0; j < NX; ++j) acc += (p.fp32 ? (double)d.K32[kr + j] : d.K[kr + j]) * dx[j];
            u[c[q / 3] ? q : 12 + q] = acc;
        }
        double *ug = U + (kb + kc) * NU;
        for (int j = 0; j < NU; ++j) { u[j] = add_step(ub[j], eps, du[j]) + u[j]; ug[j] = u[j]; }
        finish_running(p, d, b, s, kc, c, x, u);
        hkd_step(x, u, cd, p.dt, xs);
    }
}

template <bool EL>
__global__ __launch_bounds__(64) void k_rollout_ss(Params p, Bufs d, double eps, int init, int tix)
{
    if (ls_skip(d, tix)) return;
    const int b = blockIdx.x * 4 + (threadIdx.x >> 4), i = threadIdx.x & 15;
    bool mine = false, shoot = false;
    if (b < p.B) {
        const ElemState &E = d.el[b];
        const auto L = layout_of<EL>(d, b);
        mine = (init ? !E.done : E.ls_active != 0) && i < L.P();
        shoot = mine && L.ss(i) > 0;
    }
    if (shoot) ss_phase<EL>(p, d, b, i, eps, nullptr);
    __syncthreads();  // every phase's X[N] written (same block)
    if (!mine) return;
    const auto L = layout_of<EL>(d, b);
    const size_t sb = (size_t)b * p.S;
    const int s0 = L.s0(i);
    const double *X = xbuf(d, trial_buf(d, b));
    double xi[NX];
    if (i == 0) {
        for (int j = 0; j < NX; ++j) xi[j] = d.x0[(size_t)b * NX + j];
    } else {
        int cp_[4], cpn[4];
        load_contacts(d, p, b, i - 1, cp_, cpn);
        hkd_resetmap(X + (sb + s0 - 1) * NX, cp_, cpn, xi);
    }
    if (shoot) {
        double x[NX];
        for (int j = 0; j < NX; ++j) x[j] = X[(sb + s0) * NX + j];
        finish_defect(p, d, b, s0, 0, x, xi);
    } else {
        ss_phase<EL>(p, d, b, i, eps, xi);
    }
}

// A trial whose rollout breaks the 1e6 bound (SinglePhase::hybrid_rollout, SinglePhase.cpp:205-208)
// first at state slot sbrk (= s0_i + k + 1: the state simulated from knot k of phase i): the
// reference returns there and skips every later phase (MultiPhaseDDP.cpp:83-87), so X past the
// break state, U past knot k and the Defect of phase i on keep the working rows of before the
// trial, the GRF constraint values of knot k stay those of its earlier control row, and the cost
// and feasibility that follow (:116-117) are sums over those mixed rows.  The slot kernels computed
// every slot; here the element's 16 lanes (g) copy the working rows the reference keeps into the
// trial buffer, update the stored GRF values' table (Bufs::cf_flag / cf_u: the knots before the
// break now hold the trial's values, the break knot keeps its earlier ones, the later knots are
// untouched) and recompute the slot outputs from the break knot on.  No cross-lane operation (the
// caller's lanes diverge).
template <bool EL>
DEV void diverged_fixup(const Params &p, const Bufs &d, const LayT<EL> &L, int b, int g, int sbrk)
{
    int i, ks;
    slot_phase(L, sbrk, i, ks);
    const int kb = ks - 1, s0 = L.s0(i), kcb = L.k0(i) + kb, sbb = s0 + kb, S = L.S();
    const int q = d.sel[b], nb = q & 3, wb = (q >> 2) & 3, tb = trial_of(nb, wb);
    const size_t sb = (size_t)b * p.S, kq = (size_t)b * p.Kc;
    double *XT = xbuf(d, tb), *UT = ubuf(d, tb), *DT = dbuf(d, tb);
    const double *XW = xbuf(d, wb), *UW = ubuf(d, wb), *DW = dbuf(d, wb);
    for (long e = g; e < (long)(S - sbrk) * NX; e += 16) XT[(sb + sbrk) * NX + e] = XW[(sb + sbrk) * NX + e];
    for (long e = g; e < (long)(p.Kc - kcb - 1) * NX; e += 16) UT[(kq + kcb + 1) * NX + e] = UW[(kq + kcb + 1) * NX + e];
    for (long e = g; e < (long)(S - s0) * NX; e += 16) DT[(sb + s0) * NX + e] = DW[(sb + s0) * NX + e];
    int c[4], cn[4];
    load_contacts(d, p, b, i, c, cn);
    ElemState &E = d.el[b];
    // the knots before the break were passed: their stored values are the trial's (flags cleared);
    // the break knot's stay what they were — the forces of its entry if it has one, else those of
    // its working control row (the one U[kcb] held before this trial), which becomes its entry
    int *cf = d.cf_flag + kq;
    // (while E.ovr is 0 the flags are not read and their contents are arbitrary: cleared here first)
    for (int kc = g; kc < (E.ovr ? kcb : p.Kc); kc += 16)
        if (kc != kcb) cf[kc] = 0;  // (lane 0 writes the break knot's)
    if (g == 0) {
        if (!(E.ovr && cf[kcb])) {
            for (int r = 0; r < 12; ++r) d.cf_u[(kq + kcb) * 12 + r] = UW[(kq + kcb) * NX + r];
            cf[kcb] = 1;
        }
        E.ovr = 1;
    }
    __threadfence();  // rows and table visible to the other lanes of the element
    // slot outputs over the mixed rows: |Defect|^2 of phase i on, costs from the break knot on
    int ip = i;
#pragma unroll 1
    for (int s = s0 + g; s < S; s += 16) {
        while (ip + 1 < L.P() && s >= L.s0(ip + 1)) ++ip;
        const int k = s - L.s0(ip);
        const double *dr = DT + (sb + s) * NX;
        double fs = 0.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) fs += dr[j] * dr[j];
        d.slot_feas[sb + s] = fs;
        d.slot_div[sb + s] = 0;
        if (s < sbb) continue;
        load_contacts(d, p, b, ip, c, cn);
        // (rows read in place, not staged in registers: this rare path stays light on the decide
        // kernel's registers; the arithmetic is the slot kernels')
        const double *x = XT + (sb + s) * NX;
        if (k == L.N(ip)) {
            finish_terminal(p, d, b, s, ip, c, cn, x, true);
            continue;
        }
        const int kc = L.k0(ip) + k;
        const double *u = UT + (kq + kc) * NU;
        const double *ovr = constraint_forces(d, E, b, kc);
        const double *xr = ref_ptr(p, d.ref_x, b, s, NX), *pf = ref_ptr(p, d.ref_foot, b, s, 12);
        const double *ur = ref_ptr(p, d.ref_u, b, s, NU);
        const double *dl = d.reb_delta + (kq + kc) * 20, *ep = d.reb_eps + (kq + kc) * 20;
        double viol;
        d.slot_cost[sb + s] = running_cost(p, c, x, u, xr, ur, pf, dl, ep, viol, ovr);
        d.slot_viol[sb + s] = viol;
    }
}

// k_decide: reductions of one trial + merit acceptance (MultiPhaseDDP.cpp:113-133) + the
// later-termination test (:358).  16 lanes per element, one per phase: each lane sums its phase's
// slots in order, and the phase sums are added in phase order — the reference's summation order
// (compute_cost, MultiPhaseDDP.cpp:431-440; SinglePhase.cpp:235-262).  A trial whose rollout broke
// the 1e6 bound (slot_div) is rejected after its rows and slot outputs are made the reference's
// mixed ones (diverged_fixup); max_tconstr / max_pconstr then cover the phases before the break
// only (MultiPhaseDDP.cpp:83-92).
template <bool EL>
DEV void decide_group(const Params &p, const Bufs &d, double eps, int last, int init, int tix, int group)
{
    const int lane = threadIdx.x, g = lane & 15, base = lane & ~15;
    const int b = group * 4 + (lane >> 4);
    const bool valid = b < p.B;
    const ElemState *Ep = valid ? &d.el[b] : nullptr;
    const bool act = valid && (init ? !Ep->done : Ep->ls_active);
    const auto L = layout_of<EL>(d, valid ? b : 0);
    const int P = L.P();
    constexpr int NONE = 0x7fffffff;
    double ci = 0.0, fi = 0.0, pv = 0.0, tv = 0.0;
    int kd = NONE;  // first knot of the lane's phase whose simulated state breaks the bound
    auto sums = [&]() {
        ci = 0.0; fi = 0.0; pv = 0.0; tv = 0.0;
        if (!(act && g < P)) return;
        const size_t sb = (size_t)b * p.S + L.s0(g);
        const int N = L.N(g);
        // one pass, unrolled so that the loads of several slots are in flight together (each sum
        // keeps its slot order)
#pragma unroll 10
        for (int k = 0; k < N; ++k) {
            ci += d.slot_cost[sb + k];
            pv = fmin(pv, d.slot_viol[sb + k]);
            fi += d.slot_feas[sb + k];
            kd = (d.slot_div[sb + k] && k < kd) ? k : kd;
        }
        ci += d.slot_cost[sb + N];
        fi += d.slot_feas[sb + N];
        kd = (d.slot_div[sb + N] && N < kd) ? N : kd;
        tv = d.slot_viol[sb + N];
    };
    sums();
    double cost = 0.0, feas = 0.0, max_p = 0.0, max_t = 0.0;
    int sbrk = NONE;  // the element's first breaking slot
    for (int i = 0; i < p.P; ++i)
        sbrk = min(sbrk, __shfl(kd < NONE && g < P ? L.s0(g) + kd : NONE, base + i));
    const bool dvg = act && sbrk < NONE;
    int ibrk = NONE;
    if (__builtin_amdgcn_ballot_w64(dvg)) {  // (wave-uniform: the lanes of other elements repeat their sums)
        if (dvg) diverged_fixup<EL>(p, d, L, b, g, sbrk);
        __threadfence();
        kd = NONE;
        sums();
        if (dvg) {
            int ks;
            slot_phase(L, sbrk, ibrk, ks);
            if (g >= ibrk) { pv = 0.0; tv = 0.0; }  // phases from the break on: not reached
        }
    }
    if (act) {
        const ElemState &Er = d.el[b];
        // (a rollout that passed every knot computed every stored GRF value from its rows: E.ovr = 0
        // below, and the per-knot flags are not read until a fix-up sets it again)
        // the phases it completed computed their touchdown residuals
        if (Er.td_stale && g < P && g < ibrk)
            for (int j = 0; j < MTD; ++j) d.td_mask[((size_t)b * p.P + g) * MTD + j] &= ~TD_STALE;
    }
    for (int i = 0; i < p.P; ++i) {  // uniform bound (lanes g >= P add exact zeros)
        cost += __shfl(ci, base + i);
        feas += __shfl(fi, base + i);
        max_p = fmin(max_p, __shfl(pv, base + i));
        max_t = fmax(max_t, __shfl(tv, base + i));
    }
    if (!act || g != 0) return;
    ElemState &E = d.el[b];
    feas = sqrt(feas);
    E.max_p = max_p;
    E.max_t = max_t;
    if (!dvg) { E.ovr = 0; E.td_stale = 0; }  // (the stale bits cleared above)
    // one entry of the solver-info buffers (cost_buffer, dyn_feas_buffer, eqn_feas_buffer,
    // ineq_feas_buffer; MultiPhaseDDP.cpp:277-280, 368-371), float as the reference's vectors
    auto push_info = [&]() {
        if (E.hist_n < p.hcap) {
            float *hv = d.hist + ((size_t)b * p.hcap + E.hist_n) * 4;
            hv[0] = (float)E.cost; hv[1] = (float)E.feas; hv[2] = (float)E.max_t; hv[3] = (float)E.max_p;
        }
        E.hist_n += 1;
    };
    const int q = d.sel[b], nb = q & 3, tb = trial_of(nb, (q >> 2) & 3);
    if (init) {  // the initial rollout is taken (update_nominal_trajectory, MultiPhaseDDP.cpp:258)
        d.sel[b] = sel_code(tb, tb);
        E.cost = cost; E.feas = feas; E.accepted = 1;
        push_info();  // the initial information (:277-280)
        return;
    }
    E.n_ls += 1;
    const double merit = cost + E.merit_rho * feas;
    const double exp_cost = eps * E.dV1 + 0.5 * eps * eps * E.dV2;
    const double exp_merit = exp_cost - eps * E.merit_rho * E.feas_prev;
    E.cost = cost; E.feas = feas; E.merit = merit;
    bool fin = false;
    if ((merit <= E.merit_prev + p.gamma * exp_merit) && !dvg) {
        E.accepted = 1; E.ls_active = 0; fin = true;
        d.sel[b] = sel_code(tb, tb);  // the trial becomes the nominal and the working trajectory
    } else {
        // the trial's rows are the working ones (the reference's X): the next trial writes the
        // third buffer, and after the last one they stay (quirk A2)
        d.sel[b] = sel_code(nb, tb);
        if (last) { E.accepted = 0; E.ls_active = 0; E.cost = E.cost_prev; E.merit = E.merit_prev; fin = true; }
    }
    if (!fin && tix >= 0 && tix < LS_LIVE) d.ls_live[tix] = 1;  // still searching (same value from every writer)
    if (fin && p.trace && E.iters >= 1 && E.iters <= 64) {
        // diagnostic trace (HSDDP_TRACE): 16 bits per inner iteration — trials (bits 0..2), accepted
        // (3), the sweep's regularisation as round(log2 mu) + 64 (bits 4..15; 0: mu = 0)
        const double mu = E.reg * 20;  // (k_riccati leaves mu / 20, or 0 below 1e-6 / 20)
        const int code = mu > 0 ? min(4095, max(1, (int)rint(log2(mu)) + 64)) : 0;
        const unsigned long long v = (unsigned long long)((tix + 1) | (E.accepted << 3) | (code << 4)) & 0xffffull;
        const int it = E.iters - 1;
        d.dbg[(size_t)b * 16 + it / 4] |= v << (16 * (it % 4));
    }
    if (fin) {
        // the later-termination test breaks before the iteration's entry is buffered (:358-371)
        if (!p.no_early_exit && fabs((E.cost_prev - E.cost) / E.cost_prev) < p.cost_thresh && E.feas <= p.feas_thresh)
            E.inner_done = 1;
        else
            push_info();
    }
}

// (six waves per SIMD as before the divergence path: that rare path spills instead)
template <bool EL>
__global__ __launch_bounds__(64) void k_decide(Params p, Bufs d, double eps, int last,
                                                                                         int init, int tix)
{
    if (ls_skip(d, tix)) return;
    decide_group<EL>(p, d, eps, last, init, tix, blockIdx.x);
}

// One line-search trial: the slot and boundary blocks (rollout_block), and — FUSE, small batches
// without non-shooting tails (launch_rollout) — the trial's decision by the last block to finish:
// every block publishes its slot outputs (device-scope release) and takes a ticket; the block
// holding the last ticket (acquire) runs k_decide's work for the batch, four elements at a time,
// and resets the ticket counter.  One launch less per trial on the latency path of C1.
template <bool EL, bool FUSE, bool WIDE>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(HSDDP_ROLLOUT_WAVES))) void k_rollout(
    Params p, Bufs d, double eps, int init, int tix, int last)
{
    if (ls_skip(d, tix)) return;
    rollout_block<EL, WIDE>(p, d, eps, init, tix);
    if constexpr (FUSE) {
        __shared__ int ticket;
        __threadfence();
        if (threadIdx.x == 0) ticket = atomicAdd(&d.counter[7], 1);
        __syncthreads();
        if (ticket != (int)gridDim.x - 1) return;
        __threadfence();
        for (int q = 0; q < (p.B + 3) / 4; ++q) decide_group<EL>(p, d, eps, last, init, tix, q);
        if (threadIdx.x == 0) d.counter[7] = 0;
    }
}

// Trajectory::update_nominal_vals (TrajectoryManagement.cpp:110-115) is k_decide's flip of
// Bufs::sel: the accepted trial's buffer becomes the nominal one, no rows are copied.  (Defect_bar
// is never read by the solver, MultiPhaseDDP.cpp / SinglePhase.cpp, and is not kept.)

// one element's nominal rows into buffer 0 (a swap of buffer 0 with the nominal's, rows of X, U and
// Defect): host downloads and uploads see Xbar / Ubar in buffer 0; sel is fixed up by k_normalize_sel
__global__ __launch_bounds__(256) void k_normalize(Params p, Bufs d)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long per = (long)p.S * (NX / 2);
    if (gid >= (long)p.B * per) return;
    const int b = (int)(gid / per);
    const int nb = nom_buf(d, b);
    if (nb == 0) return;
    auto swap2 = [&](double *a0, double *a1, long at) {
        double2 *x0 = reinterpret_cast<double2 *>(a0), *x1 = reinterpret_cast<double2 *>(a1);
        const double2 t = x0[at];
        x0[at] = x1[at];
        x1[at] = t;
    };
    swap2(xbuf(d, 0), xbuf(d, nb), gid);
    swap2(dbuf(d, 0), dbuf(d, nb), gid);
    const long r = gid % per;
    if (r < (long)p.Kc * (NU / 2)) swap2(ubuf(d, 0), ubuf(d, nb), (long)b * p.Kc * (NU / 2) + r);
}
__global__ void k_normalize_sel(Params p, Bufs d)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    const int nb = nom_buf(d, b), wb = work_buf(d, b);
    if (nb == 0) return;
    // nominal now in 0; buffers 0 and nb traded their rows, the working index follows its rows
    d.sel[b] = sel_code(0, wb == nb ? 0 : wb == 0 ? nb : wb);
}

// the working trajectory back at the nominal one (X = Xbar, U = Ubar) with a zero Defect, rows left
// where they are: first the nominal buffer's Defect rows are zeroed (k_reset_defect), then the
// working index follows the nominal (k_reset_sel)
__global__ __launch_bounds__(256) void k_reset_defect(Params p, Bufs d)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    const long per = (long)p.S * (NX / 2);
    if (gid >= (long)p.B * per) return;
    reinterpret_cast<double2 *>(dbuf(d, nom_buf(d, (int)(gid / per))))[gid] = double2{0.0, 0.0};
}
__global__ void k_reset_sel(Params p, Bufs d)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b < p.B) d.sel[b] = sel_code(nom_buf(d, b), nom_buf(d, b));
}

__global__ void k_outer_begin(Params p, Bufs d)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    ElemState &E = d.el[b];
    if (E.done) return;
    E.outer_iters += 1;
    E.max_t_prev = E.max_t;
    E.max_p_prev = E.max_p;
    E.reg = 0.0;
    E.inner_done = 0;
}

// update_REB_params (ConstraintsBase.h:168-183) per (element, control slot)
template <bool EL>
__global__ __launch_bounds__(256) void k_reb_update(Params p, Bufs d)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)p.B * p.Kc) return;
    const int b = (int)(gid / p.Kc), kc = (int)(gid % p.Kc);
    if (d.el[b].done) return;
    const auto L = layout_of<EL>(d, b);
    int i = 0;
    for (int j = 1; j < L.P(); ++j)
        if (kc >= L.k0(j)) i = j;
    int c[4], cn[4];
    load_contacts(d, p, b, i, c, cn);
    const double *u = ubuf(d, work_buf(d, b)) + gid * NU;
    // the knot's stored GRF constraint values: from the control row, or older forces
    const double *ovr = constraint_forces(d, d.el[b], b, kc);
    double *dl = d.reb_delta + gid * 20, *ep = d.reb_eps + gid * 20;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        if (!c[l]) continue;
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            const double f[3] = {grf_force(u, ovr, 3 * l), grf_force(u, ovr, 3 * l + 1), grf_force(u, ovr, 3 * l + 2)};
            double g = grf_value(p.mu, r, f);
            if (g > -p.pconstr_thresh) continue;
            ep[5 * l + r] *= p.update_ReB;
            dl[5 * l + r] *= p.update_relax;
            dl[5 * l + r] = fmax(dl[5 * l + r], p.grf_delta_min);
        }
    }
}

// update_AL_params (ConstraintsBase.h:349-365) + outer convergence tests (MultiPhaseDDP.cpp:397-408)
template <bool EL>
__global__ void k_outer_end(Params p, Bufs d)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    ElemState &E = d.el[b];
    if (E.done) return;
    if (p.AL_active) {
        const int P = layout_of<EL>(d, b).P();
        // TerminalConstraintBase::update_params (ConstraintsBase.h:354-372) of every touchdown
        // constraint of every phase, leg by leg
        for (int i = 0; i < P; ++i)
            for (int j = 0; j < MTD; ++j) {
                const int m = d.td_mask[((size_t)b * p.P + i) * MTD + j];
                for (int l = 0; l < 4; ++l) {
                    if (!((m >> l) & 1)) continue;
                    // the constraint's stored h: 0 when never computed since it was registered
                    const double h = (m & TD_STALE) ? 0.0 : d.term_h[((size_t)b * p.P + i) * 4 + l];
                    const size_t q = (((size_t)b * p.P + i) * MTD + j) * 4 + l;
                    if (fabs(h) < p.tconstr_thresh) continue;
                    if (fabs(h) > 0.005) {
                        d.al_sigma[q] *= p.update_penalty;
                        d.al_sigma[q] = fmin(d.al_sigma[q], p.td_sigma_max);
                    } else {
                        d.al_lambda[q] += h * d.al_sigma[q];
                    }
                }
            }
    }
    if (p.no_early_exit) return;
    if (E.max_t < p.tconstr_thresh && fabs(E.max_p) < p.pconstr_thresh && E.feas <= p.feas_thresh) E.done = 1;
    else if (fabs(E.max_t - E.max_t_prev) < 0.0001 && fabs(E.max_p - E.max_p_prev) < 0.0001 &&
             E.feas <= p.feas_thresh)
        E.done = 1;
}

__global__ void k_reset_elements(Params p, Bufs d)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= p.B) return;
    ElemState &E = d.el[b];
    const int ovr = E.ovr, tds = E.td_stale;  // (the constraint objects outlive the solve)
    E = ElemState{};
    E.ovr = ovr;
    E.td_stale = tds;
}

__global__ __launch_bounds__(256) void k_init_params(Params p, Bufs d)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < (long)p.B * p.Kc * 20) { d.reb_delta[gid] = p.grf_delta; d.reb_eps[gid] = p.grf_eps; }
    if (gid < (long)p.B * p.P * MTD * 4) { d.al_sigma[gid] = p.td_sigma; d.al_lambda[gid] = p.td_lambda; }
    // one touchdown constraint per phase towards the next phase's contact (HKDProblem::
    // initialization's add_tconstr_one_phase, HKDProblem.cpp:104), resolved from the contact rows
    if (gid < (long)p.B * p.P * MTD) d.td_mask[gid] = gid % MTD == 0 ? TD_PENDING | TD_STALE : 0;
    // a new problem's constraint values are zero (create_data, ConstraintsBase.h:26-34, 50-54):
    // every knot's GRF values from zero forces, every touchdown h zero (TD_STALE above)
    if (gid < (long)p.B * p.Kc * 12) d.cf_u[gid] = 0.0;
    if (gid < (long)p.B * p.Kc) d.cf_flag[gid] = 1;
    if (gid < (long)p.B) { d.el[gid].ovr = 1; d.el[gid].td_stale = 1; }
}

// Px rows 0 .. 11 of every terminal record slot (the allocation's B x MAXP, whatever the
// layout): the reset map leaves the orientation, position and velocity rows as the identity's
// (HKDReset.h:78-136), so k_terminal writes only rows 12 .. 23
__global__ __launch_bounds__(256) void k_term_identity(Params p, Bufs d)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)p.B * MAXP * 12 * NX) return;
    const long rec = gid / (12 * NX);
    const int e = (int)(gid % (12 * NX));
    d.term[rec * TW + TM_PX + e] = (e / NX == e % NX) ? 1.0 : 0.0;
}

// TD_PENDING slots take the touchdown legs of their phase's contact rows (0: no constraint)
template <bool EL>
__global__ __launch_bounds__(256) void k_resolve_td(Params p, Bufs d)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (long)p.B * p.P * MTD) return;
    const int b = (int)(gid / ((long)p.P * MTD)), i = (int)(gid / MTD % p.P);
    int &m = d.td_mask[gid];
    if (i >= layout_of<EL>(d, b).P()) { m = 0; return; }
    if (!(m & TD_PENDING)) return;
    int c[4], cn[4];
    load_contacts(d, p, b, i, c, cn);
    const int legs = td_bits(c, cn);
    m = legs ? legs | (m & TD_STALE) : 0;
}

// Bufs::ref_t: one thread per (entry j, column r), j-major so that the column stores are contiguous
__global__ __launch_bounds__(256) void k_ref_columns(Bufs d, long ncol)
{
    const long gid = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= ncol * REF_COLS) return;
    const int j = (int)(gid / ncol);
    const long r = gid % ncol;
    const double v = j < NX ? d.ref_x[r * NX + j] : j < NX + NU ? d.ref_u[r * NU + j - NX] : d.ref_foot[r * 12 + j - NX - NU];
    d.ref_t[((size_t)(j >> 1) * d.ref_tw + r) * 2 + (j & 1)] = v;
}

void launch_ref_columns(const Params &p, const Bufs &d, int Bref, hipStream_t st)
{
    const long ncol = (long)Bref * p.S, n = ncol * REF_COLS;
    hipLaunchKernelGGL(k_ref_columns, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d, ncol);
}

// which: 0 = elements with ls_active, 1 = elements still iterating (!done && !inner_done), 2 = !done
__global__ void k_count(Params p, Bufs d, int which)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    int v = 0;
    if (b < p.B) {
        const ElemState &E = d.el[b];
        v = which == 0 ? E.ls_active : which == 1 ? (!E.done && !E.inner_done) : !E.done;
    }
    unsigned long long m = __ballot(v);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(&d.counter[which], __popcll(m));
}

// sums of n_ls and iters over the elements into counter[4], counter[5] (hsddp_stats)
__global__ void k_stat_sums(Params p, Bufs d)
{
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    int a = 0, c = 0;
    if (b < p.B) {
        a = d.el[b].n_ls;
        c = d.el[b].iters;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        a += __shfl_xor(a, o);
        c += __shfl_xor(c, o);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(&d.counter[4], a);
        atomicAdd(&d.counter[5], c);
    }
}

// ---------------------------------------------------------------------------------------------
// model primitives
__global__ void k_model_dynamics(const double *x, const double *u, const double *c, double dt, double *xn, int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    hkd_step(x + (size_t)q * NX, u + (size_t)q * NU, c + (size_t)q * 4, dt, xn + (size_t)q * NX);
}

__global__ void k_model_partial(const double *x, const double *u, const double *c, double dt, double *A, double *B,
                                int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    double Se[SE_N], Sw[SW_N], Bw[BW_N];
    hkd_partial_compact(x + (size_t)q * NX, u + (size_t)q * NU, c + (size_t)q * 4, dt, Se, Sw, Bw);
    hkd_expand_colmajor(Se, Sw, Bw, c + (size_t)q * 4, dt, A + (size_t)q * NN, B + (size_t)q * NN);
}

__global__ void k_model_foot(const double *x, const int *leg, double *p, double *J, int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const double *xx = x + (size_t)q * NX;
    const int l = leg[q];
    if (p) hkd_foot_position(l, xx + 3, xx, xx + 12 + 3 * l, p + (size_t)q * 3);
    if (J) {
        double Jr[54];
        hkd_foot_jacobian(l, xx, xx + 12 + 3 * l, Jr);
        for (int r = 0; r < 3; ++r)
            for (int cc = 0; cc < 18; ++cc) J[(size_t)q * 54 + r + 3 * cc] = Jr[18 * r + cc];
    }
}

// ---- cost / constraint plugin primitives (the facade's hkd:: plugin bodies) ------------------
// One thread per point.  Params carries the weights (hsddp_hkd_weights via fill_weights) and dt;
// every index below is compile-time, so the by-value Params stays in SGPRs.
struct PluginOut {
    double *l, *lx, *lu, *lxx, *luu;  // running: RCostData (matrices column-major, = row-major: symmetric)
};
__global__ void k_model_running_cost(Params p, const double *x, const double *u, const int *cc, const double *xr,
                                     const double *ur, const double *pf, int terms, PluginOut o, int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const double *xq = x + (size_t)q * NX, *uq = u + (size_t)q * NU, *rq = xr + (size_t)q * NX,
                 *vq = ur + (size_t)q * NU, *fq = pf + (size_t)q * 12;
    int c[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) c[l] = cc[(size_t)q * 4 + l];
    double L = 0.0, gx[NX], gu[NU];
#pragma unroll
    for (int j = 0; j < NX; ++j) { gx[j] = 0.0; gu[j] = 0.0; }
    if (terms & 1) {  // HKDTrackingCost (HKDCost.h:8-38): .5 dt (e' Q e + eu' R eu)
        double lt = 0.0, lu = 0.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) { const double e = xq[j] - rq[j]; lt += e * q_diag(p, c, j) * e; gx[j] = p.dt * q_diag(p, c, j) * e; }
#pragma unroll
        for (int j = 0; j < NU; ++j) { const double e = uq[j] - vq[j]; lu += e * r_diag(p, j) * e; gu[j] = p.dt * r_diag(p, j) * e; }
        L += p.dt * (0.5 * lt + 0.5 * lu);
    }
    if (terms & 2) {  // HKDFootPlaceReg (HKDCost.cpp:5-33): .5 dt d' Qfoot d, d = prel - prel_r
        double lf = 0.0;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double e = (xq[12 + j] - xq[3 + j % 3]) - (fq[j] - rq[3 + j % 3]);
            const double w = foot_weight(p, c, j);
            lf += e * w * e;
            gx[3 + j % 3] += -(p.dt * w * e);
            gx[12 + j] += p.dt * w * e;
        }
        L += p.dt * (.5 * lf);
    }
    if (o.l) o.l[q] = L;
    if (o.lx) for (int j = 0; j < NX; ++j) o.lx[(size_t)q * NX + j] = gx[j];
    if (o.lu) for (int j = 0; j < NU; ++j) o.lu[(size_t)q * NU + j] = gu[j];
    if (o.lxx) {
        double *m = o.lxx + (size_t)q * NN;
        for (int e = 0; e < NN; ++e) m[e] = 0.0;
        if (terms & 1)
#pragma unroll
            for (int j = 0; j < NX; ++j) m[j * NX + j] = p.dt * q_diag(p, c, j);
        if (terms & 2)
#pragma unroll
            for (int j = 0; j < 12; ++j) {
                const double w = p.dt * foot_weight(p, c, j);
                const int a = 3 + j % 3, bb = 12 + j;
                m[a * NX + a] += w; m[bb * NX + bb] += w; m[a * NX + bb] -= w; m[bb * NX + a] -= w;
            }
    }
    if (o.luu) {
        double *m = o.luu + (size_t)q * NN;
        for (int e = 0; e < NN; ++e) m[e] = 0.0;
        if (terms & 1)
#pragma unroll
            for (int j = 0; j < NU; ++j) m[j * NU + j] = p.dt * r_diag(p, j);
    }
}

__global__ void k_model_terminal_cost(Params p, const double *x, const int *cc, const double *xr, const double *pf,
                                      int terms, double *Phi, double *Phix, double *Phixx, int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const double *xq = x + (size_t)q * NX, *rq = xr + (size_t)q * NX, *fq = pf + (size_t)q * 12;
    int c[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) c[l] = cc[(size_t)q * 4 + l];
    double F = 0.0, g[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) g[j] = 0.0;
    if (terms & 1) {  // HKDTrackingCost::terminal_cost(_par): .5 e' Qf e
        double phi = 0.0;
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            const double e = xq[j] - rq[j], w = p.qf_gain * p.qf_scale[j] * q_diag(p, c, j);
            phi += e * w * e;
            g[j] = w * e;
        }
        F += 0.5 * phi;
    }
    if (terms & 2) {  // HKDFootPlaceReg::terminal_cost(_par) (HKDCost.cpp:35-63): 10 d' Qfoot d, 20 D' Qfoot d
        double fc = 0.0;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double e = (xq[12 + j] - xq[3 + j % 3]) - (fq[j] - rq[3 + j % 3]);
            const double w = foot_weight(p, c, j);
            fc += e * w * e;
            g[3 + j % 3] += -(p.foot_term_grad * w * e);
            g[12 + j] += p.foot_term_grad * w * e;
        }
        F += p.foot_term_cost * fc;
    }
    if (Phi) Phi[q] = F;
    if (Phix) for (int j = 0; j < NX; ++j) Phix[(size_t)q * NX + j] = g[j];
    if (Phixx) {
        double *m = Phixx + (size_t)q * NN;
        for (int e = 0; e < NN; ++e) m[e] = 0.0;
        if (terms & 1)
#pragma unroll
            for (int j = 0; j < NX; ++j) m[j * NX + j] = p.qf_gain * p.qf_scale[j] * q_diag(p, c, j);
        if (terms & 2)
#pragma unroll
            for (int j = 0; j < 12; ++j) {
                const double w = p.foot_term_grad * foot_weight(p, c, j);
                const int a = 3 + j % 3, bb = 12 + j;
                m[a * NX + a] += w; m[bb * NX + bb] += w; m[a * NX + bb] -= w; m[bb * NX + a] -= w;
            }
    }
}

// GRFConstraint (HKDConstraints.cpp:7-66): 5 friction-pyramid rows per stance leg, in leg order;
// g [n][20] and gu [n][20][24] (rows past 5 x stance legs are zero)
__global__ void k_model_grf(const double *u, const int *cc, double mu, double *g, double *gu, int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    int row = 0;
    for (int e = 0; e < 20; ++e) {
        if (g) g[(size_t)q * 20 + e] = 0.0;
        if (gu) for (int j = 0; j < NU; ++j) gu[((size_t)q * 20 + e) * NU + j] = 0.0;
    }
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        if (!cc[(size_t)q * 4 + l]) continue;
#pragma unroll
        for (int r = 0; r < 5; ++r, ++row) {
            double a[3];
            grf_row(mu, r, a);
            if (g) g[(size_t)q * 20 + row] = grf_value(mu, r, u + (size_t)q * NU + 3 * l);
            if (gu) for (int k = 0; k < 3; ++k) gu[((size_t)q * 20 + row) * NU + 3 * l + k] = a[k];
        }
    }
}

// TouchDownConstraint (HKDConstraints.cpp:69-171): h = foot height - ground for each leg touching
// down (c = 0, next c = 1), in leg order; h [n][4], hx [n][4][24] (unused rows zero)
__global__ void k_model_touchdown(const double *x, const int *cc, const int *cn, double ground, double *h, double *hx,
                                  int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const double *xq = x + (size_t)q * NX;
    for (int e = 0; e < 4; ++e) {
        if (h) h[(size_t)q * 4 + e] = 0.0;
        if (hx) for (int j = 0; j < NX; ++j) hx[((size_t)q * 4 + e) * NX + j] = 0.0;
    }
    int row = 0;
    for (int l = 0; l < 4; ++l) {
        if (!(cc[(size_t)q * 4 + l] == 0 && cn[(size_t)q * 4 + l] == 1)) continue;
        double ge[3], gq[3];
        const double hv = hkd_foot_height_grad_sparse(l, xq, ge, gq) - ground;
        if (h) h[(size_t)q * 4 + row] = hv;
        if (hx) {
            double *r = hx + ((size_t)q * 4 + row) * NX;
            for (int k = 0; k < 3; ++k) { r[k] = ge[k]; r[12 + 3 * l + k] = gq[k]; }
            r[5] = 1.0;
        }
        ++row;
    }
}

__global__ void k_model_reset(const double *x, const int *c, const int *cn, double *xn, double *Px, int n)
{
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= n) return;
    const double *xx = x + (size_t)q * NX;
    if (xn) hkd_resetmap(xx, c + (size_t)q * 4, cn + (size_t)q * 4, xn + (size_t)q * NX);
    if (Px)
        for (int r = 0; r < NX; ++r) {
            double row[NX];
            hkd_resetmap_partial_row(xx, c + (size_t)q * 4, cn + (size_t)q * 4, r, row);
            for (int cc = 0; cc < NX; ++cc) Px[(size_t)q * NN + r + NX * cc] = row[cc];
        }
}

// ---------------------------------------------------------------------------------------------
static inline unsigned blocks_for(long n, int bs) { return (unsigned)((n + bs - 1) / bs); }

// the kernel instantiation for the handle's layout mode (shared / per element)
#define LAUNCH_EL(kern, grid, block, st, ...)                                                       \
    do {                                                                                            \
        if (p.elem_layout) hipLaunchKernelGGL(kern<true>, grid, block, 0, st, __VA_ARGS__);         \
        else hipLaunchKernelGGL(kern<false>, grid, block, 0, st, __VA_ARGS__);                      \
    } while (0)

// small batches without non-shooting tails decide each trial in its rollout launch (k_rollout FUSE);
// HSDDP_NO_FUSED_DECIDE=1 (read at every launch: a test switches it in-process) keeps k_decide's
// launch, for the equality test of the two paths
static bool fused_decide(const Params &p)
{
    if (p.B > 16 || p.has_tail || p.ms0) return false;
    const char *e = std::getenv("HSDDP_NO_FUSED_DECIDE");
    return !(e && *e && *e != '0');
}

void launch_rollout(const Params &p, const Bufs &d, double eps, int last, int init, int tix, hipStream_t st)
{
    if (p.ms0) {  // single shooting: every knot simulated (k_rollout_ss)
        LAUNCH_EL(k_rollout_ss, dim3((p.B + 3) / 4), dim3(64), st, p, d, eps, init, tix);
        return;
    }
    // slot waves, then the phase-boundary waves (k_rollout, rollout_boundary)
    const dim3 g(blocks_for((long)p.B * p.S, 64) + blocks_for((long)p.B * p.P, 64));
    const bool wide = p.S >= RW;  // (rollout_block)
    if (fused_decide(p)) {
        if (p.elem_layout) {
            if (wide) hipLaunchKernelGGL((k_rollout<true, true, true>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
            else hipLaunchKernelGGL((k_rollout<true, true, false>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
        } else {
            if (wide) hipLaunchKernelGGL((k_rollout<false, true, true>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
            else hipLaunchKernelGGL((k_rollout<false, true, false>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
        }
        return;
    }
    if (p.elem_layout) {
        if (wide) hipLaunchKernelGGL((k_rollout<true, false, true>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
        else hipLaunchKernelGGL((k_rollout<true, false, false>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
    } else {
        if (wide) hipLaunchKernelGGL((k_rollout<false, false, true>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
        else hipLaunchKernelGGL((k_rollout<false, false, false>), g, dim3(64), 0, st, p, d, eps, init, tix, last);
    }
    if (p.has_tail) LAUNCH_EL(k_rollout_tail, dim3((p.B + 63) / 64), dim3(64), st, p, d, eps, init, tix);
}
void launch_decide(const Params &p, const Bufs &d, double eps, int last, int init, int tix, hipStream_t st)
{
    if (fused_decide(p)) return;  // decided by the rollout launch
    LAUNCH_EL(k_decide, dim3((p.B + 3) / 4), dim3(64), st, p, d, eps, last, init, tix);
}
void launch_normalize(const Params &p, const Bufs &d, hipStream_t st)
{
    hipLaunchKernelGGL(k_normalize, dim3(blocks_for((long)p.B * p.S * (NX / 2), 256)), dim3(256), 0, st, p, d);
    hipLaunchKernelGGL(k_normalize_sel, dim3(blocks_for(p.B, 256)), dim3(256), 0, st, p, d);
}
// The terminal tasks, TERM_TPW per wave, two waves per block: a launch of their own (82 VGPRs,
// 4.3 KB of LDS per task: 4.5 waves per SIMD; as the tail of k_lq's launch they ran at its two).
// The first wave
// also resets the iteration's counters: the parallel-retry list of the k_riccati launch that
// follows starts empty (its only reader before then is the previous iteration's
// k_riccati_select), no element has been seen searching after any trial yet (ls_live), and
// k_count's activity counts start from zero (the graph-replayed iteration has no memset launches).
template <bool EL>
__global__ __launch_bounds__(128, 4) void k_terminal(Params p, Bufs d)
{
    __shared__ TermLds S[2 * TERM_TPW];
    const int w = threadIdx.x >> 6;
    terminal_wave<EL>(p, d, S + w * TERM_TPW, (long)blockIdx.x * 2 + w, threadIdx.x & 63);
}

void launch_lq(const Params &p, const Bufs &d, hipStream_t st)
{
    // the terminal waves: a launch of their own (five waves per SIMD), or, for a small batch whose
    // knot and terminal blocks all fit the chip at once (C1: one robot), the blocks after k_lq's
    // knot blocks in the same launch — one launch less on the latency path
    const unsigned nterm = blocks_for((long)p.B * p.P, 4 * TERM_TPW);
    const bool merged = nterm <= 256;
    const bool by_knot = !p.lq_slots && !p.fp32;  // k_lq's grid: control knots or state slots
    if (!merged) {
        const unsigned nt2 = blocks_for((long)p.B * p.P, 2 * TERM_TPW);
        if (p.elem_layout) hipLaunchKernelGGL((k_terminal<true>), dim3(nt2), dim3(128), 0, st, p, d);
        else hipLaunchKernelGGL((k_terminal<false>), dim3(nt2), dim3(128), 0, st, p, d);
    }
    const dim3 g(blocks_for((long)p.B * (by_knot ? p.Kc : p.S), 256) + (merged ? nterm : 0));
    if (p.fp32) {
#define HSDDP_LQ(f, e)                                                          \
    do {                                                                        \
        if (p.lq_slots) hipLaunchKernelGGL((k_lq<f, e, true>), g, dim3(256), 0, st, p, d); \
        else hipLaunchKernelGGL((k_lq<f, e, false>), g, dim3(256), 0, st, p, d);           \
    } while (0)
        if (p.elem_layout) HSDDP_LQ(true, true);
        else HSDDP_LQ(true, false);
    } else {
        if (p.elem_layout) HSDDP_LQ(false, true);
        else HSDDP_LQ(false, false);
#undef HSDDP_LQ
    }
}

__global__ __launch_bounds__(256) void k_broadcast(double *dst, const double *src, size_t n, size_t total)
{
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid < total) dst[gid] = src[gid % n];
}
void launch_broadcast(double *dst, const double *src, size_t n, size_t copies, hipStream_t st)
{
    const size_t total = n * copies;
    if (total) hipLaunchKernelGGL(k_broadcast, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, dst, src, n, total);
}

void launch_reset_working(const Params &p, const Bufs &d, hipStream_t st)
{
    hipLaunchKernelGGL(k_reset_defect, dim3(blocks_for((long)p.B * p.S * (NX / 2), 256)), dim3(256), 0, st, p, d);
    hipLaunchKernelGGL(k_reset_sel, dim3(blocks_for(p.B, 256)), dim3(256), 0, st, p, d);
}
void launch_outer_begin(const Params &p, const Bufs &d, hipStream_t st)
{
    hipLaunchKernelGGL(k_outer_begin, dim3(blocks_for(p.B, 256)), dim3(256), 0, st, p, d);
}
void launch_reb_update(const Params &p, const Bufs &d, hipStream_t st)
{
    LAUNCH_EL(k_reb_update, dim3(blocks_for((long)p.B * p.Kc, 256)), dim3(256), st, p, d);
}
void launch_outer_end(const Params &p, const Bufs &d, hipStream_t st)
{
    LAUNCH_EL(k_outer_end, dim3(blocks_for(p.B, 256)), dim3(256), st, p, d);
}
void launch_reset_elements(const Params &p, const Bufs &d, hipStream_t st)
{
    hipLaunchKernelGGL(k_reset_elements, dim3(blocks_for(p.B, 256)), dim3(256), 0, st, p, d);
}
void launch_init_params(const Params &p, const Bufs &d, hipStream_t st)
{
    long n = (long)p.B * p.Kc * 20;
    if ((long)p.B * p.P * MTD * 4 > n) n = (long)p.B * p.P * MTD * 4;
    hipLaunchKernelGGL(k_init_params, dim3(blocks_for(n, 256)), dim3(256), 0, st, p, d);
    hipLaunchKernelGGL(k_term_identity, dim3(blocks_for((long)p.B * MAXP * 12 * NX, 256)), dim3(256), 0, st, p, d);
}
void launch_resolve_td(const Params &p, const Bufs &d, hipStream_t st)
{
    LAUNCH_EL(k_resolve_td, dim3(blocks_for((long)p.B * p.P * MTD, 256)), dim3(256), st, p, d);
}
void launch_stat_sums(const Params &p, const Bufs &d, hipStream_t st)
{
    hipLaunchKernelGGL(k_stat_sums, dim3((p.B + 255) / 256), dim3(256), 0, st, p, d);
}

void launch_count(const Params &p, const Bufs &d, int which, hipStream_t st)
{
    hipLaunchKernelGGL(k_count, dim3(blocks_for(p.B, 256)), dim3(256), 0, st, p, d, which);
}
void launch_model_dynamics(const double *x, const double *u, const double *c, double dt, double *xn, int n,
                           hipStream_t st)
{
    hipLaunchKernelGGL(k_model_dynamics, dim3(blocks_for(n, 128)), dim3(128), 0, st, x, u, c, dt, xn, n);
}
void launch_model_partial(const double *x, const double *u, const double *c, double dt, double *A, double *B,
                          int n, hipStream_t st)
{
    hipLaunchKernelGGL(k_model_partial, dim3(blocks_for(n, 64)), dim3(64), 0, st, x, u, c, dt, A, B, n);
}
void launch_model_foot(const double *x, const int *leg, double *p, double *J, int n, hipStream_t st)
{
    hipLaunchKernelGGL(k_model_foot, dim3(blocks_for(n, 64)), dim3(64), 0, st, x, leg, p, J, n);
}
void launch_model_running_cost(const Params &p, const double *x, const double *u, const int *c, const double *xr,
                               const double *ur, const double *pf, int terms, double *l, double *lx, double *lu,
                               double *lxx, double *luu, int n, hipStream_t st)
{
    hipLaunchKernelGGL(k_model_running_cost, dim3(blocks_for(n, 64)), dim3(64), 0, st, p, x, u, c, xr, ur, pf, terms,
                       PluginOut{l, lx, lu, lxx, luu}, n);
}
void launch_model_terminal_cost(const Params &p, const double *x, const int *c, const double *xr, const double *pf,
                                int terms, double *Phi, double *Phix, double *Phixx, int n, hipStream_t st)
{
    hipLaunchKernelGGL(k_model_terminal_cost, dim3(blocks_for(n, 64)), dim3(64), 0, st, p, x, c, xr, pf, terms, Phi,
                       Phix, Phixx, n);
}
void launch_model_grf(const double *u, const int *c, double mu, double *g, double *gu, int n, hipStream_t st)
{
    hipLaunchKernelGGL(k_model_grf, dim3(blocks_for(n, 64)), dim3(64), 0, st, u, c, mu, g, gu, n);
}
void launch_model_touchdown(const double *x, const int *c, const int *cn, double ground, double *h, double *hx, int n,
                            hipStream_t st)
{
    hipLaunchKernelGGL(k_model_touchdown, dim3(blocks_for(n, 64)), dim3(64), 0, st, x, c, cn, ground, h, hx, n);
}
void launch_model_reset(const double *x, const int *c, const int *cn, double *xn, double *Px, int n,
                        hipStream_t st)
{
    hipLaunchKernelGGL(k_model_reset, dim3(blocks_for(n, 64)), dim3(64), 0, st, x, c, cn, xn, Px, n);
}

}  // namespace hsddp
