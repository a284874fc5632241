// hsddp_linear.hip — the multiple-shooting linear rollout that follows a successful sweep.
//
// MultiPhaseDDP::linear_rollout (HSDDPSolver/source/MultiPhaseDDP.cpp:20-50) over
// SinglePhase::linear_rollout (SinglePhase.cpp:144-178), then the merit function
// (MultiPhaseDDP.cpp:309-318), one wave per element: dX, du = dU + K dX, and the expected cost
// change of quirk A3 (it replaces the sweep's dV).  Templates on `real` as the sweep
// (hsddp_sweep.hip): double, or float in config C5's fp32 mode.
#include "hsddp_wave.h"

namespace hsddp {

using namespace hkd;

constexpr int HC = 12;  // coupled controls per knot

// Per-precision buffers: LQ record (stride LQS), compact gains and the Defect copy the sweep reads.
template <typename real> struct Prec;
template <> struct Prec<double> {
    static constexpr int LQS = LQW;
    static DEV const double *lq(const Bufs &d) { return d.lq; }
    static DEV double *K(const Bufs &d) { return d.K; }
    static DEV const double *def(const Bufs &d) { return d.Defect; }
};
template <> struct Prec<float> {
    static constexpr int LQS = LQW32;
    static DEV const float *lq(const Bufs &d) { return d.lq32; }
    static DEV float *K(const Bufs &d) { return d.K32; }
    static DEV const float *def(const Bufs &d) { return d.def32; }
};

// per-phase constants of one element
template <typename real>
struct PhaseConst {
    int c[4];
    int cmask;   // bit l = c_l: a lane-dependent leg index becomes one shift, not a select chain
    real bv[4];  // dt c_l / m     (B rows 9..11)
    real bq[4];  // dt (1 - c_l)   (B rows 12..23)
};

// Wave-uniform: contacts through the scalar cache, and selects instead of arithmetic so the
// constants stay in SGPRs (dt * c / m is dt / m or 0 exactly for c in {0, 1}).
template <typename real>
DEV void load_phase(const Params &p, const Bufs &d, size_t b, int i, PhaseConst<real> &pc)
{
    typedef const __attribute__((address_space(4))) int cint;
    cint *cs = (cint *)(d.contacts + (b * (p.P + 1) + i) * 4);
    pc.cmask = 0;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        pc.c[l] = cs[l];
        pc.cmask |= (pc.c[l] != 0) << l;
        pc.bv[l] = pc.c[l] ? (real)p.dt_m : (real)0;
        pc.bq[l] = pc.c[l] ? (real)0 : (real)p.dt;
    }
}

// lxx (dt Q + dt D^T Qfoot D, HKDCost.cpp:32) row r as: diagonal + cross terms with the foot columns
template <typename real>
struct LxxRow {
    real diag, xq[4], xp;  // xq[l]: (r in pos) x (col 12+3l+(r-3)); xp: (r in q) x (col 3+(r-12)%3)
};

// contact of leg l (runtime, lane-dependent) as 0 / 1
template <typename real>
DEV int contact(const PhaseConst<real> &pc, int l) { return (pc.cmask >> l) & 1; }

// a[i] for a runtime i, as selects (a runtime index would put the array in scratch)
template <typename T>
DEV T pick4(const T (&a)[4], int i)
{
    return i == 0 ? a[0] : i == 1 ? a[1] : i == 2 ? a[2] : a[3];
}

// a[i] for a runtime i < N, as selects over the (wave-uniform) entries
template <int N>
DEV double pick(const double (&a)[N], int i)
{
    double e[N];
#pragma unroll
    for (int k = 0; k < N; ++k) {
        e[k] = a[k];
        asm volatile("" : "+s"(e[k]));  // opaque: keeps the selects from folding back into an indexed load
    }
    double v = e[0];
#pragma unroll
    for (int k = 1; k < N; ++k) v = i == k ? e[k] : v;
    return v;
}

// q_diag / foot_weight (hsddp_device.h) with the lane-dependent indices resolved by selects:
// a lane-indexed read of a kernel-argument array is a memory round trip
template <typename real>
DEV void lxx_row(const Params &p, const PhaseConst<real> &pc, int r, LxxRow<real> &L)
{
    L.diag = 0.0; L.xp = 0.0;
#pragma unroll
    for (int l = 0; l < 4; ++l) L.xq[l] = 0.0;
    if (r >= NX) return;
    double dg = p.dt * (r < 12 ? pick(p.qbase, r) : p.q_qJ * (1 - contact(pc, (r - 12) / 3)));
    if (r >= 3 && r < 6) {
        // dt c^2 (foot_gain w c) = dt foot_gain w for c = 1, else 0 (selects: no per-phase
        // conversions kept live across the knot loop)
        const double fw = p.dt * (p.foot_gain * pick(p.foot_w, r - 3));
#pragma unroll
        for (int l = 0; l < 4; ++l) {
            const double w = pc.c[l] ? fw : 0.0;
            dg += w;
            L.xq[l] = -w;
        }
    } else if (r >= 12) {
        const int m = r - 12;
        const double w = contact(pc, m / 3) ? p.dt * (p.foot_gain * pick(p.foot_w, m % 3)) : 0.0;
        dg += w;
        L.xp = -w;
    }
    L.diag = dg;
}

// ---------------------------------------------------------------------------------------------
// MultiPhaseDDP::linear_rollout(1.0): dX, du = dU + K dX, and the expected cost change (quirk
// A3: it replaces the sweep's dV), then the merit function (MultiPhaseDDP.cpp:309-318).
// Lanes r < 24 of each half compute row r of the same vectors; the first half stores them.
// A knot's inputs (compact K, LQ record, Defect[k+1], dU) are one LDS image (4080 bytes in fp64,
// 2144 in the fp32 mode) filled by 16-byte-per-lane LDS-DMA loads (global_load_lds_dwordx4, four
// or three instructions); the next knot's image is loaded into the other buffer while this knot
// computes.
template <typename real>
struct LinImg {
    static constexpr int K = 0;                                       // byte offsets
    static constexpr int LQ = K + KCW * (int)sizeof(real);
    static constexpr int D = LQ + Prec<real>::LQS * (int)sizeof(real);
    static constexpr int DU = D + NX * (int)sizeof(real);
    static constexpr int END = DU + NX * 8;                           // dU stays fp64
    static constexpr int NI = (END / 16 + 63) / 64;                   // DMA instructions
    static_assert(LQ % 16 == 0 && D % 16 == 0 && DU % 16 == 0 && END % 16 == 0 && NI <= 4, "16-byte pieces");
};
template <typename real>
struct LinBuf {
    alignas(16) char v[LinImg<real>::NI * 64 * 16];
};
template <typename real>
struct LinElem {
    real dx[NX], du[NX];
};

// Issued as inline asm so the waitcnt pass does not track the LDS writes (it would otherwise wait
// for every DMA in flight before any LDS read); lin_knot waits explicitly.  LDS destination of
// piece t: M0 + 16 * lane, contiguous.
template <typename real>
DEV void lin_fetch(LinBuf<real> &buf, const Params &p, const Bufs &d, size_t b, int s, int kc, int lane)
{
    using I = LinImg<real>;
    const size_t kq = b * p.Kc + kc;
    // one base per segment, biased so that base + o addresses image byte o
    const size_t kB = (size_t)(Prec<real>::K(d) + kq * KCW) - I::K,
                 lB = (size_t)(Prec<real>::lq(d) + kq * Prec<real>::LQS) - I::LQ,
                 dB = (size_t)(Prec<real>::def(d) + (b * p.S + s + 1) * NX) - I::D,
                 uB = (size_t)(d.dU + kq * NX) - I::DU;
#pragma unroll
    for (int t = 0; t < I::NI; ++t) {
        int o = 16 * (64 * t + lane);    // first byte of this lane's 16-byte piece
        o = o < I::END ? o : I::END - 16;  // spare pieces repeat the last
        const size_t base = o < I::LQ ? kB : o < I::D ? lB : o < I::DU ? dB : uB;
        const char *src = (const char *)(base + (size_t)o);
        const unsigned m0 = (unsigned)(size_t)(buf.v + 1024 * t);
        unsigned keep;  // M0 is compiler-reserved: saved, set (one wait state before the DMA), restored
        asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                     : "=&s"(keep)
                     : "v"(src), "s"(m0)
                     : "memory");
    }
}

// one knot of SinglePhase::linear_rollout (SinglePhase.cpp:144-178) from the LDS image `cur`;
// when `more`, the next knot's image is requested into `nxt` first
template <typename real>
DEV void lin_knot(const Params &p, const Bufs &d, LinElem<real> &S, LinBuf<real> &cur, LinBuf<real> &nxt, bool more,
                  size_t b, int s, int kc, const PhaseConst<real> &pc, const LxxRow<real> &lx_, real ru, bool cpl,
                  int krow0, real &dx, real &v1, real &v2)
{
    using I = LinImg<real>;
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5, cb = HC * hf;
    const bool rowl = r < NX, st = rowl && hf == 0;
    const int rr = rowl ? r : 0;
    const real dt = p.dt;
#ifndef HSDDP_LIN_NOWAIT
#define HSDDP_LIN_NOWAIT 0  // diagnostic (wrong results): no wait for the knot's image
#endif
    if (more) {
        lin_fetch(nxt, p, d, b, s + 1, kc + 1, lane);
        // all but the I::NI just issued
        if (HSDDP_LIN_NOWAIT) {
        } else if constexpr (I::NI == 4)
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    static_assert(I::NI == 4 || I::NI == 3, "waitcnt above");
    LSYNC();
    const real *kimg = (const real *)(cur.v + I::K), *lq = (const real *)(cur.v + I::LQ),
               *dd = (const real *)(cur.v + I::D);
    const double *dUi = (const double *)(cur.v + I::DU);
    real krow[HC];
#pragma unroll
    for (int c = 0; c < HC; ++c) krow[c] = cpl ? kimg[krow0 + c] : (real)0;
    const real dUr = (real)dUi[rr];
    if (lane < NX) S.dx[lane] = dx;
    LSYNC();
    real kd = 0;
#pragma unroll
    for (int c = 0; c < HC; ++c) kd += krow[c] * S.dx[cb + c];
    kd += other_half(kd);
    const real du = dUr + kd;
    if (lane < NX) S.du[lane] = du;
    LSYNC();
    real nx = 0, q1 = 0, q2 = 0;
    if (rowl) {
        real sdx = 0;
        if (r < 3) {
#pragma unroll
            for (int q = 0; q < 5; ++q) sdx += lq[LQ_SE + 5 * r + q] * S.dx[se_col(q)];
        } else if (r < 6) {
            sdx = dt * S.dx[r + 6];
        } else if (r < 9) {
#pragma unroll
            for (int q = 0; q < 17; ++q) sdx += lq[sw_at(r - 6, q)] * S.dx[sw_col(q)];
        }
        real bdu = 0, lxd = lx_.diag * dx, lud = ru * du;
        if (r < 6) {
            if (r >= 3) {
#pragma unroll
                for (int l = 0; l < 4; ++l) lxd += lx_.xq[l] * S.dx[12 + 3 * l + r - 3];
            }
        } else if (r < 9) {
#pragma unroll
            for (int c = 0; c < 12; ++c) bdu += lq[bw_at(r - 6, c)] * S.du[c];
        } else if (r < 12) {
#pragma unroll
            for (int l = 0; l < 4; ++l) bdu += pc.bv[l] * S.du[3 * l + r - 9];
        } else {
            bdu = pick4(pc.bq, (r - 12) / 3) * S.du[r];
            lxd += lx_.xp * S.dx[3 + (r - 12) % 3];
        }
        if (r < 12) {
            const real *rb = lq + LQ_RB + 6 * (r / 3);
            const int a = r % 3, u0 = 3 * (r / 3);
            const real b0 = a == 0 ? rb[0] : a == 1 ? rb[1] : rb[2];
            const real b1 = a == 0 ? rb[1] : a == 1 ? rb[3] : rb[4];
            const real b2 = a == 0 ? rb[2] : a == 1 ? rb[4] : rb[5];
            lud += b0 * S.du[u0] + b1 * S.du[u0 + 1] + b2 * S.du[u0 + 2];
        }
        nx = (dx + sdx) + bdu + dd[r];
        q1 = lq[LQ_LX + r] * dx + lq[LQ_LU + r] * du;
        q2 = dx * lxd + du * lud;
        if (st) {
            const size_t kq = b * p.Kc + kc;
            d.du[kq * NX + r] = du;
            d.dX[(b * p.S + s + 1) * NX + r] = nx;
        }
    }
    v1 += half_sum(q1);
    v2 += half_sum(q2);
    dx = nx;
    LSYNC();
}

template <typename real, bool EL>
__global__ __launch_bounds__(64) void k_lin_rollout(Params p, Bufs d)
{
    __shared__ LinElem<real> S;
    __shared__ LinBuf<real> B0;
    __shared__ LinBuf<real> B1;
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5, cb = HC * hf;
    const size_t b = blockIdx.x;
    ElemState &E = d.el[b];
    if (E.done || E.inner_done) return;
    const bool rowl = r < NX, st = rowl && hf == 0;
    const int rr = rowl ? r : 0;
    const real *defg = Prec<real>::def(d);
    real v1 = 0, v2 = 0, dx = 0;
    const auto LY = layout_of<EL>(d, (int)b);
    const int P = LY.P();
    for (int i = 0; i < P; ++i) {
        PhaseConst<real> pc;
        load_phase(p, d, b, i, pc);
        const int N = LY.N(i), s0 = LY.s0(i), k0 = LY.k0(i);
        lin_fetch(B0, p, d, b, s0, k0, lane);  // the phase's first knot (its wait is in lin_knot)
        if (i > 0) { // dx_init = Px dX_end
            const double *Px = d.term + (b * p.P + (i - 1)) * TW + TM_PX;
            if (lane < NX) S.dx[lane] = dx;
            LSYNC();
            real a = 0;
            if (rowl)
                for (int j = 0; j < NX; ++j) a += (real)Px[r * NX + j] * S.dx[j];
            dx = a;
            LSYNC();
        } else {
            dx = 0;
        }
        if (rowl) {
            dx = dx + defg[(b * p.S + s0) * NX + r];
            if (st) d.dX[(b * p.S + s0) * NX + r] = dx;
        }
        // lxx row r (HKDCost.cpp:32): diagonal + foot cross terms
        LxxRow<real> lx_;
        lxx_row(p, pc, r, lx_);
        const real ru = rowl ? (real)(p.dt * r_diag(p, r)) : (real)0;
        // control r has a gain row only when its B column is non-zero (KCW layout)
        const bool stl = contact(pc, (rr % HC) / 3) != 0;
        const bool cpl = rowl && (rr < HC ? stl : !stl);
        const int krow0 = (rr % HC) * NX + cb;
        for (int k = 0; k < N; k += 2) {
            lin_knot(p, d, S, B0, B1, k + 1 < N, b, s0 + k, k0 + k, pc, lx_, ru, cpl, krow0, dx, v1, v2);
            if (k + 1 < N)
                lin_knot(p, d, S, B1, B0, k + 2 < N, b, s0 + k + 1, k0 + k + 1, pc, lx_, ru, cpl, krow0, dx, v1, v2);
        }
        const double *rec = d.term + (b * p.P + i) * TW;
        if (lane < NX) S.dx[lane] = dx;
        LSYNC();
        real q1 = 0, q2 = 0;
        if (rowl) {
            q1 = (real)rec[TM_PHIX + r] * dx;
            real a = 0;
            for (int c = 0; c < NX; ++c) a += (real)rec[TM_PHIXX + r * NX + c] * S.dx[c];
            q2 = dx * a;
        }
        v1 += half_sum(q1);
        v2 += half_sum(q2);
        LSYNC();
    }
    if (lane == 0) {
        const double cost = E.cost, feas = E.feas, w1 = v1, w2 = v2;
        const double dV_abs = fabs(w1 + 0.5 * w2);
        const double rho = (feas > p.feas_thresh) ? dV_abs / ((1 - p.merit_scale) * feas) + p.merit_offset : 0;
        const double merit = cost + rho * feas;
        E.dV1 = w1; E.dV2 = w2; E.merit_rho = rho; E.merit = merit;
        E.cost_prev = cost; E.merit_prev = merit; E.feas_prev = feas;
        if (!p.no_early_exit && dV_abs < p.cost_thresh && feas <= p.feas_thresh) { E.inner_done = 1; E.ls_active = 0; }
        else E.ls_active = 1;
    }
}

void launch_lin_rollout(const Params &p, const Bufs &d, hipStream_t st)
{
    if (p.fp32) {
        if (p.elem_layout) hipLaunchKernelGGL((k_lin_rollout<float, true>), dim3(p.B), dim3(64), 0, st, p, d);
        else hipLaunchKernelGGL((k_lin_rollout<float, false>), dim3(p.B), dim3(64), 0, st, p, d);
    } else {
        if (p.elem_layout) hipLaunchKernelGGL((k_lin_rollout<double, true>), dim3(p.B), dim3(64), 0, st, p, d);
        else hipLaunchKernelGGL((k_lin_rollout<double, false>), dim3(p.B), dim3(64), 0, st, p, d);
    }
}

}  // namespace hsddp
