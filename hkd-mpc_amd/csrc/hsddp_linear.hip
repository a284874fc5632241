// hsddp_linear.hip — the multiple-shooting linear rollout that follows a successful sweep.
//
// MultiPhaseDDP::linear_rollout (HSDDPSolver/source/MultiPhaseDDP.cpp:20-50) over
// SinglePhase::linear_rollout (SinglePhase.cpp:144-178), then the merit function
// (MultiPhaseDDP.cpp:309-318), two elements per wave: dX, du = dU + K dX, and the expected cost
// change of quirk A3 (it replaces the sweep's dV).  Templates on `real` as the sweep
// (hsddp_sweep.hip): double, or float in config C5's fp32 mode.
#include "hsddp_wave.h"

namespace hsddp {

using namespace hkd;

constexpr int HC = 12;  // coupled controls per knot

#ifndef HSDDP_STAMPS
#define HSDDP_STAMPS 0
#endif
#ifndef HSDDP_LIN_EXP
#define HSDDP_LIN_EXP 0  // timing experiments only: 1 no dX / du stores, 2 no arithmetic, 3 no decoupled du stores
#endif
// the knot images requested with the non-temporal policy: the iteration's last read of K, the
// records and dU (0.82 -> 0.73 ms on one box; the sweep's image requests, which the linear rollout
// reads again, stay default: nt there cost the rollout 0.045 ms)
#ifndef HSDDP_LIN_NT
#define HSDDP_LIN_NT 1
#endif
// Diagnostic build (make stamps): s_memtime at the stage boundaries of a knot, differences summed
// per stage into LDS and written to Bufs::dbg of the wave's second element (tools/stamps.py)
#if HSDDP_STAMPS
struct LinStamps {
    unsigned long long st[8], tprev;
};
DEV LinStamps &lin_stamps()
{
    __shared__ LinStamps s;
    return s;
}
#define LSTAMP(n)                                                                             \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        unsigned long long t_;                                                                \
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        if (threadIdx.x == 0) {                                                               \
            if ((n) > 0) lin_stamps().st[n] += t_ - lin_stamps().tprev;                       \
            lin_stamps().tprev = t_;                                                          \
        }                                                                                     \
    } while (0)
#else
#define LSTAMP(n) \
    do {          \
    } while (0)
#endif

// Per-precision buffers: LQ record (stride LQS), compact gains and the Defect copy the sweep reads.
template <typename real> struct Prec;
template <> struct Prec<double> {
    static constexpr int LQS = LQW;
    static DEV const double *lq(const Bufs &d) { return d.lq; }
    static DEV double *K(const Bufs &d) { return d.K; }
    static DEV const double *def(const Bufs &d, int b) { return kdbuf(work_buf(d, b)); }  // the working rows' Defect (kernel (Params, Bufs, ...))
};
template <> struct Prec<float> {
    static constexpr int LQS = LQW32;
    static DEV const float *lq(const Bufs &d) { return d.lq32; }
    static DEV float *K(const Bufs &d) { return d.K32; }
    static DEV const float *def(const Bufs &d, int) { return d.def32; }  // (k_lq's copy of the working Defect)
};

// per-phase constants of one element
template <typename real>
struct PhaseConst {
    int c[4];
    int cmask;   // bit l = c_l: a lane-dependent leg index becomes one shift, not a select chain
    real bv[4];  // dt c_l / m     (B rows 9..11)
    real bq[4];  // dt (1 - c_l)   (B rows 12..23)
};

// Both elements' contacts through the scalar cache, then this half's by selects; dt * c / m is
// dt / m or 0 exactly for c in {0, 1}.
template <typename real>
DEV void load_phase(const Params &p, const Bufs &d, const size_t (&b)[2], int hf, int i, PhaseConst<real> &pc)
{
    typedef const __attribute__((address_space(4))) int cint;
    cint *c0 = (cint *)(d.contacts + (b[0] * (p.P + 1) + i) * 4), *c1 = (cint *)(d.contacts + (b[1] * (p.P + 1) + i) * 4);
    pc.cmask = 0;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const int a0 = c0[l], a1 = c1[l];
        pc.c[l] = hf ? a1 : a0;
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
// MultiPhaseDDP::linear_rollout(1.0): dX, du = dU + K dX, and the expected cost change (quirk A3:
// it replaces the sweep's dV), then the merit function (MultiPhaseDDP.cpp:309-318).
// Two elements per wave, one per half-wave (the sweep's pairing, hsddp_sweep.hip): lane r < 24 of
// half h computes row r of element h's vectors.  A knot's inputs (compact K, LQ record,
// Defect[k+1], dU) are one LDS image per element (4080 bytes in fp64, 2144 in the fp32 mode) filled
// by 16-byte-per-lane LDS-DMA loads (global_load_lds_dwordx4, four or three instructions per
// element); the next knot's images are loaded into the other buffer while this knot computes.  The
// per-lane DMA sources advance by a fixed per-segment stride from knot to knot, and a knot's dX /
// du stores are issued after the next knot's DMA so that the wait for the current image never
// waits for them.
template <typename real>
struct LinImg {
    static constexpr int K = 0;                                       // byte offsets
    static constexpr int LQ = K + KCW * (int)sizeof(real);
    static constexpr int D = LQ + Prec<real>::LQS * (int)sizeof(real);
    static constexpr int DU = D + NX * (int)sizeof(real);
    static constexpr int END = DU + NX * 8;                           // dU stays fp64
    static constexpr int NI = (END / 16 + 63) / 64;                   // DMA instructions per element
    static_assert(LQ % 16 == 0 && D % 16 == 0 && DU % 16 == 0 && END % 16 == 0 && (NI == 4 || NI == 3), "16-byte pieces");
};
template <typename real>
struct LinBuf {
    alignas(16) char v[2][LinImg<real>::NI * 1024];  // element h's image at v[h]
};
// dX / du rows of the current knot (slots 24..31 stay zero: the index of an absent term) and a
// zero region standing for the coefficients of structurally absent terms
constexpr int LZ = 31;  // a zero slot of dx / du
template <typename real>
struct LinVec {
    real dx[2][32], du[2][32];
    real zero[64];
};

// This lane's LDS-DMA sources: piece 64 j + lane of each element's image (spare pieces repeat the
// last), and the per-knot stride of the segment the piece lies in.
template <typename real>
struct LinSrc {
    using I = LinImg<real>;
    const char *p[2][I::NI];
    unsigned step[I::NI];

    static DEV int piece(int j, int lane)
    {
        const int o = 16 * (64 * j + lane);
        return o < I::END ? o : I::END - 16;
    }
    DEV void init(const Params &pr, const Bufs &d, const size_t (&b)[2], int s, int kc, int lane)
    {
#pragma unroll
        for (int j = 0; j < I::NI; ++j) {
            const int o = piece(j, lane);
            step[j] = o < I::LQ ? KCW * sizeof(real) : o < I::D ? Prec<real>::LQS * sizeof(real) : o < I::DU ? NX * sizeof(real) : NX * 8;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const size_t kq = b[h] * pr.Kc + kc;
                const char *base = o < I::LQ ? (const char *)(Prec<real>::K(d) + kq * KCW) - I::K
                                 : o < I::D  ? (const char *)(Prec<real>::lq(d) + kq * Prec<real>::LQS) - I::LQ
                                 : o < I::DU ? (const char *)(Prec<real>::def(d, (int)b[h]) + (b[h] * pr.S + s + 1) * NX) - I::D
                                             : (const char *)(d.dU + kq * NX) - I::DU;
                p[h][j] = base + o;
            }
        }
    }
    DEV void advance()
    {
#pragma unroll
        for (int j = 0; j < I::NI; ++j) {
            p[0][j] += step[j];
            p[1][j] += step[j];
        }
    }
};

// Issued as inline asm so the waitcnt pass does not track the LDS writes (it would otherwise wait
// for every DMA in flight before any LDS read); lin_knot waits explicitly.  LDS destination of
// element h's piece 64 j + lane: v[h] + 1024 j + 16 lane.
template <typename real>
DEV void lin_fetch(LinBuf<real> &buf, const LinSrc<real> &src)
{
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int j = 0; j < LinImg<real>::NI; ++j) {
            if (HSDDP_LIN_NT) lds_dma16_nt(src.p[h][j], (unsigned)(size_t)(buf.v[h] + 1024 * j));
            else lds_dma16(src.p[h][j], (unsigned)(size_t)(buf.v[h] + 1024 * j));
        }
}

template <int W>
DEV void vm_wait()
{
    if constexpr (W == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (W == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (W == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (W == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if constexpr (W == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if constexpr (W == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (W == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else static_assert(W < 0, "wait count");
}

// wait until at most n vector memory operations are outstanding, n in {0, 2, 4, NI2, NI2 + 2,
// NI2 + 4} (a runtime choice among immediates; larger n: the conservative 0)
template <int NI2>
DEV void vm_wait_n(int n)
{
    if (n == NI2 + 4) vm_wait<NI2 + 4>();
    else if (n == NI2 + 2) vm_wait<NI2 + 2>();
    else if (n == NI2) vm_wait<NI2>();
    else if (n == 4) vm_wait<4>();
    else if (n == 2) vm_wait<2>();
    else vm_wait<0>();
}

// per-lane constants of one phase: every row's terms as one branch-free formula, a structurally
// absent term reading a zero coefficient (LinVec::zero) or the zero slot LZ of dx / du
template <typename real>
struct LinRow {
    PhaseConst<real> pc;
    LxxRow<real> lx;
    real ru;
    bool cpl;   // control r has a coupled gain row (KCW layout)
    int krow0;  // its first entry in the K image
    bool use_se, use_sw, use_rb;  // rows 0..2: A - I eul row; rows 6..8: A - I omega row, BW row; rows < 12: ReB block
    int se0, sw0, rb0, rbi[3];    // record offsets of those rows (rb: the leg's block, entry (r % 3, b))
    real c3;                      // rows 3..5: dt (dX[r + 6]); else 0
    int i3;                       // r + 6, or LZ
    real cx[4];                   // lxx cross terms: rows 3..5 xq[l] (dX[12 + 3 l + r - 3]), rows >= 12 xp (dX[3 + (r - 12) % 3])
    int ix[4];
    real cu[4];                   // rows 9..11: bv[l] (du[3 l + r - 9])
    int iu[4];
    real cq;                      // rows >= 12: dt (1 - c) on the lane's own du
    int iru;                      // rows < 12: first du of the leg's block (3 (r / 3)), else LZ
};

template <typename real>
DEV void lin_row(const Params &p, LinRow<real> &R, int r)
{
    const int rr = r < NX ? r : 0;
    R.use_se = r < 3;
    R.use_sw = r >= 6 && r < 9;
    R.use_rb = r < 12;
    R.se0 = LQ_SE + 5 * (r < 3 ? r : 0);
    R.sw0 = r >= 6 && r < 9 ? r - 6 : 0;
    R.rb0 = LQ_RB + 6 * ((r < 12 ? r : 0) / 3);
    const int a = (r < 12 ? r : 0) % 3;
#pragma unroll
    for (int b = 0; b < 3; ++b) R.rbi[b] = a == 0 ? b : a == 1 ? (b == 0 ? 1 : b == 1 ? 3 : 4) : (b == 0 ? 2 : b == 1 ? 4 : 5);
    R.iru = r < 12 ? 3 * (r / 3) : LZ;
    R.c3 = (r >= 3 && r < 6) ? (real)p.dt : (real)0;
    R.i3 = (r >= 3 && r < 6) ? r + 6 : LZ;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const bool pos = r >= 3 && r < 6, q = r >= 12 && r < NX;
        R.cx[l] = pos ? R.lx.xq[l] : (q && l == 0) ? R.lx.xp : (real)0;
        R.ix[l] = pos ? 12 + 3 * l + r - 3 : (q && l == 0) ? 3 + (r - 12) % 3 : LZ;
        const bool v = r >= 9 && r < 12;
        R.cu[l] = v ? R.pc.bv[l] : (real)0;
        R.iu[l] = v ? 3 * l + r - 9 : LZ;
    }
    R.cq = (r >= 12 && r < NX) ? pick4(R.pc.bq, (rr - 12) / 3) : (real)0;
}

// a knot's dX / du rows, stored one knot later
template <typename real>
struct LinOut {
    double *du, *dx;  // this lane's entries of the pending knot
    real vu, vx;      // the pending knot's values
    int n;            // pending knots (0 or 1)
    int nprev;        // store instructions the previous knot issued after its image requests
    bool ust;         // this lane stores its du entry
};

template <typename real>
DEV void lin_push(LinOut<real> &out, real du, real nx)
{
    out.vu = du;
    out.vx = nx;
    out.n = 1;
}

// the pending knot's rows (when `go`); returns the store instructions issued
template <typename real>
DEV int lin_store_pending(bool go, bool st, LinOut<real> &out)
{
#if HSDDP_LIN_EXP == 1
    go = false;
#endif
    if (!go || out.n == 0) return 0;
    out.n = 0;
    if (st) {
        if (out.ust) *out.du = (double)out.vu;
        *out.dx = (double)out.vx;
    }
    out.du += NX;
    out.dx += NX;
    return 2;
}

template <typename real>
DEV void lin_knot(const Params &p, LinVec<real> &S, LinBuf<real> &cur, LinBuf<real> &nxt, bool more, bool pend,
                  LinSrc<real> &src, const LinRow<real> &R, bool st, LinOut<real> &out, real &dx, real &q1s, real &q2s)
{
    using I = LinImg<real>;
    constexpr int NI2 = 2 * I::NI;
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5;
    const bool rowl = r < NX;
    const int rr = rowl ? r : 0;
    LSTAMP(0);
    if (more) {
        src.advance();
        lin_fetch(nxt, src);
    }
    const int ns = lin_store_pending(pend, st, out);
    // every vector memory operation up to this knot's image: all but the ones issued after it (the
    // stores the previous knot issued behind this image's requests, the 2 NI DMA of the next knot and
    // the stores just issued; operations complete in issue order, so a store waited for here would
    // only delay the image).  The stores left in flight are older than the next knot's image.
    vm_wait_n<NI2>(out.nprev + (more ? NI2 : 0) + ns);
    out.nprev = ns;
    LSYNC();
    LSTAMP(1);
#if HSDDP_LIN_EXP == 2
    {
        const real v = ((const real *)cur.v[hf])[r];
        lin_push(out, v, v);
        dx = v;
        return;
    }
#endif
    const char *img = cur.v[hf];
    const real *kimg = (const real *)(img + I::K), *lq = (const real *)(img + I::LQ), *dd = (const real *)(img + I::D);
    const double *dUi = (const double *)(img + I::DU);
    real *sdxv = S.dx[hf], *sduv = S.du[hf];
    // every coefficient of the knot read at once (one LDS wait, not one per multiply-add); an absent
    // term's coefficient comes from the zero region
    const real *kp = R.cpl ? kimg + R.krow0 : S.zero;
    const real *sep = R.use_se ? lq + R.se0 : S.zero, *swp = R.use_sw ? lq + LQ_SW + R.sw0 : S.zero;
    const real *bwp = R.use_sw ? lq + LQ_BW + R.sw0 : S.zero, *rbp = R.use_rb ? lq + R.rb0 : S.zero;
    const real *lxp = rowl ? lq + LQ_LX : S.zero, *lup = rowl ? lq + LQ_LU : S.zero;
    real krow[NX], cse[5], csw[17], cbw[12], crb[3];
#pragma unroll
    for (int c = 0; c < NX; ++c) krow[c] = kp[c];
    const real dUr = (real)dUi[rr];
#pragma unroll
    for (int q = 0; q < 5; ++q) cse[q] = sep[5 * 0 + q];
#pragma unroll
    for (int q = 0; q < 17; ++q) csw[q] = swp[3 * q];
    const real ddr = (rowl ? dd : S.zero)[rr], lxr = lxp[rr], lur = lup[rr];
    if (rowl) sdxv[r] = dx;  // for the terms with lane-dependent columns below
    // dX of this half's rows at every lane by DPP position (dxa: rows 0..15, dxb: rows 16..23):
    // the products with compile-time columns take it by row broadcast, not from LDS
    real dxa, dxb;
    row_pair(dx, dxa, dxb);
    asm volatile("" : "+v"(dxa), "+v"(dxb));
    asm volatile("s_nop 1");  // DPP sources just written by the permlane swaps
    pin(krow);
    // K dX as two 12-column sums (the order of the one-element-per-wave kernel's two halves)
    real k0 = 0, k1 = 0;
    static_for<HC>([&](auto C) {
        constexpr int c = C, c1 = HC + C;
        bfma<c>(k0, dxa, krow[c]);
        if constexpr (c1 < 16) bfma<c1>(k1, dxa, krow[c1]);
        else bfma<c1 - 16>(k1, dxb, krow[c1]);
    });
    const real du = dUr + (k0 + k1);
    LSTAMP(2);
    SFENCE();  // the second batch of coefficient reads after K dX (not hoisted: registers)
#pragma unroll
    for (int q = 0; q < 12; ++q) cbw[q] = bwp[3 * q];
#pragma unroll
    for (int b = 0; b < 3; ++b) crb[b] = rbp[R.rbi[b]];
    if (rowl) sduv[r] = du;
    // dX terms with lane-dependent columns (rows 3..5: dt dX[r + 6]; lxx cross terms)
    const real x3 = sdxv[R.i3];
    real xc[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) xc[l] = sdxv[R.ix[l]];
    // A - I rows 0..2 (SE) and 6..8 (SW), zero coefficients on the other rows
    pin(cse);
    pin(csw);
    real se = 0, sw = 0;
    static_for<5>([&](auto Q) { bfma<se_col(Q)>(se, dxa, cse[Q]); });
    static_for<17>([&](auto Q) {
        constexpr int col = sw_col(Q);
        if constexpr (col < 16) bfma<col>(sw, dxa, csw[Q]);
        else bfma<col - 16>(sw, dxb, csw[Q]);
    });
    real dua, dub;
    row_pair(du, dua, dub);
    asm volatile("" : "+v"(dua), "+v"(dub));
    asm volatile("s_nop 1");
    pin(cbw);
    real bw = 0;  // B rows 6..8 (BW) times du, columns 0..11
    static_for<12>([&](auto C) { bfma<C>(bw, dua, cbw[C]); });
    (void)dub;
    LSYNC();
    LSTAMP(3);
    // du terms with lane-dependent columns (rows 9..11: bv du of the legs' GRF; rows < 12: ReB block)
    real uc[4], ur[3];
#pragma unroll
    for (int l = 0; l < 4; ++l) uc[l] = sduv[R.iu[l]];
#pragma unroll
    for (int b = 0; b < 3; ++b) ur[b] = sduv[R.iru < LZ ? R.iru + b : LZ];
    // one formula for every row: absent terms add exact zeros
    const real sdx = (se + sw) + R.c3 * x3;
    real lxd = R.lx.diag * dx;
#pragma unroll
    for (int l = 0; l < 4; ++l) lxd += R.cx[l] * xc[l];
    real bdu = bw;
#pragma unroll
    for (int l = 0; l < 4; ++l) bdu += R.cu[l] * uc[l];
    bdu += R.cq * du;
    const real lud = R.ru * du + (crb[0] * ur[0] + crb[1] * ur[1] + crb[2] * ur[2]);
    const real nx = rowl ? ((dx + sdx) + bdu) + ddr : (real)0;
    q1s += lxr * dx + lur * du;
    q2s += dx * lxd + du * lud;
    lin_push(out, du, nx);
    dx = nx;
    LSYNC();
    LSTAMP(4);
}

template <typename real, bool EL>
__global__ __launch_bounds__(64, 2) void k_lin_rollout(Params p, Bufs d)
{
    __shared__ LinVec<real> S;
    __shared__ LinBuf<real> B0;
    __shared__ LinBuf<real> B1;
    const int lane = threadIdx.x, r = lane & 31, hf = lane >> 5;
    // the wave's two elements (as k_riccati): 2 blockIdx + h, or a pair of elements with one
    // layout (Bufs::pairs); an empty half runs on the other half's element, inactive
    size_t eb[2];
    bool valid;
    if constexpr (EL) {
        const int e0 = d.pairs[2 * blockIdx.x], e1 = d.pairs[2 * blockIdx.x + 1];
        eb[0] = e0;
        eb[1] = e1 >= 0 ? e1 : e0;
        valid = hf == 0 || e1 >= 0;
    } else {
        const int e0 = 2 * blockIdx.x, e1 = e0 + 1;
        eb[0] = e0;
        eb[1] = e1 < p.B ? e1 : e0;
        valid = hf == 0 || e1 < p.B;
    }
    const size_t b = hf ? eb[1] : eb[0];
    ElemState &E = d.el[b];
    const bool act = valid && !E.done && !E.inner_done;
    if (!__builtin_amdgcn_ballot_w64(act)) return;
    const bool rowl = r < NX, st = rowl && act;
    const int rr = rowl ? r : 0;
    const real *defg = Prec<real>::def(d, (int)b);
    S.zero[lane] = 0;
    S.dx[hf][r] = 0;
    S.du[hf][r] = 0;
#if HSDDP_STAMPS
    if (lane < 8) lin_stamps().st[lane] = 0;
#endif
    __syncthreads();
    real v1 = 0, v2 = 0, dx = 0;
    const auto LY = layout_of<EL>(d, (int)eb[0]);
    const int P = LY.P();
    LinOut<real> out{};
    for (int i = 0; i < P; ++i) {
        const int N = LY.N(i), s0 = LY.s0(i), k0 = LY.k0(i);
        LinSrc<real> src;
        src.init(p, d, eb, s0, k0, lane);
        lin_fetch(B0, src);  // the phase's first knot (its wait is in lin_knot)
        out.nprev = 0;       // (the stores of earlier knots are older than this image)
        LinRow<real> R;
        load_phase(p, d, eb, hf, i, R.pc);
        if (i > 0) { // dx_init = Px dX_end
            const double *Px = d.term + (b * p.P + (i - 1)) * TW + TM_PX;
            if (rowl) S.dx[hf][r] = dx;
            LSYNC();
            real a = 0;
            if (rowl)
                for (int j = 0; j < NX; ++j) a += (real)Px[r * NX + j] * S.dx[hf][j];
            dx = a;
            LSYNC();
        } else {
            dx = 0;
        }
        if (rowl) dx = dx + defg[(b * p.S + s0) * NX + r];
        if (st) d.dX[(b * p.S + s0) * NX + r] = dx;
        // lxx row r (HKDCost.cpp:32): diagonal + foot cross terms
        lxx_row(p, R.pc, r, R.lx);
        R.ru = rowl ? (real)(p.dt * r_diag(p, r)) : (real)0;
        // control r has a gain row only when its B column is non-zero (KCW layout)
        const bool stl = contact(R.pc, (rr % HC) / 3) != 0;
        R.cpl = rowl && (rr < HC ? stl : !stl);
        R.krow0 = (rr % HC) * NX;
        lin_row(p, R, r);
        out.ust = HSDDP_LIN_EXP == 3 ? R.cpl : true;  // (3: timing only, the decoupled du entries not stored)
        out.du = d.du + (b * p.Kc + k0) * NX + rr;
        out.dx = d.dX + (b * p.S + s0 + 1) * NX + rr;
        real q1s = 0, q2s = 0;
        for (int k = 0; k < N; k += 2) {
            lin_knot(p, S, B0, B1, k + 1 < N, k > 0, src, R, st, out, dx, q1s, q2s);
            if (k + 1 < N) lin_knot(p, S, B1, B0, k + 2 < N, true, src, R, st, out, dx, q1s, q2s);
        }
        lin_store_pending(true, st, out);  // the phase's last knots
        const double *rec = d.term + (b * p.P + i) * TW;
        if (rowl) S.dx[hf][r] = dx;
        LSYNC();
        if (rowl) {
            q1s += (real)rec[TM_PHIX + r] * dx;
            real a = 0;
            for (int c = 0; c < NX; ++c) a += (real)rec[TM_PHIXX + r * NX + c] * S.dx[hf][c];
            q2s += dx * a;
        }
        v1 += half_sum(q1s);
        v2 += half_sum(q2s);
        LSYNC();
    }
#if HSDDP_STAMPS
    __syncthreads();
    if (lane < 8) d.dbg[(size_t)__builtin_amdgcn_readfirstlane((int)eb[1]) * 16 + 8 + lane] += lin_stamps().st[lane];
#endif
    if (r == 0 && act) merit_step(p, E, v1, v2);
}

void launch_lin_rollout(const Params &p, const Bufs &d, hipStream_t st)
{
    const dim3 g((unsigned)(p.elem_layout ? p.n_pairs : (p.B + 1) / 2));
    if (p.fp32) {
        if (p.elem_layout) hipLaunchKernelGGL((k_lin_rollout<float, true>), g, dim3(64), 0, st, p, d);
        else hipLaunchKernelGGL((k_lin_rollout<float, false>), g, dim3(64), 0, st, p, d);
    } else {
        if (p.elem_layout) hipLaunchKernelGGL((k_lin_rollout<double, true>), g, dim3(64), 0, st, p, d);
        else hipLaunchKernelGGL((k_lin_rollout<double, false>), g, dim3(64), 0, st, p, d);
    }
}

}  // namespace hsddp
