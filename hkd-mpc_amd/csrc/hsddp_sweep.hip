// hsddp_sweep.hip — the regularised backward Riccati sweep, two elements per wave (gfx950).
//
// MultiPhaseDDP::backward_sweep_regularized / backward_sweep (HSDDPSolver/source/
// MultiPhaseDDP.cpp:141-229) over SinglePhase::backward_sweep (SinglePhase.cpp:298-367), with the
// impact-aware value transfer (MultiPhaseDDP.cpp:480-484), for B independent elements.
//
// Mapping.  One 64-lane wave sweeps two elements ("items"), one per half-wave: lane L works on
// item e = L >> 5 at position p = L & 31.  Both halves run the same instruction stream on their
// own data, so nothing branches on the half.  Position p < 24 owns row p of the value Hessian H
// (24 doubles in registers, carried from knot to knot) and, after the column exchange through
// LDS, column p of M = H A and of Qux; position 24 carries the vector terms (S^T Gn, Qu).
//
// Coefficients.  A knot's LQ record and Defect[k+1] arrive in LDS by LDS-DMA (requested during
// the previous knot's elimination).  The 128 values every lane multiplies by — A - I (69
// non-zeros), B's omega rows (36), Defect (24) — are spread over the 16 lanes of each DPP row,
// eight registers per lane, and enter the multiply-adds through row_newbcast broadcasts
// (v_fmac_f64_dpp): a broadcast coefficient costs no instruction, and the sparsity of A and B is
// compile-time, so each product issues exactly its non-zero multiply-adds.
//
// Per knot (row r of the element on each lane, all sums over the structural non-zeros):
//   Gn = G + H d;  T = H B_c;  M = H A                         (rows in registers)
//   M, T rows -> LDS; lane c reads column c of M
//   Z = M + (S^T M)^T (row c);  Qux_c column c = B_c^T M[:, c];  position 24: S^T Gn, Qu_c
//   Qxx = lxx + reg I + (Z + Z^T) / 2  (each lane adds lxx, reg to its own Z row in LDS; transposed
//                                       read)
//   Quu_cc column q = luu + reg + B_c^T T[:, q]    (T columns from LDS)
//   the next knot's images requested by LDS-DMA
//   elimination on [Quu_cc | Qux_c | Qu_c] in LDL^T order (12 pivot steps, pivots by DPP
//   broadcast, the next pivot's reciprocal threaded through the current step), back substitution
//   K = -Quu_cc^-1 Qux_c, dU, G = Qx - Qux_c^T Quu_cc^-1 Qu_c  (the sweep's dV is formed only with
//   single shooting, DV: with MS the linear rollout replaces it, quirk A3)
//   H = Qxx - Qux_c^T Quu_cc^-1 Qux_c by DPP broadcast of K from the lanes holding it
//   (HSDDP_VALUE_MFMA = 1: on the matrix cores, v_mfma_f64_16x16x4_f64, symmetric tiles)
//   K rows and dU stored after one wait for all vector memory operations (nothing waits on them)
// Only the 12 coupled controls (those whose B column is non-zero, DESIGN.md §3.1 "Decoupled controls") enter
// the elimination; the other 12 are decoupled: K row 0, dU = -lu / (dt R + reg), exactly as the
// reference's dense 24-control solve gives them.  PSD test: every elimination pivot of Quu_cc and
// every decoupled diagonal must exceed 1e-9 (the reference's LDLT of Quu - 1e-9 I).
//
// Templates on `real`: double (the reference's T = double) and float (config C5's fp32 mode).
#include "hsddp_wave.h"

namespace hsddp {

using namespace hkd;

namespace sweep {

#ifndef HSDDP_STAMPS
#define HSDDP_STAMPS 0
#endif
// value update on the matrix cores (1) or by DPP-broadcast multiply-adds from the lanes holding
// K_c (0, no LDS round trip)
// waves per SIMD the two-pair workgroups' register budget is sized for: 1 (their launches have at
// most one wave per SIMD: the spills go to AGPRs, not scratch)
#ifndef SWEEP_WPB2_WPE
#define SWEEP_WPB2_WPE 1
#endif
// knot images requested with the non-temporal policy (A/B experiment)
#ifndef HSDDP_SWEEP_NT
#define HSDDP_SWEEP_NT 0
#endif
#ifndef HSDDP_VALUE_MFMA
#define HSDDP_VALUE_MFMA 0
#endif
// In-kernel stamps (diagnostic build only, make stamps): s_memtime at the stage boundaries of a
// knot (each after a full LDS drain, so stages do not overlap), differences summed per stage into
// LDS and written to Bufs::dbg of the wave's first element (tools/stamps.py).
#if HSDDP_STAMPS
#define STAMP(n)                                                                              \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        unsigned long long t_;                                                                \
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        if (threadIdx.x == 0) {                                                               \
            if ((n) > 0) S.st[n] += t_ - S.tprev;                                             \
            S.tprev = t_;                                                                     \
        }                                                                                     \
    } while (0)
#else
#define STAMP(n) \
    do {         \
    } while (0)
#endif

// stage boundary: LDS accesses stay in their stage and the scheduler does not interleave stages
// (which would keep both stages' operands live)
#define SSYNC()                              \
    do {                                     \
        asm volatile("" ::: "memory");       \
        __builtin_amdgcn_sched_barrier(0);   \
    } while (0)

constexpr int HC = 12;        // coupled controls per knot
constexpr int MS = 26;        // M / Z / P image row stride (reals): conflict-free rows and columns
constexpr int TS = 14;        // T / Qux^T / Kp^T image row stride
constexpr int WS = 25;        // W image row stride (phase boundary)
// coefficient vector V of a knot image: record [0, 104) = SE | SW | BW, then Defect[k+1] (24), then
// record [104, 176) = LX | LU | RB
constexpr int V_SE = LQ_SE, V_D = 104, V_LX = 128, V_LU = 152, V_RB = 176, VW = 200;
static_assert(LQ_BW + 36 == V_D && LQ_LX + 24 == V_LX && LQ_LU + 24 == V_LU && LQ_RB + 24 == V_RB, "image layout");

template <typename real>
struct alignas(16) Lds {
    real img[2][VW];               // knot images of the two items (one DMA target)
    real zero[32];                 // exact zeros: reads standing for structurally absent entries
    struct alignas(16) Item {
        real TI[24 * TS];          // T rows, then Qux^T rows (25: row 24 = Qu_c)
        real MI[25 * MS];          // M rows (col 24 = Gn) -> Z rows (row 24 = S^T Gn) -> Kp^T rows -> P rows; W at phase ends
        real du[24];
        real pc[8];                // bv[4], bq[4] of the phase
    } it[2];
#if HSDDP_STAMPS
    unsigned long long st[12], tprev;  // diagnostic build: cycles per knot stage
#endif
};
static_assert(sizeof(Lds<double>) <= 20480, "two waves per SIMD on 160 KB of LDS need <= 20 KB per wave");

// The column split (k_riccati_cs, small batches): one element pair over the two waves of a
// workgroup, which share this LDS.  Knot images double-buffered (a wave requests the next knot's
// while the other may still read the current one); per item, two 25-row images that trade roles
// from knot to knot: M rows, then (after the column reads) this knot's H exchange, while the other
// holds the Z rows — so every image is rewritten only after a barrier both waves have passed since
// its last read.
template <typename real>
struct alignas(16) LdsCS {
    real img[2][2][VW];            // [buffer][item]
    real zero[32];
    struct alignas(16) Item {
        real TI[24 * TS];          // T rows (columns: the controls of both waves)
        real MZ[2][25 * MS];       // M rows -> H exchange | Z rows; W at phase ends (MZ[0])
        real du[24];
        real pc[8];
    } it[2];
    int fl[2];                     // the retry slot wave 0 took for each item
};
static_assert(sizeof(LdsCS<double>) <= 40960, "four split workgroups per CU on 160 KB of LDS need <= 40 KB each");

// knot image pieces (16 bytes) of one item: the record's coefficient part, Defect[k+1], the rest
template <typename real>
struct Pieces {
    static constexpr int E = 16 / sizeof(real);
    static constexpr int NA = V_D / E, ND = NX / E, NR = (LQW - V_D) / E, NP = NA + ND + NR;
    static constexpr int NI = (2 * NP + 63) / 64;  // DMA instructions per wave
    static_assert(NP * E == VW && V_D % E == 0, "16-byte pieces");
};

template <typename real> struct Prec;
template <> struct Prec<double> {
    static DEV const double *lq(const Bufs &d) { return d.lq; }
    static DEV double *K(const Bufs &d) { return d.K; }
    static DEV const double *def(const Bufs &d, int b) { return kdbuf(work_buf(d, b)); }  // the working rows' Defect (kernel (Params, Bufs, ...))
    static constexpr int LQS = LQW;
};
template <> struct Prec<float> {
    static DEV const float *lq(const Bufs &d) { return d.lq32; }
    static DEV float *K(const Bufs &d) { return d.K32; }
    static DEV const float *def(const Bufs &d, int) { return d.def32; }  // (k_lq's copy of the working Defect)
    static constexpr int LQS = LQW32;
};

// One sweep item: element, regularisation, outputs (gain rows, dU rows) and whether it runs.
template <typename real>
struct Item {
    int b;          // element (valid even when inactive: its rows are read, never written)
    bool act;       // this half sweeps
    real reg;
    real *K;        // [Kc][12][24]
    double *dU;     // [Kc][24]
};

// Per-lane constants of a phase (contacts of the lane's item); the B entries of the contacts
// (bv, bq) live in LDS (Lds::Item::pc), read where they are used.
template <typename real>
struct Phase {
    int cmask;      // bit l: leg l in stance
    int xmask;      // row pp's lxx cross terms present (bit t; see Lane::xc0)
    real lxd;       // row pp < 24: lxx diagonal
    real xw;        // row pp: magnitude of its lxx cross terms (each is -xw)
    real dtr;       // Quu column lane: dt R of its coupled control (stance: GRF, swing: qJd)
    real dtrz;      // position pp < 12: dt R of its decoupled control
};

// Phase layout entries with a runtime phase index, read from the kernel-argument segment (scalar
// loads): indexing the by-value Params directly makes the compiler copy it to scratch.

template <typename real, typename ItemT>
DEV void load_phase(const Params &p, const Bufs &d, ItemT &I, int b, int i, int pp, Phase<real> &ph)
{
    const int *cs = d.contacts + ((size_t)b * (p.P + 1) + i) * 4;
    int c[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) c[l] = cs[l];
    ph.cmask = 0;
#pragma unroll
    for (int l = 0; l < 4; ++l) ph.cmask |= (c[l] != 0) << l;
    SSYNC();
    if (pp < 8) {  // B rows 9..11 (dt c_l / m) and 12..23 (dt (1 - c_l)) of leg pp % 4
        const int cl = (ph.cmask >> (pp & 3)) & 1;
        I.pc[pp] = pp < 4 ? (cl ? (real)p.dt_m : (real)0) : (cl ? (real)0 : (real)p.dt);
    }
    SSYNC();
    const int pos = pp & 15, cq = (ph.cmask >> ((pos / 3) & 3)) & 1;
    ph.dtr = (real)(p.dt * (cq ? p.r_grf : p.r_qJd));
    const int cz = (ph.cmask >> ((pp < HC ? pp : 0) / 3)) & 1;
    ph.dtrz = (real)(p.dt * (cz ? p.r_qJd : p.r_grf));
    // lxx row pp (HKDCost.cpp:32: dt Q + dt D^T Qfoot D)
    const int r = pp < NX ? pp : 0;
    double dg = p.dt * (r < 12 ? kparams()->qbase[r] : p.q_qJ * (1 - ((ph.cmask >> ((r - 12) / 3)) & 1)));
    ph.xmask = 0;
    ph.xw = 0;
    if (r >= 3 && r < 6) {
        const double fw = p.dt * (p.foot_gain * kparams()->foot_w[r - 3]);
#pragma unroll
        for (int l = 0; l < 4; ++l) dg += c[l] ? fw : 0.0;
        ph.xmask = ph.cmask;
        ph.xw = (real)fw;
    } else if (r >= 12) {
        const int m = r - 12;
        const double w = ((ph.cmask >> (m / 3)) & 1) ? p.dt * (p.foot_gain * kparams()->foot_w[m % 3]) : 0.0;
        dg += w;
        ph.xmask = 1;
        ph.xw = (real)w;
    }
    ph.lxd = (real)dg;
}

// Request the knot images (record + Defect[s+1]) of both items into S.img by LDS-DMA.  The leading
// lgkmcnt(0) retires every LDS read of the old images first.
template <typename real>
DEV void fetch(Lds<real> &S, const real *rec0, const real *def0, const real *rec1, const real *def1, int lane)
{
    using PC = Pieces<real>;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int t = 0; t < PC::NI; ++t) {
        const int n = 64 * t + lane;
        if (n < 2 * PC::NP) {
            const int e = n >= PC::NP, q = n - e * PC::NP;
            const real *rec = e ? rec1 : rec0, *def = e ? def1 : def0;
            const real *src = q < PC::NA ? rec + PC::E * q : q < PC::NA + PC::ND ? def + PC::E * (q - PC::NA)
                                                                                 : rec + PC::E * (q - PC::ND);
            if (HSDDP_SWEEP_NT) lds_dma16_nt(src, (unsigned)(size_t)(&S.img[0][0]) + 1024u * t);
            else lds_dma16(src, (unsigned)(size_t)(&S.img[0][0]) + 1024u * t);
        }
    }
}

// RB (sym 3x3, stored 00,01,02,11,12,22) index of entry (a, b)
DEV constexpr int rb_index(int a, int b)
{
    return (a < b ? a : b) == 0 ? (a > b ? a : b) : (a < b ? a : b) == 1 ? 2 + (a > b ? a : b) : 5;
}

// Per-lane constants of the whole sweep (lane roles, LDS addresses)
struct Lane {
    int lane, e, pp, pos;
    bool row;       // pp < 24
    bool qlane;     // a Quu_cc column lane (pos < 12)
    int rb[3];      // image index of this Quu column's ReB row (leg pos / 3, axis pos % 3)
    int xc0, xkind;  // lxx cross terms of row pp: kind 1 (rows 3..5): columns xc0 + 3 t; kind 2 (rows >= 12): xc0
};

// Column split: wave W of k_riccati_cs forms the entries of M, Z, Qxx and H in the columns c with
// cs_wave(c) == W.  The two sets of 12 balance the structural multiply-adds of M = H A (and of
// S^T M) per column: 36 for wave 0, 33 for wave 1.
constexpr unsigned CS_COLS1 = (1u << 0) | (1u << 3) | (1u << 4) | (1u << 5) | (1u << 8) | (1u << 9) | (1u << 10) |
                              (1u << 11) | (1u << 18) | (1u << 19) | (1u << 21) | (1u << 22);
DEV constexpr int cs_wave(int c) { return (int)((CS_COLS1 >> c) & 1u); }
// column c is formed here (W < 0: the unsplit sweep forms every column)
template <int W>
DEV constexpr bool cs_mine(int c) { return W < 0 || cs_wave(c) == W; }

// acc[c] += sum_j x[j] S[j][c] (S = A - I: rows 0..2 eul, 3..5 the dt entries, 6..8 omega) in
// source order: consecutive multiply-adds feed different accumulators; W >= 0: the columns of
// wave W only
template <int W = -1, typename real>
DEV void emit_SA(real (&acc)[NX], const real (&x)[NX], const real (&cf)[8], real dt)
{
    auto sw_row = [&](auto I) {
        constexpr int i = I;
        static_for<17>([&](auto Q) {
            if constexpr (cs_mine<W>(sw_col(Q))) vfma<sw_at(i, Q)>(acc[sw_col(Q)], cf, x[6 + i]);
        });
    };
    auto se_row = [&](auto I) {
        constexpr int i = I;
        static_for<5>([&](auto Q) {
            if constexpr (cs_mine<W>(se_col(Q))) vfma<V_SE + 5 * i + Q>(acc[se_col(Q)], cf, x[i]);
        });
    };
    sw_row(std::integral_constant<int, 0>{});
    se_row(std::integral_constant<int, 0>{});
    sw_row(std::integral_constant<int, 1>{});
    se_row(std::integral_constant<int, 1>{});
    sw_row(std::integral_constant<int, 2>{});
    se_row(std::integral_constant<int, 2>{});
    static_for<3>([&](auto A) {
        if constexpr (cs_mine<W>(9 + A)) acc[9 + A] = __builtin_fma(x[3 + A], dt, acc[9 + A]);
    });
}

// acc[q] += (B_c^T y)[q] for the 12 coupled controls, y = (y6, y7, y8) on B's omega rows (BW, DPP
// broadcast), y9[a] on row 9 + a (bv: dt c / m), y12[q] on row 12 + q (bq: dt (1 - c)); the
// structurally absent half of the last two is an exact zero.  Controls Q0 .. Q1 - 1 only.
template <int Q0 = 0, int Q1 = HC, typename real>
DEV void emit_Bc(real (&acc)[HC], real y6, real y7, real y8, const real *y9, const real *y12, const real (&bv)[4],
                 const real (&bq)[4], const real (&cf)[8])
{
#pragma unroll
    for (int q = Q0; q < Q1; ++q) acc[q] = __builtin_fma(y12[q], bq[q / 3], acc[q]);
#pragma unroll
    for (int q = Q0; q < Q1; ++q) acc[q] = __builtin_fma(y9[q % 3], bv[q / 3], acc[q]);
    static_for<Q1 - Q0>([&](auto Q) { vfma<bw_at(0, Q0 + Q)>(acc[Q0 + Q], cf, y6); });
    static_for<Q1 - Q0>([&](auto Q) { vfma<bw_at(1, Q0 + Q)>(acc[Q0 + Q], cf, y7); });
    static_for<Q1 - Q0>([&](auto Q) { vfma<bw_at(2, Q0 + Q)>(acc[Q0 + Q], cf, y8); });
}

// Gaussian elimination without pivoting on the columns held in lanes, then back substitution:
// w = Quu_cc columns (DPP positions 0..11 of both DPP rows of an item), w2 = right-hand sides.
// Forward step j takes column j from DPP position j and eliminates it from the rows below; pivot
// rows are kept scaled by 1 / pivot and negated, so after the back substitution w2 =
// -Quu_cc^-1 (rhs).  The next step's pivot chain (DPP broadcast, reciprocal, Newton steps, the two
// factors) is threaded through this step's independent multiply-adds, its operand row first (the
// scalar steps are compiler builtins: the compiler places them and their wait states).  The
// pivots are those of the LDL^T factorisation of Quu_cc; bad: ballot of pivots <= 1e-9 (PSD test).
template <typename real>
DEV void eliminate(real (&w)[HC], real (&w2)[HC], unsigned long long &bad)
{
    constexpr bool F64 = sizeof(real) == 8;
    constexpr int CH = F64 ? 13 : 9;  // slot of the last chain operation
    real r, e, nf, nf2;
    {
        const real piv = row_bcast<0>(w[0]);
        bad |= __builtin_amdgcn_ballot_w64(!(piv > (real)1e-9));
        asm_rcp(r, piv);
        asm_nfma1(e, piv, r);
        asm_newton(r, e);
        if constexpr (F64) {
            asm_nfma1(e, piv, r);
            asm_newton(r, e);
        }
        asm_nmul(nf, w[0], r);
        asm_nmul(nf2, w2[0], r);
    }
    static_for<HC>([&](auto J) {
        constexpr int j = J, jn = j + 1;
        constexpr bool nx = jn < HC;
        real pivn = 0, rn = 0, en = 0, nfn = 0, nf2n = 0;
        if constexpr (nx) {  // the next pivot's row first (right-hand side before its multiplier changes)
            bfma<j>(w2[jn], w[jn], nf2);
            fmac_row_bcast<j, false>(w[jn], nf);
        }
        constexpr int NO = nx ? HC - 2 - j : 0;        // rows below jn
        constexpr int NT = (2 * NO > CH + 1) ? 2 * NO : CH + 1;
        static_for<NT>([&](auto T) {
            constexpr int t = T, i = jn + 1 + t / 2;
            if constexpr (t < 2 * NO) {
                if constexpr (t % 2 == 0)
                    bfma<j>(w2[i], w[i], nf2);
                else
                    fmac_row_bcast<j, false>(w[i], nf);
            }
            if constexpr (nx) {
                if constexpr (t == 1) pivn = row_bcast<(nx ? jn : 0)>(w[jn]);
                if constexpr (t == 3) asm_rcp(rn, pivn);
                if constexpr (t == 5) asm_nfma1(en, pivn, rn);
                if constexpr (t == 7) asm_newton(rn, en);
                if constexpr (F64 && t == 9) asm_nfma1(en, pivn, rn);
                if constexpr (F64 && t == 11) asm_newton(rn, en);
                if constexpr (t == CH) {
                    asm_nmul(nfn, w[jn], rn);
                    asm_nmul(nf2n, w2[jn], rn);
                }
            }
        });
        w[j] = nf;
        w2[j] = nf2;
        if constexpr (nx) {
            bad |= __builtin_amdgcn_ballot_w64(!(pivn > (real)1e-9));
            nf = nfn;
            nf2 = nf2n;
        }
    });
    // back substitution: x_j = w2[j] (negated), rows i < j lose U[i][j] x_j (U[i][j] = w[i] on lane j,
    // negated too: the product's sign is right), the next row first
    static_for<HC - 1>([&](auto Jr) {
        constexpr int j = HC - 1 - Jr;
        static_for<j>([&](auto Ii) {
            constexpr int i = j - 1 - Ii;
            bfma<j>(w2[i], w[i], w2[j]);
        });
    });
}

// One knot of SinglePhase::backward_sweep for the wave's two items.  h / g: H[k+1] row pp and
// G[k+1][pp] on entry, H[k], G[k] on exit.  live: this half's item is still sweeping (turns false
// at a failed PSD test: nothing of this knot or below is written).  more: the next knot's images
// are requested into S.img during the elimination (nrec*/ndef*).  DV (single shooting only): the
// knot's Qu^T dU (dV_k = -Qu^T dU, SinglePhase.cpp:359-362) is added to the lane's dvs — position 24
// the coupled controls' part, positions < 12 one decoupled control each.  Without DV (multiple
// shooting) it is not formed: the linear rollout replaces it (quirk A3), and that instantiation is
// the one the metric runs.
template <typename real, bool DV>
DEV void knot(const Params &p, Lds<real> &S, const Lane &L, const Phase<real> &ph, const Item<real> &it, int kc,
              real (&h)[NX], real &g, bool &live, bool first, bool more, const real *nrec0, const real *ndef0,
              const real *nrec1, const real *ndef1, double &dvs)
{
    typename Lds<real>::Item &I = S.it[L.e];
    const real *img = S.img[L.e];
    const int pp = L.pp, pos = L.pos;
    const real dt = (real)p.dt;
    real reg = it.reg;
    STAMP(0);
    // this knot's images: a phase's first knot waits for them here, every other knot's landed before
    // the previous knot's output stores (end of knot)
    if (first) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // coefficient registers: V[16 k + pos] on register k of every DPP row
    real cf[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cf[k] = img[16 * k + pos];
    real bv[4], bq[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) { bv[l] = I.pc[l]; bq[l] = I.pc[4 + l]; }
    STAMP(1);
    // ---- Gn = G + H d (SinglePhase.cpp:320), T = H B_c, M = H A (row pp) ----------------------
    // T and Gn read H first; M = H + H S then accumulates over H's registers (H is not read again:
    // the knot ends by forming the new H) from copies of the 9 entries S's rows read
    real t[HC], ga[4] = {g, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < HC; ++q) t[q] = 0;
    emit_Bc(t, h[6], h[7], h[8], h + 9, h + 12, bv, bq, cf);
    static_for<NX>([&](auto C) { vfma<V_D + C>(ga[C & 3], cf, h[C]); });
    const real gn = (ga[0] + ga[1]) + (ga[2] + ga[3]);
    pin(t);
    real h9[NX];  // (entries 0..8 only)
#pragma unroll
    for (int j = 0; j < 9; ++j) h9[j] = h[j];
#pragma unroll
    for (int j = 9; j < NX; ++j) h9[j] = 0;
    SSYNC();
    real (&m)[NX] = h;
    emit_SA(m, h9, cf, dt);
    pin(t);
    pin(m);
    if (L.row) {
#pragma unroll
        for (int c = 0; c < NX; ++c) I.MI[pp * MS + c] = m[c];
        I.MI[pp * MS + NX] = gn;
#pragma unroll
        for (int q = 0; q < HC; ++q) I.TI[pp * TS + q] = t[q];
    }
    SSYNC();
    STAMP(2);
    // ---- column pp of M (position 24: Gn); Z row, Qux_c column, Qu_c ---------------------------
    const int pc = pp < MS - 1 ? pp : MS - 1;
    real mc[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) mc[j] = I.MI[j * MS + pc];
    // Qux_c[q][pp] = (B_c^T M)[q][pp] (lux = 0); position 24: Qu_c = lu_c + B_c^T Gn
    real w2[HC];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const real *lcp = pp == NX ? img + V_LU + (((ph.cmask >> l) & 1) ? 3 * l : 12 + 3 * l) : S.zero;
#pragma unroll
        for (int a = 0; a < 3; ++a) w2[3 * l + a] = lcp[a];
    }
    // Z[pp][i] = M[pp][i] + sum_k M[k][pp] S[k][i] (S^T M transposed); position 24: (S^T Gn)[i]
    emit_SA(m, mc, cf, dt);
    emit_Bc(w2, mc[6], mc[7], mc[8], mc + 9, mc + 12, bv, bq, cf);
    pin(m);
    pin(w2);
    STAMP(3);
    // ---- Qxx = lxx + reg I + (Z + Z^T) / 2 (SinglePhase.cpp:323-352) ---------------------------
    if (pp <= NX) {  // Z rows (two zero columns: the column reads of positions > 24 see zeros)
#pragma unroll
        for (int c = 0; c < NX; ++c) I.MI[pp * MS + c] = m[c];
        I.MI[pp * MS + NX] = 0;
        I.MI[pp * MS + NX + 1] = 0;
    }
    SSYNC();
    // lxx + reg I into the Z image: each row lane adds its diagonal and lxx cross terms to its own
    // row by LDS atomic adds behind its row's stores (a wave's LDS operations complete in order, so
    // no read-back round trip; no two lanes touch one entry; the add is the IEEE add of the value
    // stored, as a read-add-write would form it)
    if (L.row) {
        real *zr = I.MI + pp * MS;
        lds_add(zr + pp, ph.lxd + reg);
#pragma unroll
        for (int t2 = 0; t2 < 4; ++t2)
            if ((ph.xmask >> t2) & 1) lds_add(zr + (L.xkind == 1 ? L.xc0 + 3 * t2 : L.xc0), -ph.xw);
    }
    SSYNC();
    const real *zrow = L.row ? I.MI + pp * MS : S.zero;
    real qxx[NX], zc[NX];
#pragma unroll
    for (int c = 0; c < NX; ++c) qxx[c] = zrow[c];
#pragma unroll
    for (int c = 0; c < NX; ++c) zc[c] = I.MI[c * MS + pc];
    // every row and column read in flight before the first use (one wait, not one per register reuse)
    pin(qxx);
    pin(zc);
#pragma unroll
    for (int c = 0; c < NX; ++c) qxx[c] *= (real)0.5;
    // (r + c) / 2 as r / 2 + c / 2: halving is exact, so the same value, without an add -> multiply
    // dependence per entry
#pragma unroll
    for (int c = 0; c < NX; ++c) qxx[c] = __builtin_fma(zc[c], (real)0.5, qxx[c]);
    pin(qxx);  // materialised here, not sunk to the value update (twice the registers across the elimination)
    // Qx = lx + A^T Gn = lx + Gn + S^T Gn
    const real qx = img[V_LX + (L.row ? pp : 0)] + (gn + I.MI[NX * MS + pc]);
    STAMP(4);
    // ---- Quu_cc column pos = luu + reg + B_c^T T[:, pos] (SinglePhase.cpp:324, MultiPhaseDDP.cpp:160)
    real tcol[18];
#pragma unroll
    for (int j = 0; j < 18; ++j) tcol[j] = I.TI[(6 + j) * TS + pos];
    real lbr[3];  // row pos % 3 of the leg's ReB block, dt R + reg on its diagonal
    const int aq = pos % 3;
#pragma unroll
    for (int a = 0; a < 3; ++a) lbr[a] = (L.qlane ? img + L.rb[a] : S.zero + a)[0] + (a == aq ? ph.dtr + reg : (real)0);
    const int lq = pos / 3;
    real w[HC];
#pragma unroll
    for (int q = 0; q < HC; ++q) w[q] = (L.qlane && lq == q / 3) ? lbr[q % 3] : (real)0;
    emit_Bc(w, tcol[0], tcol[1], tcol[2], tcol + 3, tcol + 6, bv, bq, cf);
    pin(w);
    // decoupled controls on positions 0..11: Qu_z = lu_z, Quu_zz = dt R_z + reg
    const bool zl = pp < HC;
    const int du_z = ((ph.cmask >> ((zl ? pp : 0) / 3)) & 1) ? 12 + pp : pp;  // the decoupled control of pp < 12
    const real quz = img[zl ? V_LU + du_z : V_LU];
    const real qzz = ph.dtrz + reg;
    // the images are read: the next knot's are requested now (in flight during the elimination)
    if (more) fetch(S, nrec0, ndef0, nrec1, ndef1, L.lane);
    STAMP(5);
    // ---- PSD test + Gauss-Jordan on [Quu_cc | Qux_c | Qu_c] --------------------------------------
    // Qux_c column pp, kept for G and the value update (positions >= 24: zero, so their H row stays 0;
    // DV: position 24 keeps Qu_c for the knot's Qu_c^T dU_c, and its H row is cleared after the update)
    real quxs[HC];
#pragma unroll
    for (int q = 0; q < HC; ++q) quxs[q] = (L.row || (DV && pp == NX)) ? w2[q] : (real)0;
    pin(quxs);
    unsigned long long bad = __builtin_amdgcn_ballot_w64(zl && !(qzz > (real)1e-9));
    // w2 becomes -Quu_cc^-1 [Qux_c | Qu_c] = [K_c | dU_c] (the reference's explicit inverse,
    // SinglePhase.cpp:351-356, as a solve)
    eliminate(w, w2, bad);
    const bool okh = L.e ? (bad >> 32) == 0 : (bad & 0xffffffffull) == 0;
    live = live && okh;
    const bool st = live;  // this half writes the knot's outputs
    STAMP(6);
    // ---- outputs: dU through LDS (K_c rows and dU go out at the end of the knot) ---------------------
    if (pp == NX)  // coupled dU from position 24
#pragma unroll
        for (int q = 0; q < HC; ++q) I.du[(((ph.cmask >> (q / 3)) & 1) ? 0 : 12) + q] = w2[q];
    if (zl) I.du[du_z] = -(quz / qzz);
#if HSDDP_VALUE_MFMA
    // K_c^T rows (row 24: dU_c) and Qux_c^T rows for the value update
    if (pp <= NX)
#pragma unroll
        for (int q = 0; q < HC; ++q) I.MI[pp * TS + q] = w2[q];
    if (L.row)
#pragma unroll
        for (int q = 0; q < HC; ++q) I.TI[pp * TS + q] = quxs[q];
    SSYNC();
    // G = Qx - Qux_c^T Quu_cc^-1 Qu_c = Qx + Qux_c^T dU_c (SinglePhase.cpp:359)
    real gq4[4] = {qx, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < HC; ++q) gq4[q & 3] = __builtin_fma(quxs[q], I.MI[NX * TS + q], gq4[q & 3]);
    const real gq = (gq4[0] + gq4[1]) + (gq4[2] + gq4[3]);
    if constexpr (DV) {
        real dq = 0;
#pragma unroll
        for (int q = 0; q < HC; ++q) dq = __builtin_fma(quxs[q], I.MI[NX * TS + q], dq);
        const double v = pp == NX ? (double)dq : zl ? (double)quz * (double)I.du[du_z] : 0.0;
        if (st) dvs += v;
    }
    STAMP(7);
    // ---- H = Qxx - Qux_c^T Quu_cc^-1 Qux_c = Qxx + Qux_c^T K_c on the matrix cores ------------------
    // (tiles (0,0), (0,1), (1,1) of the symmetric 24 x 24 product, K = 12, for both items at once;
    // rows / columns 24..31 only feed discarded outputs; SinglePhase.cpp:360)
    const int li = L.lane & 15, lk = L.lane >> 4;
    real a0[2][3], a1[2][3], b0[2][3], b1[2][3];
#pragma unroll
    for (int ei = 0; ei < 2; ++ei)
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
            const int q = 4 * ks + lk;
            a0[ei][ks] = S.it[ei].TI[li * TS + q];
            a1[ei][ks] = S.it[ei].TI[(16 + li) * TS + q];
            b0[ei][ks] = S.it[ei].MI[li * TS + q];
            b1[ei][ks] = S.it[ei].MI[(16 + li) * TS + q];
        }
    acc4<real> t00[2], t01[2], t11[2];
#pragma unroll
    for (int ei = 0; ei < 2; ++ei) t00[ei] = t01[ei] = t11[ei] = acc4<real>{0, 0, 0, 0};
#pragma unroll
    for (int ks = 0; ks < 3; ++ks)
#pragma unroll
        for (int ei = 0; ei < 2; ++ei) {
            t00[ei] = mfma16(a0[ei][ks], b0[ei][ks], t00[ei]);
            t01[ei] = mfma16(a0[ei][ks], b1[ei][ks], t01[ei]);
            t11[ei] = mfma16(a1[ei][ks], b1[ei][ks], t11[ei]);
        }
    SSYNC();  // the operands are in registers: the product overwrites the K^T images
#pragma unroll
    for (int ei = 0; ei < 2; ++ei) {
        real *P = S.it[ei].MI;
#pragma unroll
        for (int gi = 0; gi < 4; ++gi) {
            const int r0 = mfma_row<real>(lk, gi), r1 = 16 + r0, c1 = 16 + li;
            P[r0 * MS + li] = t00[ei][gi];
            if (c1 < NX) {
                P[r0 * MS + c1] = t01[ei][gi];
                P[c1 * MS + r0] = t01[ei][gi];
            }
            if (r1 < NX && c1 < NX) P[r1 * MS + c1] = t11[ei][gi];
        }
    }
    SSYNC();
    STAMP(8);
    const real *prow = L.row ? I.MI + pp * MS : S.zero;
#pragma unroll
    for (int c = 0; c < NX; ++c) h[c] = qxx[c] + prow[c];
#else
    SSYNC();
    // K_c columns of both DPP rows at every DPP position (column c of the item on position c & 15
    // of ka (c < 16) or kb (c >= 16)); the coupled dU_c is position 24's: kb at position 8
    real ka[HC], kb[HC];
#pragma unroll
    for (int q = 0; q < HC; ++q) row_pair_last(w2[q], ka[q], kb[q]);
    // G = Qx - Qux_c^T Quu_cc^-1 Qu_c = Qx + Qux_c^T dU_c (SinglePhase.cpp:359)
    real gq4[4] = {qx, 0, 0, 0};
    static_for<HC>([&](auto Q) { bfma<8>(gq4[Q & 3], kb[Q], quxs[Q]); });
    const real gq = (gq4[0] + gq4[1]) + (gq4[2] + gq4[3]);
    if constexpr (DV) {  // position 24: Qu_c^T dU_c (dU_c by broadcast from position 24 = kb's position 8)
        real dq = 0;
        static_for<HC>([&](auto Q) { bfma<8>(dq, kb[Q], quxs[Q]); });
        const double v = pp == NX ? (double)dq : zl ? (double)quz * (double)(-(quz / qzz)) : 0.0;
        if (st) dvs += v;
    }
    STAMP(7);
    // ---- H = Qxx - Qux_c^T Quu_cc^-1 Qux_c = Qxx + Qux_c^T K_c (SinglePhase.cpp:360): row pp,
    // K_c by DPP broadcast from the lanes that hold its columns
#pragma unroll
    for (int c = 0; c < NX; ++c) h[c] = qxx[c];
    static_for<HC>([&](auto Q) {
        static_for<NX>([&](auto C) {
            constexpr int c = C;
            if constexpr (c < 16)
                bfma<c & 15>(h[c], ka[Q], quxs[Q]);
            else
                bfma<c & 15>(h[c], kb[Q], quxs[Q]);
        });
    });
    if constexpr (DV)
        if (!L.row)
#pragma unroll
            for (int c = 0; c < NX; ++c) h[c] = 0;
    STAMP(8);
#endif
    g = L.row ? gq : (real)0;
    // K_c rows and dU (SinglePhase.cpp:354-356).  Issued after a wait for all vector memory
    // operations — the next knot's image DMA (requested before the elimination) and the previous
    // knot's stores, both long complete — so no later wait counts these stores: the next knot reads
    // its images without waiting (vector memory operations complete in order).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#if HSDDP_VALUE_MFMA
    if (st && L.row) {
        real *Kg = it.K + (size_t)kc * KCW;
#pragma unroll
        for (int q = 0; q < HC; ++q) Kg[q * NX + pp] = w2[q];
        it.dU[(size_t)kc * NX + pp] = I.du[pp];
    }
#else
    // from the row-pair copies (w2 is dead after the broadcast): columns 0..15 from ka by both DPP
    // rows of the item (the two write the same value), columns 16..23 from kb
    if (st) {
        real *Kg = it.K + (size_t)kc * KCW;
#pragma unroll
        for (int q = 0; q < HC; ++q) Kg[q * NX + pos] = ka[q];
        if (pos < NX - 16)
#pragma unroll
            for (int q = 0; q < HC; ++q) Kg[q * NX + 16 + pos] = kb[q];
        if (L.row) it.dU[(size_t)kc * NX + pp] = I.du[pp];
    }
#endif
    SSYNC();
    STAMP(9);
}

// Workgroup barrier of the column split: this wave's LDS writes done, both waves here.  No wait
// for vector memory (the knot images and the K / dU stores stay in flight: each wave waits for its
// own requests with vmcnt before the barrier that publishes them).
#define CSYNC()                                              \
    do {                                                     \
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
        __builtin_amdgcn_s_barrier();                        \
        asm volatile("" ::: "memory");                       \
        __builtin_amdgcn_sched_barrier(0);                   \
    } while (0)

// fetch for the column split: wave W requests its half of the two items' pieces into image buffer q
template <int W, typename real>
DEV void fetch_cs(LdsCS<real> &S, int q, const real *rec0, const real *def0, const real *rec1, const real *def1,
                  int lane)
{
    using PC = Pieces<real>;
    constexpr int H = (PC::NI + 1) / 2;
#pragma unroll
    for (int u = 0; u < H; ++u) {
        const int t = W * H + u;
        const int n = 64 * t + lane;
        if (t < PC::NI && n < 2 * PC::NP) {
            const int e = n >= PC::NP, qq = n - e * PC::NP;
            const real *rec = e ? rec1 : rec0, *def = e ? def1 : def0;
            const real *src = qq < PC::NA ? rec + PC::E * qq : qq < PC::NA + PC::ND ? def + PC::E * (qq - PC::NA)
                                                                                    : rec + PC::E * (qq - PC::ND);
            lds_dma16(src, (unsigned)(size_t)(&S.img[q][0][0]) + 1024u * t);
        }
    }
}

// One knot of the sweep for wave W of the column split (k_riccati_cs): the knot() stages with the
// column-parallel work halved — T's controls 6 W .. 6 W + 5, the columns cs_wave(c) == W of M, Z,
// Qxx and H — and the per-element chain (Gn, Qux_c, the Quu_cc columns, the elimination, the K
// broadcast, G) formed whole in both waves, so each wave holds everything it multiplies by.  Three
// barriers: M / T rows written -> column reads; Z rows written -> Qxx reads; this wave's H columns
// written (and its share of the next images landed) -> the other wave's H columns read.  ib: the
// image buffer of this knot (the next knot's go to ib ^ 1); par: which MZ image holds M (the
// other takes Z).  Both waves run the same branch decisions (live, the PSD test) on equal values.
template <int W, bool DV, typename real>
DEV void knot_cs(const Params &p, LdsCS<real> &S, const Lane &L, const Phase<real> &ph, const Item<real> &it, int kc,
                 real (&h)[NX], real &g, bool &live, bool first, bool more, int ib, int par, const real *nrec0,
                 const real *ndef0, const real *nrec1, const real *ndef1, double &dvs)
{
    constexpr int Q0 = 6 * W, Q1 = Q0 + 6;
    auto &I = S.it[L.e];
    const real *img = S.img[ib][L.e];
    real *const MA = I.MZ[par], *const ZA = I.MZ[par ^ 1];
    const int pp = L.pp, pos = L.pos;
    const real dt = (real)p.dt;
    const real reg = it.reg;
    if (first) {  // the phase's first images (each wave waits for its own requests, then both)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        CSYNC();
    }
    real cf[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) cf[k] = img[16 * k + pos];
    real bv[4], bq[4];
#pragma unroll
    for (int l = 0; l < 4; ++l) { bv[l] = I.pc[l]; bq[l] = I.pc[4 + l]; }
    // ---- Gn = G + H d, T = H B_c (this wave's controls), M = H A (this wave's columns) -------------
    real t[HC], ga[4] = {g, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < HC; ++q) t[q] = 0;
    emit_Bc<Q0, Q1>(t, h[6], h[7], h[8], h + 9, h + 12, bv, bq, cf);
    static_for<NX>([&](auto C) { vfma<V_D + C>(ga[C & 3], cf, h[C]); });
    const real gn = (ga[0] + ga[1]) + (ga[2] + ga[3]);
    pin(t);
    real h9[NX];
#pragma unroll
    for (int j = 0; j < 9; ++j) h9[j] = h[j];
#pragma unroll
    for (int j = 9; j < NX; ++j) h9[j] = 0;
    SSYNC();
    real (&m)[NX] = h;
    emit_SA<W>(m, h9, cf, dt);
    pin(t);
    pin(m);
    if (L.row) {
        static_for<NX>([&](auto C) {
            if constexpr (cs_mine<W>(C)) MA[pp * MS + C] = m[C];
        });
        if (W == 0) MA[pp * MS + NX] = gn;
#pragma unroll
        for (int q = Q0; q < Q1; ++q) I.TI[pp * TS + q] = t[q];
    }
    CSYNC();
    // ---- column pp of M (position 24: Gn); Z row (this wave's columns), Qux_c column, Qu_c ----------
    const int pc = pp < MS - 1 ? pp : MS - 1;
    real mc[NX];
#pragma unroll
    for (int j = 0; j < NX; ++j) mc[j] = MA[j * MS + pc];
    real w2[HC];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
        const real *lcp = pp == NX ? img + V_LU + (((ph.cmask >> l) & 1) ? 3 * l : 12 + 3 * l) : S.zero;
#pragma unroll
        for (int a = 0; a < 3; ++a) w2[3 * l + a] = lcp[a];
    }
    emit_SA<W>(m, mc, cf, dt);
    emit_Bc(w2, mc[6], mc[7], mc[8], mc + 9, mc + 12, bv, bq, cf);
    pin(m);
    pin(w2);
    // ---- Qxx = lxx + reg I + (Z + Z^T) / 2 on this wave's columns ----------------------------------
    if (pp <= NX) {
        static_for<NX>([&](auto C) {
            if constexpr (cs_mine<W>(C)) ZA[pp * MS + C] = m[C];
        });
        if (W == 0) {
            ZA[pp * MS + NX] = 0;
            ZA[pp * MS + NX + 1] = 0;
        }
    }
    SSYNC();
    if (L.row) {  // lxx and reg I on the entries of this wave's columns (behind its own Z stores)
        real *zr = ZA + pp * MS;
        if (cs_wave(pp) == W) lds_add(zr + pp, ph.lxd + reg);
#pragma unroll
        for (int t2 = 0; t2 < 4; ++t2) {
            const int xc = L.xkind == 1 ? L.xc0 + 3 * t2 : L.xc0;
            if (((ph.xmask >> t2) & 1) && cs_wave(xc) == W) lds_add(zr + xc, -ph.xw);
        }
    }
    CSYNC();
    const real *zrow = L.row ? ZA + pp * MS : S.zero;
    real qxx[NX], zc[NX];
    static_for<NX>([&](auto C) {
        if constexpr (cs_mine<W>(C)) {
            qxx[C] = zrow[C];
            zc[C] = ZA[C * MS + pc];
        }
    });
    static_for<NX>([&](auto C) {
        if constexpr (cs_mine<W>(C)) qxx[C] = __builtin_fma(zc[C], (real)0.5, qxx[C] * (real)0.5);
    });
    const real qx = img[V_LX + (L.row ? pp : 0)] + (gn + ZA[NX * MS + pc]);
    // ---- Quu_cc column pos = luu + reg + B_c^T T[:, pos] -------------------------------------------
    real tcol[18];
#pragma unroll
    for (int j = 0; j < 18; ++j) tcol[j] = I.TI[(6 + j) * TS + pos];
    real lbr[3];
    const int aq = pos % 3;
#pragma unroll
    for (int a = 0; a < 3; ++a) lbr[a] = (L.qlane ? img + L.rb[a] : S.zero + a)[0] + (a == aq ? ph.dtr + reg : (real)0);
    const int lq = pos / 3;
    real w[HC];
#pragma unroll
    for (int q = 0; q < HC; ++q) w[q] = (L.qlane && lq == q / 3) ? lbr[q % 3] : (real)0;
    emit_Bc(w, tcol[0], tcol[1], tcol[2], tcol + 3, tcol + 6, bv, bq, cf);
    pin(w);
    const bool zl = pp < HC;
    const int du_z = ((ph.cmask >> ((zl ? pp : 0) / 3)) & 1) ? 12 + pp : pp;
    const real quz = img[zl ? V_LU + du_z : V_LU];
    const real qzz = ph.dtrz + reg;
    // the next knot's images into the other buffer (read last in the previous knot, before its last
    // barrier)
    if (more) fetch_cs<W>(S, ib ^ 1, nrec0, ndef0, nrec1, ndef1, L.lane);
    // ---- PSD test + elimination on [Quu_cc | Qux_c | Qu_c] (both waves) ------------------------------
    real quxs[HC];
#pragma unroll
    for (int q = 0; q < HC; ++q) quxs[q] = (L.row || (DV && pp == NX)) ? w2[q] : (real)0;
    pin(quxs);
    unsigned long long bad = __builtin_amdgcn_ballot_w64(zl && !(qzz > (real)1e-9));
    eliminate(w, w2, bad);
    const bool okh = L.e ? (bad >> 32) == 0 : (bad & 0xffffffffull) == 0;
    live = live && okh;
    const bool st = live;
    // ---- dU through LDS (both waves write the same values) -------------------------------------------
    if (pp == NX)
#pragma unroll
        for (int q = 0; q < HC; ++q) I.du[(((ph.cmask >> (q / 3)) & 1) ? 0 : 12) + q] = w2[q];
    if (zl) I.du[du_z] = -(quz / qzz);
    SSYNC();
    real ka[HC], kb[HC];
#pragma unroll
    for (int q = 0; q < HC; ++q) row_pair_last(w2[q], ka[q], kb[q]);
    real gq4[4] = {qx, 0, 0, 0};
    static_for<HC>([&](auto Q) { bfma<8>(gq4[Q & 3], kb[Q], quxs[Q]); });
    const real gq = (gq4[0] + gq4[1]) + (gq4[2] + gq4[3]);
    if constexpr (DV) {  // as knot(): Qu_c^T dU_c on position 24, the decoupled controls' on pp < 12
        real dq = 0;
        static_for<HC>([&](auto Q) { bfma<8>(dq, kb[Q], quxs[Q]); });
        const double v = pp == NX ? (double)dq : zl ? (double)quz * (double)(-(quz / qzz)) : 0.0;
        if (st) dvs += v;
    }
    // ---- H = Qxx + Qux_c^T K_c on this wave's columns ------------------------------------------------
    static_for<NX>([&](auto C) {
        if constexpr (cs_mine<W>(C)) h[C] = qxx[C];
    });
    static_for<HC>([&](auto Q) {
        static_for<NX>([&](auto C) {
            constexpr int c = C;
            if constexpr (cs_mine<W>(c)) {
                if constexpr (c < 16)
                    bfma<c & 15>(h[c], ka[Q], quxs[Q]);
                else
                    bfma<c & 15>(h[c], kb[Q], quxs[Q]);
            }
        });
    });
    if constexpr (DV)  // (position 24's row took Qu_c through the update: not a row of H)
        if (!L.row)
            static_for<NX>([&](auto C) {
                if constexpr (cs_mine<W>(C)) h[C] = 0;
            });
    g = L.row ? gq : (real)0;
    // this wave's H columns into the M image (its column reads ended before the last barrier)
    if (L.row)
        static_for<NX>([&](auto C) {
            if constexpr (cs_mine<W>(C)) MA[pp * MS + C] = h[C];
        });
    // K_c rows and dU: wave 0 columns 0..15, wave 1 columns 16..23 and dU; issued after this wave's
    // image requests are complete (the barrier below publishes them)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (st) {
        real *Kg = it.K + (size_t)kc * KCW;
        if (W == 0) {
#pragma unroll
            for (int q = 0; q < HC; ++q) Kg[q * NX + pos] = ka[q];
        } else {
            if (pos < NX - 16)
#pragma unroll
                for (int q = 0; q < HC; ++q) Kg[q * NX + 16 + pos] = kb[q];
            if (L.row) it.dU[(size_t)kc * NX + pp] = I.du[pp];
        }
    }
    CSYNC();
    // the other wave's columns of row pp
    static_for<NX>([&](auto C) {
        if constexpr (!cs_mine<W>(C)) h[C] = L.row ? MA[pp * MS + C] : (real)0;
    });
    SSYNC();
}

// MultiPhaseDDP::backward_sweep (MultiPhaseDDP.cpp:190-229) for the wave's two items with their
// own regularisation.  Returns, per half, -1 (success) or the control slot of the first knot whose
// Quu fails the PSD test (that knot and the ones below it are not written).  DV: dv = the half's
// sum over every knot of Qu^T dU (= dV_1 = -dV_2 of the sweep, SinglePhase.cpp:359-362,
// MultiPhaseDDP.cpp:224-226), on every lane of the half.
template <typename real, bool EL, bool DV, int CSW = -1, typename LdsT = Lds<real>>
DEV int sweep_pair(const Params &p, const Bufs &d, LdsT &S, const Lane &L, const Item<real> &it, double &dv)
{
    constexpr bool CS = CSW >= 0;  // wave CSW of the column split (k_riccati_cs)
    int ib = 0, par = 0;           // (CS) image buffer, M / Z image roles
    double dvs = 0.0;
    const int pp = L.pp;
    const real *lqg = Prec<real>::lq(d);
    // the other item of the wave (its element's records feed the DMA even when this half is idle)
    const int b = it.b;
    const int b0 = __builtin_amdgcn_readlane(b, 0), b1 = __builtin_amdgcn_readlane(b, 32);  // wave-uniform (SGPRs)
    // each item's working Defect rows (the buffer its working trajectory is in)
    const real *defg0 = Prec<real>::def(d, b0), *defg1 = Prec<real>::def(d, b1);
    bool live = it.act;
    int fail = -1;
    real h[NX], g = 0;
    // both items share one layout (the handle's, or paired by layout: Bufs::pairs)
    const auto PL = layout_of<EL>(d, b0);
    const int P = PL.P();
    for (int i = P - 1; i >= 0; --i) {
        Phase<real> ph;
        load_phase<real>(p, d, S.it[L.e], b, i, pp, ph);
        const double *rec = d.term + ((size_t)b * p.P + i) * TW;
        if (i == P - 1) {
#pragma unroll
            for (int c = 0; c < NX; ++c) h[c] = L.row ? (real)rec[TM_PHIXX + pp * NX + c] : (real)0;
            g = L.row ? (real)rec[TM_PHIX + pp] : (real)0;
        } else {
            // impact-aware step G' = Phix + Px^T G0, H' = Phixx + Px^T H0 Px (MultiPhaseDDP.cpp:480-484):
            // W = H0 Px by rows (Px by DPP broadcast), then row pp of W^T Px from column pp of W
            auto &I = S.it[L.e];
            // scratch rows: the item's M image (CS: both waves form the same values into it, each
            // reading only what it wrote itself; barriers on both sides keep the knots' images apart)
            real *WI;
            if constexpr (CS) {
                WI = I.MZ[0];
                CSYNC();
            } else {
                WI = I.MI;
            }
            const double *Px = rec + TM_PX;
            // W = H0 Px by rows: Px in three 8-row chunks of DPP-broadcast coefficients
            real wr[NX];
#pragma unroll
            for (int c = 0; c < NX; ++c) wr[c] = 0;
            static_for<3>([&](auto Kc) {
                real px[12];
#pragma unroll
                for (int k = 0; k < 12; ++k) px[k] = (real)Px[192 * Kc + 16 * k + L.pos];
                if constexpr (sizeof(real) == 4) dpp_ready(px);  // converted by VALU: DPP sources
                static_for<8>([&](auto Kk) {
                    static_for<NX>([&](auto Cc) { vfma<NX * Kk + Cc>(wr[Cc], px, h[8 * Kc + Kk]); });
                });
            });
            SSYNC();
            if (L.row) {
#pragma unroll
                for (int c = 0; c < NX; ++c) WI[pp * WS + c] = wr[c];
                WI[pp * WS + NX] = g;  // column 24: G0
            }
            SSYNC();
            const int pc = pp < NX ? pp : NX;
            real wc[NX];
#pragma unroll
            for (int j = 0; j < NX; ++j) wc[j] = WI[j * WS + pc];
            real vr[NX];
#pragma unroll
            for (int c = 0; c < NX; ++c) vr[c] = 0;
            static_for<3>([&](auto Kc) {
                real px[12];
#pragma unroll
                for (int k = 0; k < 12; ++k) px[k] = (real)Px[192 * Kc + 16 * k + L.pos];
                if constexpr (sizeof(real) == 4) dpp_ready(px);  // converted by VALU: DPP sources
                static_for<8>([&](auto Jj) {
                    static_for<NX>([&](auto Cc) { vfma<NX * Jj + Cc>(vr[Cc], px, wc[8 * Kc + Jj]); });
                });
            });
            SSYNC();
            if (pp == NX)
#pragma unroll
                for (int c = 0; c < NX; ++c) WI[NX * WS + c] = vr[c];  // Px^T G0
            SSYNC();
            const real gp = WI[NX * WS + (L.row ? pp : 0)];
#pragma unroll
            for (int c = 0; c < NX; ++c) h[c] = L.row ? (real)rec[TM_PHIXX + pp * NX + c] + vr[c] : (real)0;
            g = L.row ? (real)rec[TM_PHIX + pp] + gp : (real)0;
            SSYNC();
            if constexpr (CS) CSYNC();
        }
        const int N = PL.N(i), s0 = PL.s0(i), k0 = PL.k0(i);
        auto recp = [&](int bb, int k) { return lqg + ((size_t)bb * p.Kc + k0 + k) * Prec<real>::LQS; };
        auto defp0 = [&](int k) { return defg0 + ((size_t)b0 * p.S + s0 + k + 1) * NX; };
        auto defp1 = [&](int k) { return defg1 + ((size_t)b1 * p.S + s0 + k + 1) * NX; };
        if constexpr (CS) fetch_cs<CSW>(S, ib, recp(b0, N - 1), defp0(N - 1), recp(b1, N - 1), defp1(N - 1), L.lane);
        else fetch(S, recp(b0, N - 1), defp0(N - 1), recp(b1, N - 1), defp1(N - 1), L.lane);
        int k = N - 1;
#pragma unroll 1
        for (; k >= 0; --k) {
            const bool more = k > 0;
            const int kn = more ? k - 1 : 0;
            const bool was = live;
            if constexpr (CS) {
                knot_cs<CSW, DV>(p, S, L, ph, it, k0 + k, h, g, live, k == N - 1, more, ib, par, recp(b0, kn),
                                 defp0(kn), recp(b1, kn), defp1(kn), dvs);
                ib ^= more ? 1 : 0;
                par ^= 1;
            } else {
                knot<real, DV>(p, S, L, ph, it, k0 + k, h, g, live, k == N - 1, more, recp(b0, kn), defp0(kn), recp(b1, kn),
                               defp1(kn), dvs);
            }
            if (was && !live) fail = k0 + k;
            if (!__builtin_amdgcn_ballot_w64(live)) break;
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA left in flight
        if (!__builtin_amdgcn_ballot_w64(live)) break;
        // G[0] += H[0] Defect[0] (SinglePhase.cpp:365)
        const real *d0 = (L.e ? defg1 : defg0) + ((size_t)b * p.S + s0) * NX;
        real dc[2] = {d0[L.pos], L.pos < NX - 16 ? d0[16 + L.pos] : (real)0};
        real a = 0;
        static_for<NX>([&](auto Cc) { vfma<Cc>(a, dc, h[Cc]); });
        if (L.row) g += a;
        // SinglePhase::get_value_approx (G[0], H[0] of the phase, SinglePhase.cpp:365) for callers
        // that read the value function (hsddp_set_value_export)
        if (p.store_value && live && L.row && CSW <= 0) {
            double *V = d.value0 + ((size_t)b * p.P + i) * (NX + NN);
#pragma unroll
            for (int c = 0; c < NX; ++c) V[NX + pp * NX + c] = (double)h[c];
            V[pp] = (double)g;
        }
    }
    if constexpr (DV) {
#pragma unroll
        for (int o = 16; o > 0; o >>= 1) dvs += __shfl_xor(dvs, o);
    }
    dv = dvs;
    return it.act ? fail : -1;
}

// ElemState cost / feasibility of element b at the start of the inner iteration
// (MultiPhaseDDP.cpp:306-307; the reference's summation order): the half-wave's 32 lanes stage the
// element's slot costs and |Defect|^2 in `stg` (the item's LDS, not yet in use; every load in flight
// at once), then lane g < P sums phase g's slots in slot order and every lane adds the phase sums in
// phase order (compute_cost's order).  stg == nullptr (horizons too long for it): the lanes read
// global memory directly, ten slots' loads in flight.
template <bool EL>
DEV void element_cost(const Params &p, const Bufs &d, int b, int lane, double *stg, double &cost, double &feas)
{
    const auto LY = layout_of<EL>(d, b);
    const int P = LY.P(), g = lane & 31;
    const double *c = d.slot_cost + (size_t)b * p.S, *f = d.slot_feas + (size_t)b * p.S;
    if (stg) {  // (p.S <= 512: the fp64 item holds two arrays of 509)
        const int Sel = LY.S();
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const int sl = g + 32 * t;
            if (sl < Sel) {
                stg[sl] = c[sl];
                stg[p.S + sl] = f[sl];
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        c = stg;
        f = stg + p.S;
    }
    double ci = 0.0, fi = 0.0;
    if (g < P) {
        const int N = LY.N(g), s0 = LY.s0(g);
#pragma unroll 10
        for (int k = 0; k < N; ++k) {
            ci += c[s0 + k];
            fi += f[s0 + k];
        }
        ci += c[s0 + N];
        fi += f[s0 + N];
    }
    cost = 0.0; feas = 0.0;
    for (int i = 0; i < P; ++i) {
        cost += __shfl(ci, (lane & 32) + i);
        feas += __shfl(fi, (lane & 32) + i);
    }
    feas = sqrt(feas);
}

DEV Lane make_lane()
{
    Lane L;
    L.lane = threadIdx.x & 63;  // (k_riccati_cs: the lane within its wave)
    L.e = L.lane >> 5;
    L.pp = L.lane & 31;
    L.pos = L.lane & 15;
    L.row = L.pp < NX;
    L.qlane = L.pos < HC;
    const int lq = (L.qlane ? L.pos : 0) / 3, aq = L.pos % 3;
#pragma unroll
    for (int a = 0; a < 3; ++a) L.rb[a] = V_RB + 6 * lq + rb_index(aq, a);
    L.xkind = (L.pp >= 3 && L.pp < 6) ? 1 : (L.pp >= 12 && L.pp < NX) ? 2 : 0;
    L.xc0 = L.xkind == 1 ? 12 + (L.pp - 3) : L.xkind == 2 ? 3 + (L.pp - 12) % 3 : MS - 1;
    return L;
}

template <typename LdsT>
DEV void zero_init(LdsT &S, int lane)
{
    if (lane < 32) S.zero[lane] = 0;
    SSYNC();
}

}  // namespace sweep

using namespace sweep;

// backward_sweep_regularized (MultiPhaseDDP.cpp:141-181) for elements 2 blockIdx and 2 blockIdx + 1:
// the sweep with each element's mu, then (for an element whose first sweep fails and that the
// parallel retry cannot take) mu = max(mu * update_regularization, 1e-3) until a sweep succeeds or
// mu > 1e2, then mu / 20 (0 below 1e-6) as the next regularisation.
template <typename real, bool EL, bool DV, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(WPB == 2 ? SWEEP_WPB2_WPE : 2))) void k_riccati(Params p, Bufs d)
{
    // WPB independent waves per workgroup, each with its own LDS and element pair (no barrier couples
    // them; sweep_wpb)
    __shared__ Lds<real> SS[WPB];
    const int wv = WPB > 1 ? __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) : 0;
    Lds<real> &S = SS[wv];
    const int pair = (int)blockIdx.x * WPB + wv;
    const Lane L = make_lane();
    zero_init(S, L.lane);
#if HSDDP_STAMPS
    if (L.lane < 12) S.st[L.lane] = 0;
#endif
    // the wave's two elements: 2 pair + e, or a pair of elements with one layout (Bufs::pairs);
    // an empty half runs on the other half's element, inactive
    int b, bv;
    bool valid;
    if constexpr (EL) {
        if (pair >= p.n_pairs) return;
        const int e0 = d.pairs[2 * pair], e1 = d.pairs[2 * pair + 1];
        b = L.e ? e1 : e0;
        valid = b >= 0;
        bv = valid ? b : (L.e ? e0 : e1);
    } else {
        b = 2 * pair + L.e;
        valid = b < p.B;
        bv = valid ? b : p.B - 1;
    }
    ElemState &E = d.el[bv];
    bool act = valid && !E.done && !E.inner_done;
    if (!__builtin_amdgcn_ballot_w64(act)) return;
    // the slot sums come from k_lq's pass: taken here, all lanes active
    double ecost, efeas;
    {
        // the slot values staged in this item's LDS (free until the sweep starts), two arrays of p.S
        double *stg = 2 * (size_t)p.S * sizeof(double) <= sizeof(S.it[0]) ? reinterpret_cast<double *>(&S.it[L.e]) : nullptr;
        element_cost<EL>(p, d, bv, L.lane, stg, ecost, efeas);
        SSYNC();
    }
    double reg = E.reg;
    Item<real> it;
    it.b = bv;
    it.K = Prec<real>::K(d) + (size_t)bv * p.Kc * KCW;
    it.dU = d.dU + (size_t)bv * p.Kc * NX;
    bool need = act, ok = false;
    double dvk = 0.0;  // DV: Qu^T dU summed over the successful sweep
    for (int attempt = 0; __builtin_amdgcn_ballot_w64(need); ++attempt) {
        it.act = need;
        it.reg = (real)reg;
        double dv;
        const int fk = sweep_pair<real, EL, DV>(p, d, S, L, it, dv);
        if (need) {
            if (fk < 0) {
                ok = true;
                need = false;
                dvk = dv;
            } else {
                bool deferred = false;
                if (attempt == 0 && p.retry_cap > 0) {
                    // the retries run in parallel in k_riccati_retry (the first retry_cap failures
                    // of this launch); k_riccati_select takes the first mu that succeeds
                    int f = 0;
                    if (L.pp == 0) {
                        f = atomicAdd(d.retry_count, 1);
                        if (f < p.retry_cap) d.retry_list[f] = RetryEntry{bv, 0, reg};
                    }
                    f = __shfl(f, L.lane & 32);
                    deferred = f < p.retry_cap;
                }
                if (deferred) {
                    need = false;
                    if (L.pp == 0) { E.iters += 1; E.cost = ecost; E.feas = efeas; E.accepted = 0; }
                    act = false;  // finished by k_riccati_select
                } else {
                    reg = fmax(reg * p.update_regularization, 1e-03);
                    if (reg > 1e2 || attempt >= MAX_REG_ATTEMPTS) need = false;  // goto bad_solve
                }
            }
        }
    }
#if HSDDP_STAMPS
    SSYNC();
    if (L.lane < 12) d.dbg[(size_t)__builtin_amdgcn_readfirstlane(bv) * 16 + L.lane] += S.st[L.lane];
#endif
    if (act && L.pp == 0) {
        double rn = reg / 20;
        if (rn < 1e-06) rn = 0;
        E.iters += 1; E.cost = ecost; E.feas = efeas; E.accepted = 0;
        if (ok) E.reg = rn;
        else { E.reg = rn; E.status = 1; E.done = 1; E.ls_active = 0; }
        // single shooting: merit and early exit from the sweep's dV (MultiPhaseDDP.cpp:326-343)
        if (DV && ok) merit_step(p, E, dvk, -dvk);
    }
}

// k_riccati for small batches (column split, launch_riccati's choice): one element pair per
// workgroup of two waves, wave W running sweep_pair with knot_cs<W> — the same sweeps, attempts and
// outcomes as k_riccati (each wave computes the values the other multiplies by, so both take the
// same branches); wave 0 alone writes the element state and the retry list.  fp64; DV: single
// shooting's dV from the sweep, as k_riccati.  At small batches k_riccati runs one wave per SIMD and its knot is one dependent chain
// of ~11 k cycles; split, each wave issues ~970 of the 1 197 VALU instructions of a knot (static
// count of the knot loops) and the knot takes ~10 % less (sweep_split).
template <bool EL, bool DV, int W>
DEV void riccati_cs_wave(const Params &p, const Bufs &d, LdsCS<double> &S)
{
    using real = double;
    const Lane L = make_lane();
    int b, bv;
    bool valid;
    if constexpr (EL) {
        const int e0 = d.pairs[2 * blockIdx.x], e1 = d.pairs[2 * blockIdx.x + 1];
        b = L.e ? e1 : e0;
        valid = b >= 0;
        bv = valid ? b : (L.e ? e0 : e1);
    } else {
        b = 2 * blockIdx.x + L.e;
        valid = b < p.B;
        bv = valid ? b : p.B - 1;
    }
    ElemState &E = d.el[bv];
    bool act = valid && !E.done && !E.inner_done;
    // (act is the same in both waves: both return here, or neither)
    if (!__builtin_amdgcn_ballot_w64(act)) return;
    double ecost = 0, efeas = 0;
    if (W == 0) {
        double *stg = 2 * (size_t)p.S * sizeof(double) <= sizeof(S.it[0]) ? reinterpret_cast<double *>(&S.it[L.e]) : nullptr;
        element_cost<EL>(p, d, bv, L.lane, stg, ecost, efeas);
    }
    CSYNC();  // (the staging area is the item's images)
    double reg = E.reg;
    Item<real> it;
    it.b = bv;
    it.K = d.K + (size_t)bv * p.Kc * KCW;
    it.dU = d.dU + (size_t)bv * p.Kc * NX;
    bool need = act, ok = false;
    double dvk = 0.0;  // DV: Qu^T dU summed over the successful sweep
    for (int attempt = 0; __builtin_amdgcn_ballot_w64(need); ++attempt) {
        it.act = need;
        it.reg = (real)reg;
        double dv;
        const int fk = sweep_pair<real, EL, DV, W>(p, d, S, L, it, dv);
        if (attempt == 0 && p.retry_cap > 0) {  // wave 0 takes the retry slots, both read them
            if (W == 0 && need && fk >= 0 && L.pp == 0) {
                const int f = atomicAdd(d.retry_count, 1);
                if (f < p.retry_cap) d.retry_list[f] = RetryEntry{bv, 0, reg};
                S.fl[L.e] = f;
            }
            CSYNC();
        }
        if (need) {
            if (fk < 0) {
                ok = true;
                need = false;
                dvk = dv;
            } else {
                const bool deferred = attempt == 0 && p.retry_cap > 0 && S.fl[L.e] < p.retry_cap;
                if (deferred) {
                    need = false;
                    if (W == 0 && L.pp == 0) { E.iters += 1; E.cost = ecost; E.feas = efeas; E.accepted = 0; }
                    act = false;
                } else {
                    reg = fmax(reg * p.update_regularization, 1e-03);
                    if (reg > 1e2 || attempt >= MAX_REG_ATTEMPTS) need = false;
                }
            }
        }
        CSYNC();  // (S.fl read by both before a later attempt could rewrite it)
    }
    if (W == 0 && act && L.pp == 0) {
        double rn = reg / 20;
        if (rn < 1e-06) rn = 0;
        E.iters += 1; E.cost = ecost; E.feas = efeas; E.accepted = 0;
        E.reg = rn;
        if (!ok) { E.status = 1; E.done = 1; E.ls_active = 0; }
        if (DV && ok) merit_step(p, E, dvk, -dvk);  // single shooting (k_riccati's epilogue)
    }
}

template <bool EL, bool DV>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void k_riccati_cs(Params p, Bufs d)
{
    __shared__ LdsCS<double> S;
    zero_init(S, threadIdx.x & 63);
    __syncthreads();
    if (threadIdx.x < 64) riccati_cs_wave<EL, DV, 0>(p, d, S);
    else riccati_cs_wave<EL, DV, 1>(p, d, S);
}

// The retries of backward_sweep_regularized for the elements k_riccati deferred, all at once:
// item (f, a) sweeps deferred element f with the a-th next mu of the schedule into its own scratch
// rows, two items per wave.  Every attempt is the sweep the sequential loop would run with that mu,
// so taking the first success (k_riccati_select) gives the loop's result.
template <typename real, bool EL, bool DV>
__global__ __launch_bounds__(64, 2) void k_riccati_retry(Params p, Bufs d)
{
    __shared__ Lds<real> S;
    const Lane L = make_lane();
    zero_init(S, L.lane);
    const int n = min(*d.retry_count, p.retry_cap);
    // attempts a = 1 .. retry_m of deferred element f, padded to an even count so that a wave's two
    // items always belong to one element (one layout)
    const int mpad = p.retry_m + (p.retry_m & 1);
    const int item = 2 * blockIdx.x + L.e, f = item / mpad, a = item % mpad + 1;
    bool act = f < n && a <= p.retry_m;
    if (!__builtin_amdgcn_ballot_w64(act)) return;
    const int fv = f < n ? f : 0;
    const RetryEntry e = d.retry_list[fv];
    double reg = e.reg;
    for (int t = 0; t < a; ++t) reg = fmax(reg * p.update_regularization, 1e-03);
    const int av = a <= p.retry_m ? a : p.retry_m;  // a padding item addresses the last attempt's rows, inactive
    int *flag = d.retry_flag + fv * p.retry_m + (av - 1);
    if (act && reg > 1e2) {  // past the loop's exit: never tried (the schedule is non-decreasing)
        if (L.pp == 0) *flag = 2;
        act = false;
    }
    if (!__builtin_amdgcn_ballot_w64(act)) return;
    const size_t slot = (size_t)fv * p.retry_m + (av - 1);
    Item<real> it;
    it.b = e.b;
    it.act = act;
    it.reg = (real)reg;
    it.K = (real *)d.retry_K + slot * p.Kc * KCW;
    it.dU = d.retry_dU + slot * p.Kc * NX;
    double dv;
    const int fk = sweep_pair<real, EL, DV>(p, d, S, L, it, dv);
    if (act && L.pp == 0) *flag = fk < 0 ? 1 : -1 - fk;  // success, or -1 - (the failing control slot)
    if (DV && act && L.pp == 0) d.retry_dv[slot] = dv;
}

// The outcome of backward_sweep_regularized for each deferred element: the first attempt that
// succeeded (its gains and dU rows copied to the element), mu / 20 (0 below 1e-6) as the next
// regularisation; when none succeeds (mu passed 1e2: status 1, bad_solve) the element's rows are
// left as the sequential loop leaves them: row kc from the last attempt that got past it.
template <typename real>
__global__ __launch_bounds__(64) void k_riccati_select(Params p, Bufs d)
{
    const int f = blockIdx.x, lane = threadIdx.x;
    if (f >= min(*d.retry_count, p.retry_cap)) return;
    const RetryEntry e = d.retry_list[f];
    const size_t b = e.b;
    double reg = e.reg;
    int win = 0;
    for (int a = 1; a <= p.retry_m; ++a) {
        reg = fmax(reg * p.update_regularization, 1e-03);
        if (reg > 1e2) break;
        if (d.retry_flag[f * p.retry_m + a - 1] == 1) { win = a; break; }
    }
    real *Ko = Prec<real>::K(d) + b * p.Kc * KCW;
    double *dUo = d.dU + b * p.Kc * NX;
    if (win) {
        const size_t slot = (size_t)f * p.retry_m + (win - 1);
        const real *Ks = (const real *)d.retry_K + slot * p.Kc * KCW;
        const double *Us = d.retry_dU + slot * p.Kc * NX;
        for (size_t q = lane; q < (size_t)p.Kc * KCW; q += 64) Ko[q] = Ks[q];
        for (size_t q = lane; q < (size_t)p.Kc * NX; q += 64) dUo[q] = Us[q];
    } else {
        const int *fl = d.retry_flag + f * p.retry_m;
        // attempt a wrote the rows above its failing slot -1 - fl[a - 1]; attempts stop at flag 2
        auto source = [&](int kc) {
            int src = 0;
            for (int a = 1; a <= p.retry_m && fl[a - 1] != 2; ++a)
                if (-1 - fl[a - 1] < kc) src = a;
            return src;
        };
        const real *K0 = (const real *)d.retry_K + (size_t)f * p.retry_m * p.Kc * KCW;
        const double *U0 = d.retry_dU + (size_t)f * p.retry_m * p.Kc * NX;
        for (size_t q = lane; q < (size_t)p.Kc * KCW; q += 64) {
            const int a = source((int)(q / KCW));
            if (a) Ko[q] = K0[(size_t)(a - 1) * p.Kc * KCW + q];
        }
        for (size_t q = lane; q < (size_t)p.Kc * NX; q += 64) {
            const int a = source((int)(q / NX));
            if (a) dUo[q] = U0[(size_t)(a - 1) * p.Kc * NX + q];
        }
    }
    if (lane == 0) {
        ElemState &E = d.el[b];
        double rn = reg / 20;
        if (rn < 1e-06) rn = 0;
        E.reg = rn;
        if (!win) { E.status = 1; E.done = 1; E.ls_active = 0; }  // goto bad_solve
        else if (p.ms0) {  // single shooting: merit from the winning attempt's dV (k_riccati's epilogue)
            const double dv = d.retry_dv[(size_t)f * p.retry_m + (win - 1)];
            merit_step(p, E, dv, -dv);
        }
    }
}

// the column split (k_riccati_cs) when its workgroups take at most one CU each (B <= 512), in fp64
// (multiple or single shooting); HSDDP_SWEEP_SPLIT = 0 / 1 forces it off / on (tests, A/B).  Measured
// (one box, sweep ms per step at B = 64 / 256 / 512 / 1024 / 2048): split 0.738 / 0.740 / 0.757 /
// 1.075 / 1.343, one-wave 0.821 / 0.825 / 0.836 / 0.951 / 1.372 — from two workgroups per CU on,
// the waves of one CU slow each other (the one-wave kernel too: 0.84 -> 0.95 ms from 256 to 512
// waves at an unchanged 2.3 GHz clock), and the split's two waves per pair lose.
// The thresholds below scale with the current device's CU count (256 on an MI355X: the
// measurements above), so a partitioned or smaller device keeps the same placement rules.
static int device_cus()
{
    static int cus[64] = {0};
    int dev = 0;
    hipGetDevice(&dev);
    if (dev < 0 || dev >= 64) return 256;
    if (!cus[dev]) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n < 1) n = 256;
        cus[dev] = n;
    }
    return cus[dev];
}

static bool sweep_split(const Params &p)
{
    if (p.fp32) return false;
    const char *e = std::getenv("HSDDP_SWEEP_SPLIT");
    if (e && *e) return *e != '0';
    return (p.elem_layout ? p.n_pairs : (p.B + 1) / 2) <= device_cus();  // one workgroup per CU
}

// waves (element pairs) per workgroup of the one-wave sweep k_riccati in fp64: 2 while the launch has
// at most one wave per SIMD (257 .. 1024 pairs), 1 from two waves per SIMD on; HSDDP_SWEEP_WPB = 1 / 2
// forces it (tests, A/B).  Measured (one box, split off, sweep ms per step at B = 512 / 1024 / 2048 /
// 4096): two per workgroup 0.866 / 0.883 / 1.29 / 1.61, one 0.812 / 0.913 / 1.36 / 1.59 — a
// workgroup's two waves go to different SIMDs of one CU, which the single-wave workgroups of a
// half-full launch do not reliably do.
static int sweep_wpb(const Params &p)
{
    if (p.fp32) return 1;
    const char *e = std::getenv("HSDDP_SWEEP_WPB");
    if (e && *e) return *e == '2' ? 2 : 1;
    const int pairs = p.elem_layout ? p.n_pairs : (p.B + 1) / 2, cus = device_cus();
    return pairs > cus && pairs <= 4 * cus ? 2 : 1;  // at most one wave per SIMD (4 per CU)
}

void launch_riccati(const Params &p, const Bufs &d, hipStream_t st)
{
    // (the retry list count is zeroed by the k_lq launch just before, in its first terminal task)
    const dim3 g1((unsigned)(p.elem_layout ? p.n_pairs : (p.B + 1) / 2));
    // instantiations: precision x layout mode x single shooting (DV)
#define HSDDP_RIC(kern, grid, real)                                                                          \
    do {                                                                                                     \
        if (p.ms0) {                                                                                         \
            if (p.elem_layout) hipLaunchKernelGGL((kern<real, true, true>), grid, dim3(64), 0, st, p, d);      \
            else hipLaunchKernelGGL((kern<real, false, true>), grid, dim3(64), 0, st, p, d);                   \
        } else {                                                                                             \
            if (p.elem_layout) hipLaunchKernelGGL((kern<real, true, false>), grid, dim3(64), 0, st, p, d);     \
            else hipLaunchKernelGGL((kern<real, false, false>), grid, dim3(64), 0, st, p, d);                  \
        }                                                                                                    \
    } while (0)
    const int wpb = sweep_wpb(p);
    const dim3 gw((unsigned)(((p.elem_layout ? p.n_pairs : (p.B + 1) / 2) + wpb - 1) / wpb));
#define HSDDP_RIC_W(real, W)                                                                                   \
    do {                                                                                                       \
        if (p.ms0) {                                                                                           \
            if (p.elem_layout) hipLaunchKernelGGL((k_riccati<real, true, true, W>), gw, dim3(64 * W), 0, st, p, d);  \
            else hipLaunchKernelGGL((k_riccati<real, false, true, W>), gw, dim3(64 * W), 0, st, p, d);               \
        } else {                                                                                               \
            if (p.elem_layout) hipLaunchKernelGGL((k_riccati<real, true, false, W>), gw, dim3(64 * W), 0, st, p, d); \
            else hipLaunchKernelGGL((k_riccati<real, false, false, W>), gw, dim3(64 * W), 0, st, p, d);              \
        }                                                                                                      \
    } while (0)
    if (p.fp32) HSDDP_RIC_W(float, 1);
    else if (sweep_split(p)) {
        if (p.ms0) {
            if (p.elem_layout) hipLaunchKernelGGL((k_riccati_cs<true, true>), g1, dim3(128), 0, st, p, d);
            else hipLaunchKernelGGL((k_riccati_cs<false, true>), g1, dim3(128), 0, st, p, d);
        } else {
            if (p.elem_layout) hipLaunchKernelGGL((k_riccati_cs<true, false>), g1, dim3(128), 0, st, p, d);
            else hipLaunchKernelGGL((k_riccati_cs<false, false>), g1, dim3(128), 0, st, p, d);
        }
    } else if (wpb == 2) HSDDP_RIC_W(double, 2);
    else HSDDP_RIC_W(double, 1);
#undef HSDDP_RIC_W
    if (p.retry_cap > 0) {
        const dim3 gr((unsigned)(p.retry_cap * (p.retry_m + (p.retry_m & 1)) / 2)), gs((unsigned)p.retry_cap);
        if (p.fp32) {
            HSDDP_RIC(k_riccati_retry, gr, float);
            hipLaunchKernelGGL(k_riccati_select<float>, gs, dim3(64), 0, st, p, d);
        } else {
            HSDDP_RIC(k_riccati_retry, gr, double);
            hipLaunchKernelGGL(k_riccati_select<double>, gs, dim3(64), 0, st, p, d);
        }
    }
#undef HSDDP_RIC
}

}  // namespace hsddp
