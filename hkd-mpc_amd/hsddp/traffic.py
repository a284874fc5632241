"""Algorithmic HBM bytes and fp64 FLOPs of one DDP inner iteration, per kernel.

These are the bytes each kernel must move in THIS design's compact layout (hsddp_internal.h): a
knot's LQ model is the 176-value record (A - I and B non-zeros, lx, lu, dt * ReB Hessian), the
gains are the 12 coupled rows (12 x 24), lxx and luu's diagonal are rebuilt from parameters.  They
replace SURVEY.md §8(d)'s dense per-knot model (A, B, lxx, luu, lux materialised as 24 x 24
matrices, 88 KB per knot), which prices traffic this design never generates.

Every figure counts each byte a kernel reads or writes in HBM once per launch (reads of the same
row by neighbouring lanes or knots are one read).  Per-handle constants (contacts, the shared
reference of a common gait, Params) are < 0.1 % and left out; per-element references (mixed
gaits) are counted.

    B  elements, S state slots (sum N_i + 1), Kc control slots (sum N_i), P phases.
"""
from __future__ import annotations

NX = 24
LQW, LQW32 = 176, 176   # compact LQ record (fp64 / fp32 stride), hsddp_internal.h
KCW = 12 * 24           # compact gain rows
TW_PHI = 24 + 576       # Phix + Phixx per phase end
TW_PX = 576             # reset-map Jacobian per phase boundary (read)
TW_PX_W = 288           # its rows 12 .. 23 (written: rows 0 .. 11 are the identity's, set once at create)


def kernel_bytes(B: int, S: int, Kc: int, P: int, fp32: bool = False, ref_per_element: bool = False,
                 reb_rows: float = 0.0) -> dict:
    """Algorithmic bytes per launch of each kernel of one inner iteration.  reb_rows: GRF rows per
    control knot whose per-knot ReB parameters (delta, eps) the cost kernels read — 5 per stance leg
    unless the schedule keeps them uniform (Params::reb_uniform: then 0, two scalars instead)."""
    d = 8                              # fp64
    f = 4 if fp32 else 8               # Riccati precision: LQ record, gains, Defect copy (C5)
    rec = (LQW32 * 4) if fp32 else (LQW * 8)
    ref = (S * (24 + 12) + Kc * 24) * d if ref_per_element else 0   # ref_x, ref_foot per slot, ref_u per knot
    term = (P * TW_PHI + (P - 1) * TW_PX) * d                      # Phix, Phixx (every phase end), Px (boundaries)
    out = {}
    # k_lq inside the inner loop: per slot X read (the slot costs and |Defect|^2 are the last
    # rollout's: Params::lq_slots = 0), in the fp32 mode Defect read and its fp32 copy written; per
    # control knot U read and the record written
    reb = 2 * reb_rows * d  # delta and eps of the knot's stance-leg GRF rows
    out["k_lq"] = B * (S * (NX * d + (NX * d + NX * 4 if fp32 else 0)) + Kc * (NX * d + rec + reb) + ref)
    # k_terminal: per phase end X read (+ AL sigma, lambda), Phix, Phixx, Px rows 12 .. 23 and the
    # terminal cost written
    out["k_terminal"] = B * (P * (NX + 8 + 1) * d + (P * TW_PHI + (P - 1) * TW_PX_W) * d)
    # k_riccati: per control knot the record and Defect[k+1] read, gain rows and dU written; per
    # element the terminal records and the slot cost / feasibility partial sums read
    out["k_riccati"] = B * (Kc * (rec + NX * f + KCW * f + NX * d) + term + 2 * S * d)
    # k_lin_rollout: per control knot gains, record, Defect, dU read, du and dX written; terminal
    # records read per phase
    out["k_lin_rollout"] = B * (Kc * (KCW * f + rec + NX * f + NX * d + 2 * NX * d) + term)
    # k_rollout (one line-search trial): per slot Xbar, dX read, X, Defect written, cost /
    # feasibility / violation / divergence written; per control knot Ubar, du read, U written
    out["k_rollout"] = B * (S * (4 * NX * d + 4 * d) + Kc * (3 * NX * d + reb) + ref)
    # (Trajectory::update_nominal_vals moves no bytes: k_decide flips the element's buffer selector)
    return out


def step_bytes(B: int, S: int, Kc: int, P: int, n_trials: float, fp32: bool = False,
               ref_per_element: bool = False, reb_rows: float = 0.0) -> float:
    """Algorithmic bytes of one inner iteration: every kernel once, k_rollout n_trials times
    (the measured mean number of line-search trials)."""
    kb = kernel_bytes(B, S, Kc, P, fp32, ref_per_element, reb_rows)
    return sum(v for k, v in kb.items() if k != "k_rollout") + n_trials * kb["k_rollout"]


def reb_rows_per_knot(prob: dict, options, constraint_delta: float = 1.0, constraint_delta_min: float = 0.0) -> float:
    """reb_rows for kernel_bytes: 0 when the ReB schedule keeps (delta, eps) uniform (update_ReB =
    update_relax = 1, hsddp_api.cpp fill_params), else 5 GRF rows per stance leg, averaged over the
    batch's control knots."""
    import numpy as np
    if options.update_ReB == 1.0 and options.update_relax == 1.0 and constraint_delta >= constraint_delta_min:
        return 0.0
    c = np.asarray(prob["contacts"])
    lays = prob.get("layouts")
    if lays:
        per = [sum(n * float(np.sum(c[b, i] != 0)) for i, n in enumerate(h)) / sum(h) for b, h in enumerate(lays)]
        return 5.0 * float(np.mean(per))
    h = prob["horizons"]
    stance = np.array([[float(np.sum(c[b, i] != 0)) for i in range(len(h))] for b in range(c.shape[0])])
    return 5.0 * float(np.mean(stance @ np.asarray(h, float)) / sum(h))


# fp64 FMAs of one knot of the backward sweep as k_riccati evaluates it (structure exploited:
# A = I + S with 69 non-zeros of S, B_c with 48 non-zeros, 12 coupled controls, symmetric value
# update).  Each term is the product's multiply-add count.
RICCATI_FMA_PER_KNOT = {
    "Gn = G + H d": 24 * 24,
    "T = H B_c": 24 * 48,
    "M = H A (S part)": 24 * 69,
    "Qx = lx + A^T Gn": 69,
    "Qu_c = lu + B_c^T Gn": 48,
    "Qxx = lxx + A^T M (S part)": 24 * 69,
    "Qux_c = B_c^T M": 12 * 24 * 4,
    "Quu_cc = luu + B_c^T T": 12 * 48,
    "[Quu_cc | Qux_c | Qu_c] elimination": 12 * 11 * 37,
    "P = Qux_c^T Kp": 24 * 24 * 12,
    "G = Qx - Qux_c^T k": 24 * 12,
}
RICCATI_FLOP_PER_KNOT = 2 * sum(RICCATI_FMA_PER_KNOT.values())
