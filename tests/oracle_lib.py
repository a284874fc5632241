"""ctypes bindings for the oracle (test infrastructure: oracle/liboracle.so, oracle/_ref).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB_PATH = os.path.join(ORACLE_DIR, "liboracle.so")
REF_PATH = os.path.join(ORACLE_DIR, "_ref", "libhkd_casadi_ref.so")

DP = C.POINTER(C.c_double)
IP = C.POINTER(C.c_int)


class OrcOptions(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("alpha", "gamma", "update_penalty", "update_relax",
                                          "update_regularization", "update_ReB")] + \
               [(n, C.c_int) for n in ("max_DDP_iter", "max_AL_iter", "max_DDP_iter_runtime",
                                       "max_AL_iter_runtime")] + \
               [(n, C.c_double) for n in ("cost_thresh", "tconstr_thresh", "pconstr_thresh",
                                          "dynamics_feas_thresh", "merit_rho", "merit_scale",
                                          "merit_offset")] + \
               [(n, C.c_int) for n in ("AL_active", "ReB_active", "smooth_active", "MS",
                                       "nsteps_per_node", "no_early_exit")]


class OrcWeights(C.Structure):
    _fields_ = [("q_eul", C.c_double * 3), ("q_pos", C.c_double * 3), ("q_omega", C.c_double * 3),
                ("q_v", C.c_double * 3), ("q_qJ", C.c_double), ("qf_scale", C.c_double * 24),
                ("qf_gain", C.c_double), ("r_grf", C.c_double), ("r_qJd", C.c_double),
                ("foot_w", C.c_double * 3), ("foot_gain", C.c_double),
                ("foot_term_cost", C.c_double), ("foot_term_grad", C.c_double)]


class OrcProblem(C.Structure):
    _fields_ = [("n_phases", C.c_int), ("horizons", IP), ("dt", C.c_double), ("mu_fric", C.c_double),
                ("grf_delta", C.c_double), ("grf_delta_min", C.c_double), ("grf_eps", C.c_double),
                ("td_sigma", C.c_double), ("td_sigma_max", C.c_double), ("td_lambda", C.c_double),
                ("ground_height", C.c_double), ("w", OrcWeights), ("shooting", IP)]


class OrcElement(C.Structure):
    _fields_ = [("contacts", IP), ("x0", DP), ("ref_x", DP), ("ref_u", DP), ("ref_foot", DP),
                ("Xbar", DP), ("X", DP), ("Defect", DP), ("Defect_bar", DP), ("dX", DP),
                ("Ubar", DP), ("U", DP), ("dU", DP), ("K", DP),
                ("reb_delta", DP), ("reb_eps", DP), ("al_sigma", DP), ("al_lambda", DP), ("td_mask", IP),
                ("grf_g", DP), ("td_h", DP),
                ("cost", C.c_double), ("feas", C.c_double), ("merit", C.c_double),
                ("max_tconstr", C.c_double), ("max_pconstr", C.c_double),
                ("iters", C.c_int), ("outer_iters", C.c_int), ("status", C.c_int),
                ("n_ls_trials", C.c_int), ("hist", C.POINTER(C.c_float)), ("hist_cap", C.c_int),
                ("hist_n", C.c_int), ("diverged_init", C.c_int), ("n_diverged", C.c_int)]


def build(quiet: bool = True) -> None:
    """Compile oracle/liboracle.so (and oracle/_ref when /root/reference is present)."""
    out = subprocess.run(["make", "-C", ORACLE_DIR, "all"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)


_lib = None
_ref = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = C.CDLL(LIB_PATH)
        _lib.orc_solve_batch.argtypes = [C.POINTER(OrcProblem), C.POINTER(OrcOptions),
                                         C.POINTER(OrcElement), C.c_int, C.c_int]
        _lib.orc_solve.argtypes = [C.POINTER(OrcProblem), C.POINTER(OrcOptions), C.POINTER(OrcElement)]
        for f in ("orc_hkd_step",):
            getattr(_lib, f).argtypes = [DP, DP, C.c_double, DP, DP]
        _lib.orc_hkd_partial.argtypes = [DP, DP, C.c_double, DP, DP, DP]
        _lib.orc_foot_position.argtypes = [C.c_int, DP, DP, DP, DP]
        _lib.orc_foot_jacobian.argtypes = [C.c_int, DP, DP, DP, DP]
        _lib.orc_resetmap.argtypes = [DP, IP, IP, DP]
        _lib.orc_resetmap_partial.argtypes = [DP, IP, IP, DP]
        _lib.orc_knot_eval.argtypes = [C.POINTER(OrcProblem), C.POINTER(OrcOptions), IP, IP] + [DP] * 13
        _lib.orc_riccati_lq.argtypes = [C.c_int] + [DP] * 8 + [C.c_double] + [DP] * 4
    return _lib


def ref_lib():
    """The reference's own CasADi kernels (oracle/_ref); None when not built."""
    global _ref
    if _ref is None and os.path.exists(REF_PATH):
        _ref = C.CDLL(REF_PATH)
        _ref.ref_hkinodyn.argtypes = [DP, DP, C.c_double, DP, DP]
        _ref.ref_hkinodyn_par.argtypes = [DP, DP, C.c_double, DP, DP, DP]
        _ref.ref_foot_position.argtypes = [DP, DP, DP, C.c_double, DP]
        _ref.ref_foot_jacobian.argtypes = [C.c_int, DP, DP, DP, DP]
    return _ref


def dp(a):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(DP)


def ip(a):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(IP)


def default_options(**kw) -> OrcOptions:
    o = OrcOptions()
    lib().orc_default_options(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def default_problem(horizons, dt=0.01) -> tuple:
    hz = np.asarray(horizons, dtype=np.int32)
    p = OrcProblem()
    p.n_phases = len(hz)
    p.horizons = ip(hz)
    p.dt = dt
    p.mu_fric = 0.7
    p.grf_delta, p.grf_delta_min, p.grf_eps = 0.1, 0.1, 0.1
    p.td_sigma, p.td_sigma_max, p.td_lambda = 50.0, 1e4, 0.0
    p.ground_height = 0.0
    lib().orc_default_weights(C.byref(p.w))
    return p, hz


# ---- model wrappers ---------------------------------------------------------------------------
def hkd_step(x, u, dt, c):
    o = np.zeros(24)
    lib().orc_hkd_step(dp(np.ascontiguousarray(x, float)), dp(np.ascontiguousarray(u, float)), dt,
                       dp(np.ascontiguousarray(c, float)), dp(o))
    return o


def hkd_partial(x, u, dt, c):
    A = np.zeros((24, 24)); B = np.zeros((24, 24))
    lib().orc_hkd_partial(dp(np.ascontiguousarray(x, float)), dp(np.ascontiguousarray(u, float)), dt,
                          dp(np.ascontiguousarray(c, float)), dp(A), dp(B))
    return A, B


def resetmap(x, c, cn):
    o = np.zeros(24)
    lib().orc_resetmap(dp(np.ascontiguousarray(x, float)), ip(np.asarray(c, np.int32)),
                       ip(np.asarray(cn, np.int32)), dp(o))
    return o


def resetmap_partial(x, c, cn):
    o = np.zeros((24, 24))
    lib().orc_resetmap_partial(dp(np.ascontiguousarray(x, float)), ip(np.asarray(c, np.int32)),
                               ip(np.asarray(cn, np.int32)), dp(o))
    return o


def knot_eval(c, cn, x, u, xr, ur, pf, x_end=None, xr_end=None, pf_end=None, reb_delta=None, reb_eps=None,
              sigma=None, lam=None, options=None, dt=0.01, weights=None) -> dict:
    """orc_knot_eval: one knot's cost and LQ model, and one phase end's terminal data, alone."""
    p, _hz = default_problem([1], dt)
    for k, v in (weights or {}).items():
        setattr(p.w, k, v)
    o = options or default_options()
    f = lambda a, n: np.ascontiguousarray(np.zeros(n) if a is None else a, dtype=np.float64)
    args = [f(x, 24), f(u, 24), f(xr, 24), f(ur, 24), f(pf, 12), f(x if x_end is None else x_end, 24),
            f(xr if xr_end is None else xr_end, 24), f(pf if pf_end is None else pf_end, 12),
            f(np.full(20, p.grf_delta) if reb_delta is None else reb_delta, 20),
            f(np.full(20, p.grf_eps) if reb_eps is None else reb_eps, 20),
            f(np.full(4, p.td_sigma) if sigma is None else sigma, 4), f(np.full(4, p.td_lambda) if lam is None else lam, 4)]
    out = np.zeros(2 + 3 * 24 + 6 * 576)
    ci = np.asarray(c, np.int32); cni = np.asarray(cn, np.int32)
    lib().orc_knot_eval(C.byref(p), C.byref(o), ip(ci), ip(cni), *[dp(a) for a in args], dp(out))
    N = 576
    r = {"l": out[0], "Phi": out[1], "lx": out[2:26], "lu": out[26:50]}
    q = 50
    for k in ("lxx", "luu", "lux"):
        r[k] = out[q:q + N].reshape(24, 24); q += N
    r["Phix"] = out[q:q + 24]; q += 24
    for k in ("Phixx", "A", "B"):
        r[k] = out[q:q + N].reshape(24, 24); q += N
    return r


def riccati_lq(N, A, B, lxx, luu, lx=None, lu=None, Phix=None, Phixx=None, reg=0.0):
    """orc_riccati_lq: SinglePhase::backward_sweep on time-invariant LQ data over N knots (zero
    defects); returns (ok, K0, dU0, G0, H0)."""
    f = lambda a, shape: np.ascontiguousarray(np.zeros(shape) if a is None else a, dtype=np.float64)  # noqa: E731
    args = [f(A, (24, 24)), f(B, (24, 24)), f(lxx, (24, 24)), f(luu, (24, 24)), f(lx, 24), f(lu, 24), f(Phix, 24),
            f(Phixx, (24, 24))]
    K0, H0, dU0, G0 = np.zeros((24, 24)), np.zeros((24, 24)), np.zeros(24), np.zeros(24)
    ok = lib().orc_riccati_lq(int(N), *[dp(a) for a in args], float(reg), dp(K0), dp(dU0), dp(G0), dp(H0))
    return bool(ok), K0, dU0, G0, H0


# ---- solver -----------------------------------------------------------------------------------
MAX_TD = 4  # ORC_MAX_TD / HSDDP_MAX_TD
CONSTRAINT_FIELDS = ("reb_delta", "reb_eps", "al_sigma", "al_lambda", "td_mask")
# what else lives on from solve to solve in the reference's objects: the working trajectory (X, U,
# Defect: Trajectory, TrajectoryManagement.cpp) and the constraint objects' stored values (GRF g per
# knot and row, touchdown h per constraint and leg: ConstraintsBase.h:12-55)
STATE_FIELDS = ("X", "U", "Defect", "grf_g", "td_h")


def solve_batch(prob: dict, options: OrcOptions | None = None, n_threads: int = 1,
                elements=None, weights: dict | None = None, constraints: dict | None = None,
                state: dict | None = None) -> dict:
    """Run the oracle solve on (a subset of) a synthetic batch; returns per-element outputs.
    weights: HKD cost-weight overrides by field name (e.g. {"r_qJd": -0.5}).
    constraints: the elements' constraint parameters (CONSTRAINT_FIELDS, [B] leading axis) to start
    from instead of a new problem's (orc_init_element) — an MPC tick's carried-over ReB / AL
    parameters and touchdown constraints; the outputs carry them after the solve.
    state: STATE_FIELDS ([B] leading axis) to start from instead of a new problem's (X = Xbar,
    U = Ubar, Defect = 0, zero constraint values) — the previous tick's, shifted (mpc_oracle)."""
    options = options or default_options()
    B = prob["batch"]
    idx = list(range(B)) if elements is None else list(elements)
    n = len(idx)
    S, Kc, P = prob["S"], prob["Kc"], len(prob["horizons"])
    p, hz = default_problem(prob["horizons"], prob["dt"])
    for k, v in (weights or {}).items():
        setattr(p.w, k, v)
    ss = None
    if prob.get("shooting") is not None:  # shooting states per phase (after a receding-horizon shift)
        ss = np.ascontiguousarray(prob["shooting"], dtype=np.int32)
        p.shooting = ip(ss)
    st = {
        "Xbar": np.ascontiguousarray(prob["Xbar"][idx]).copy(),
        "X": np.ascontiguousarray(prob["Xbar"][idx]).copy(),
        "Defect": np.zeros((n, S, 24)), "Defect_bar": np.zeros((n, S, 24)), "dX": np.zeros((n, S, 24)),
        "Ubar": np.ascontiguousarray(prob["Ubar"][idx]).copy(),
        "U": np.ascontiguousarray(prob["Ubar"][idx]).copy(), "dU": np.zeros((n, Kc, 24)),
        "K": (np.zeros((n, Kc, 24, 24)) if prob.get("K") is None else np.ascontiguousarray(prob["K"][idx]).copy()),
        "reb_delta": np.zeros((n, Kc, 20)), "reb_eps": np.zeros((n, Kc, 20)),
        "al_sigma": np.zeros((n, P, MAX_TD, 4)), "al_lambda": np.zeros((n, P, MAX_TD, 4)),
        "td_mask": np.zeros((n, P, MAX_TD), np.int32),
        "grf_g": np.zeros((n, Kc, 20)), "td_h": np.zeros((n, P, MAX_TD, 4)),
    }
    contacts = np.ascontiguousarray(prob["contacts"][idx])
    x0 = np.ascontiguousarray(prob["x0"][idx])
    shared = prob["ref_x"].shape[0] == 1
    elems = (OrcElement * n)()
    keep = [contacts, x0, hz, ss]
    for j, b in enumerate(idx):
        e = elems[j]
        rb = 0 if shared else b
        e.contacts = ip(contacts[j])
        e.x0 = dp(x0[j])
        rx = np.ascontiguousarray(prob["ref_x"][rb]); ru = np.ascontiguousarray(prob["ref_u"][rb])
        rf = np.ascontiguousarray(prob["ref_foot"][rb])
        keep += [rx, ru, rf]
        e.ref_x, e.ref_u, e.ref_foot = dp(rx), dp(ru), dp(rf)
        for k in st:
            setattr(e, k, ip(st[k][j]) if st[k].dtype == np.int32 else dp(st[k][j]))
        lib().orc_init_element(C.byref(p), C.byref(e))
        if constraints is not None:
            for k in CONSTRAINT_FIELDS:
                st[k][j] = constraints[k][b]
        if state is not None:
            for k in STATE_FIELDS:
                st[k][j] = state[k][b]
    hcap = 1 + options.max_AL_iter * options.max_DDP_iter
    hist = np.zeros((n, hcap, 4), np.float32)
    for j in range(n):
        elems[j].hist = hist[j].ctypes.data_as(C.POINTER(C.c_float))
        elems[j].hist_cap = hcap
    lib().orc_solve_batch(C.byref(p), C.byref(options), elems, n, n_threads)
    out = dict(st)
    for f in ("cost", "feas", "merit", "max_tconstr", "max_pconstr", "iters", "outer_iters", "status",
              "n_ls_trials", "diverged_init", "n_diverged"):
        out[f] = np.array([getattr(elems[j], f) for j in range(n)])
    # get_solver_info buffers per element: [n_j][4] (cost, dyn_feas, eqn_feas, ineq_feas)
    out["solver_info"] = [hist[j, :min(elems[j].hist_n, hcap)].copy() for j in range(n)]
    return out
