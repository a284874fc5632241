"""Synthetic batches whose line-search rollouts break the reference's divergence bound (test
infrastructure for tests/test_gpu_divergence.py).

SinglePhase::hybrid_rollout stops at the first knot whose simulated state has a 2-norm above 1e6
(SinglePhase.cpp:205-208).  The HKD model is invariant under a translation along x of the body
position and of the stance feet's world positions (the lever arms, foot residuals and foot heights
are differences or z-coordinates; swing feet are joint angles and the tracking weight of a stance
foot state is zero), so translating an element by T leaves its solve unchanged while its state
norms grow like T (sqrt(1 + stance legs) T).  The first iteration's trial states of the
untranslated problem (Xbar + eps dX at the shooting states, Ubar + eps (dU + K dX)) come from one
oracle iteration; per element, T is then set by bisection so that the bound falls between the
largest simulated-state norm at two step sizes:
  "none": below every trial;   "one": eps = 1 breaks, eps = 0.1 does not;
  "all":  eps = 0.001 (every trial) breaks, the nominal (eps = 0, the initial rollout) does not.
"""
import os
import sys

import numpy as np

import oracle_lib as O
from hsddp import synthetic as syn

BOUND = 1e6


def _phases(horizons):
    s0 = np.cumsum([0] + [n + 1 for n in horizons])
    k0 = np.cumsum([0] + list(horizons))
    return s0, k0


def direction(prob, b):
    """[S][24] translation direction of element b: body x and the stance feet's x per slot"""
    hz = prob["horizons"]
    s0, _ = _phases(hz)
    e = np.zeros((prob["S"], 24))
    c = prob["contacts"][b]
    for i, n in enumerate(hz):
        for k in range(n + 1):
            e[s0[i] + k, 3] = 1
            for l in range(4):
                if c[i][l]:
                    e[s0[i] + k, 12 + 3 * l] = 1
    return e


def _sim_norms(prob, r, b, eps, T, e):
    """norms of the simulated states at slots with k >= 1 of the first trial with step eps"""
    hz = prob["horizons"]
    s0, k0 = _phases(hz)
    out = []
    for i, n in enumerate(hz):
        c = prob["contacts"][b][i].astype(float)
        for k in range(1, n + 1):
            s, kc = s0[i] + k, k0[i] + k - 1
            dx = eps * r["dX"][b, s - 1]
            x = prob["Xbar"][b, s - 1] + dx
            u = prob["Ubar"][b, kc] + eps * r["dU"][b, kc] + r["K"][b, kc] @ dx
            xn = O.hkd_step(x, u, prob["dt"], c) + T * e[s]
            out.append(np.linalg.norm(xn))
    return np.array(out)


def make(gait, P, N, B, seed=syn.SEED):
    """(prob, kinds [B], T [B], e [B][S][24]): a per-element-reference batch, element b translated by
    T[b] e[b] to be of kind kinds[b].  Elements whose largest simulated-state norm grows with the
    step size take "one" and "all" in turn, the others "none"."""
    base = syn.make_batch(B, P, N, gait, seed=seed)
    kw = dict(no_early_exit=1, max_AL_iter=1, max_DDP_iter=1, gamma=1e6)
    r = O.solve_batch(base, O.default_options(**kw), n_threads=min(B, 8))
    S = base["S"]
    T = np.zeros(B)
    es = np.stack([direction(base, b) for b in range(B)])
    kinds, nxt = [], "one"
    for b in range(B):
        m = [_sim_norms(base, r, b, eps, 0.5 * BOUND, es[b]).max() for eps in (0.0, 1e-3, 0.1, 1.0)]
        if m[0] < m[1] < m[2] < m[3] and m[1] - m[0] > 1e-6:
            kinds.append(nxt)
            nxt = "all" if nxt == "one" else "one"
        else:
            kinds.append("none")
    for b, kind in enumerate(kinds):
        if kind == "none":
            continue
        lo, hi = {"one": (0.1, 1.0), "all": (0.0, 1e-3)}[kind]
        M = lambda eps, t: _sim_norms(base, r, b, eps, t, es[b]).max()  # noqa: E731
        a, z = 0.0, 2 * BOUND
        for _ in range(200):  # the bound halfway between the two step sizes' largest norms
            t = 0.5 * (a + z)
            if 0.5 * (M(lo, t) + M(hi, t)) > BOUND:
                z = t
            else:
                a = t
        T[b] = 0.5 * (a + z)
        m_lo, m_hi, m0 = M(lo, T[b]), M(hi, T[b]), M(0.0, T[b])
        assert m_lo < BOUND - 1e-7 and m_hi > BOUND + 1e-7 and m0 < BOUND - 1e-7, (b, kind, m0, m_lo, m_hi)
    prob = dict(base)
    sh = T[:, None, None] * es
    rx = np.repeat(base["ref_x"], B, axis=0) if base["ref_x"].shape[0] == 1 else base["ref_x"].copy()
    ru = np.repeat(base["ref_u"], B, axis=0) if base["ref_u"].shape[0] == 1 else base["ref_u"].copy()
    rf = np.repeat(base["ref_foot"], B, axis=0) if base["ref_foot"].shape[0] == 1 else base["ref_foot"].copy()
    prob["ref_x"] = rx + sh
    prob["ref_u"] = ru
    rf = rf.copy()
    rf[:, :, 0::3] += T[:, None, None]  # every foot's world x (the swing legs' is weighted zero)
    prob["ref_foot"] = rf
    prob["Xbar"] = base["Xbar"] + sh
    prob["x0"] = base["x0"] + T[:, None] * es[:, 0, :]
    assert prob["Xbar"].shape == (B, S, 24)
    return prob, kinds, T, es


def untranslate(X, T, es):
    """state rows [B][S][24] with the elements' translations removed"""
    return X - T[:, None, None] * es


# ---- rollouts that break before any trial: a new problem, an MPC tick ---------------------------
def _nominal_norms(prob, b, T, e):
    """norms of the initial rollout's simulated states (eps = 0: X = Xbar at every shooting state,
    U = Ubar) at slots with k >= 1, element b translated by T e"""
    hz = prob["horizons"]
    s0, k0 = _phases(hz)
    out = []
    for i, n in enumerate(hz):
        c = prob["contacts"][b][i].astype(float)
        for k in range(1, n + 1):
            s, kc = s0[i] + k, k0[i] + k - 1
            out.append(np.linalg.norm(O.hkd_step(prob["Xbar"][b, s - 1], prob["Ubar"][b, kc], prob["dt"], c) + T * e[s]))
    return np.array(out)


def _bisect(f):
    """the T at which the increasing f(T) crosses the bound"""
    a, z = 0.0, 2 * BOUND
    for _ in range(200):
        t = 0.5 * (a + z)
        if f(t) > BOUND:
            z = t
        else:
            a = t
    return 0.5 * (a + z)


def _translated(base, T, es):
    B = base["batch"]
    prob = dict(base)
    sh = T[:, None, None] * es
    rep = lambda a: np.repeat(a, B, axis=0) if a.shape[0] == 1 else a.copy()  # noqa: E731
    prob["ref_x"] = rep(base["ref_x"]) + sh
    prob["ref_u"] = rep(base["ref_u"])
    rf = rep(base["ref_foot"])
    rf[:, :, 0::3] += T[:, None, None]
    prob["ref_foot"] = rf
    prob["Xbar"] = base["Xbar"] + sh
    prob["x0"] = base["x0"] + T[:, None] * es[:, 0, :]
    return prob


def make_init(gait, P, N, B, at=0.5, seed=syn.SEED):
    """(prob, breaks [B], T [B], e [B][S][24]): every other element translated so that the initial
    rollout of a new problem breaks the bound first at the simulated state of knot breaks[b] (about
    `at` of the horizon; -1: untranslated).  The warm-start controls are the reference's (stance
    GRFs carrying the weight), so the zero constraint values a new problem starts from (create_data)
    differ from the values of its control rows at every stance knot the rollout does not reach."""
    base = syn.make_batch(B, P, N, gait, seed=seed)
    s0, _ = _phases(base["horizons"])
    idx = np.concatenate([np.arange(s0[i], s0[i] + n) for i, n in enumerate(base["horizons"])])
    rep = base["ref_u"] if base["ref_u"].shape[0] == B else np.repeat(base["ref_u"], B, axis=0)
    base["Ubar"] = np.ascontiguousarray(rep[:, idx])
    es = np.stack([direction(base, b) for b in range(B)])
    T, breaks = np.zeros(B), []
    for b in range(B):
        if b % 2:
            breaks.append(-1)
            continue
        n0 = _nominal_norms(base, b, 0.5 * BOUND, es[b])
        j = int(at * len(n0))
        while n0[j] <= n0[:j].max():  # the first knot whose norm exceeds every earlier one
            j += 1
        t_at = _bisect(lambda t: _nominal_norms(base, b, t, es[b])[j])
        t_before = _bisect(lambda t: _nominal_norms(base, b, t, es[b])[:j].max())
        assert t_at < t_before, (b, t_at, t_before)
        T[b] = 0.5 * (t_at + t_before)
        m = _nominal_norms(base, b, T[b], es[b])
        assert m[j] > BOUND + 1e-4 and m[:j].max() < BOUND - 1e-4, (b, m[j] - BOUND, m[:j].max() - BOUND)
        breaks.append(j)
    return _translated(base, T, es), breaks, T, es


def stale_knots(prob, U, grf_g, b, mu=0.7):
    """element b's control knots in stance phases whose stored GRF values are not those of its
    working control row U[kc] (GRFConstraint rows, HKDConstraints.cpp:15-22)"""
    hz = prob["horizons"]
    _, k0 = _phases(hz)
    out = []
    for i, n in enumerate(hz):
        c = prob["contacts"][b][i]
        for k in range(n):
            kc = k0[i] + k
            for l in range(4):
                if not c[l]:
                    continue
                f = U[b, kc, 3 * l:3 * l + 3]
                g = np.array([f[2], -f[0] + mu * f[2], f[0] + mu * f[2], -f[1] + mu * f[2], f[1] + mu * f[2]])
                if np.any(g != grf_g[b, kc, 5 * l:5 * l + 5]):
                    out.append(kc)
                    break
    return out


def direction_of(contacts, horizons):
    """direction() of one element from its contact rows and a layout"""
    return direction({"horizons": list(horizons), "S": sum(n + 1 for n in horizons), "contacts": [contacts]}, 0)


def translate_inputs(inp, horizons, T):
    """an MPC tick's inputs (mpc_scenario.Scenario.inputs) with element b translated by T[b]"""
    B = len(T)
    es = np.stack([direction_of(inp["contacts"][b], horizons) for b in range(B)])
    out = dict(inp)
    out["ref_x"] = inp["ref_x"] + T[:, None, None] * es
    rf = inp["ref_foot"].copy()
    rf[:, :, 0::3] += T[:, None, None]
    out["ref_foot"] = rf
    return out, es


def scenario_batch(B, P, N):
    """tests/test_gpu_mpc.py's receding-horizon batch: trot, pace, bound, pronk in turn"""
    from mpc_scenario import Scenario
    names = ["trot", "pace", "bound", "pronk"]
    sc = Scenario([names[b % 4] for b in range(B)], P, N)
    prob = syn.make_batch(B, P, N, "trot")
    inp = sc.inputs(prob["x0"])
    prob.update(inp)
    prob["Xbar"] = inp["ref_x"].copy()
    return sc, prob


def mpc_loop_oracle(B, P, N, T, ticks, ms=1, perturb=0.0):
    """The oracle side of an MPC loop (HKDMPCSolver::update, HKDMPC.cpp:96-165) with element b
    translated by T[b]: a full solve, then per tick one shift (mpc_oracle: warm start, working
    trajectory, constraint objects with their stored values), new inputs, a solve with max_AL_iter =
    2, max_DDP_iter = 1 that starts from the carried state.  Returns (prob, r0, [tick dicts with
    flags, inp (translated), layout, r])."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import mpc_oracle as M
    sc, prob = scenario_batch(B, P, N)
    hz = list(prob["horizons"])
    inp, es = translate_inputs(prob, hz, T)
    prob.update(inp)
    prob["Xbar"] = inp["ref_x"].copy()
    prob["x0"] = prob["x0"] + T[:, None] * es[:, 0, :]
    if perturb:
        prob["x0"] = prob["x0"] * (1 + perturb)
    r = O.solve_batch(prob, O.default_options(MS=ms), n_threads=8)
    r0 = r
    kw = dict(max_AL_iter=2, max_DDP_iter=1, MS=ms)
    op, _ = O.default_problem(hz, prob["dt"])
    shooting, reach = [n + 1 for n in hz], [0] * len(hz)
    out = []
    for _ in range(ticks):
        flags = sc.step(1)
        sh = [M.shift(hz, shooting, reach, r["Xbar"][b], r["X"][b], r["Ubar"][b], r["K"][b], flags) for b in range(B)]
        wk = [M.shift_working(hz, reach, r["X"][b], r["U"][b], r["Defect"][b], flags) for b in range(B)]
        cons = [M.shift_constraints(hz, reach, {k: r[k][b] for k in O.CONSTRAINT_FIELDS + ("grf_g", "td_h")}, flags,
                                    op.grf_delta, op.grf_eps, op.td_sigma, op.td_lambda) for b in range(B)]
        hz, shooting, reach = sh[0][0], sh[0][1], sh[0][2]
        inp, _ = translate_inputs(sc.inputs(np.stack([q[3][0] for q in sh])), hz, T)
        cons = [M.resolve_td(c, inp["contacts"][b]) for b, c in enumerate(cons)]
        state = {"X": np.stack([w[0] for w in wk]), "U": np.stack([w[1] for w in wk]),
                 "Defect": np.stack([w[2] for w in wk]), "grf_g": np.stack([c["grf_g"] for c in cons]),
                 "td_h": np.stack([c["td_h"] for c in cons])}
        p2 = {"batch": B, "horizons": hz, "shooting": shooting, "dt": prob["dt"], "S": sum(n + 1 for n in hz),
              "Kc": sum(hz), **inp, "Xbar": np.stack([q[3] for q in sh]), "Ubar": np.stack([q[4] for q in sh]),
              "K": np.stack([q[5] for q in sh])}
        r = O.solve_batch(p2, O.default_options(**kw), n_threads=8,
                          constraints={k: np.stack([c[k] for c in cons]) for k in O.CONSTRAINT_FIELDS}, state=state)
        out.append({"flags": flags, "inp": inp, "prob": p2, "r": r})
    return prob, r0, out
