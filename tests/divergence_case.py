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
