"""Independent dense numpy restatement of one HS-DDP backward sweep + linear rollout (test infra).

Follows the reference equations directly with numpy.linalg (no code shared with the oracle's C):
  LQ        SinglePhase::LQ_approximation  SinglePhase.cpp:264-296, HKD costs HKDCost.{h,cpp},
            GRF ReB ConstraintsBase.h:224-263, TD AL ConstraintsBase.h:386-399
  backward  SinglePhase::backward_sweep    SinglePhase.cpp:298-367; MultiPhaseDDP.cpp:190-229
  linear    SinglePhase::linear_rollout    SinglePhase.cpp:144-178; MultiPhaseDDP.cpp:20-50
Only the model (x+, A, B, FK, reset maps) comes from oracle_lib, itself pinned to the reference's
CasADi kernels by the golden vectors.
"""
import numpy as np

import oracle_lib as O

MU = 0.7
MASS_G = 8.912 * 9.81


def weights(c):
    q = np.array([1, 4, 5, 1, 1, 30, .2, .2, .2, 4, 1, .5] + [.2 * (1 - c[l]) for l in range(4) for _ in range(3)])
    sc = np.array([1, 1, 2, 1, 1, 20, .3, .3, .3, 1, 3, 1] + [.01] * 12)
    Qf = 20 * sc * q
    R = np.array([.2] * 12 + [.1] * 12)
    W = np.array([20 * w * c[l] for l in range(4) for w in (3, 1, 0)])
    D = np.zeros((12, 24))
    for l in range(4):
        D[3 * l:3 * l + 3, 3:6] = -c[l] * np.eye(3)
        D[3 * l:3 * l + 3, 12 + 3 * l:15 + 3 * l] = c[l] * np.eye(3)
    return np.diag(q), np.diag(Qf), np.diag(R), np.diag(W), D


def grf_A(c):
    rows = []
    for l in range(4):
        if c[l]:
            for r in ([0, 0, 1], [-1, 0, MU], [1, 0, MU], [0, -1, MU], [0, 1, MU]):
                a = np.zeros(24); a[3 * l:3 * l + 3] = r; rows.append(a)
    return np.array(rows).reshape(-1, 24)


def foot_height_grad(x, l):
    J = np.zeros(54)
    O.lib().orc_foot_jacobian(l, O.dp(np.ascontiguousarray(x[3:6])), O.dp(np.ascontiguousarray(x[0:3])),
                              O.dp(np.ascontiguousarray(x[12 + 3 * l:15 + 3 * l])), O.dp(J))
    J = J.reshape(3, 18)
    p = np.zeros(3)
    O.lib().orc_foot_position(l, O.dp(np.ascontiguousarray(x[3:6])), O.dp(np.ascontiguousarray(x[0:3])),
                              O.dp(np.ascontiguousarray(x[12 + 3 * l:15 + 3 * l])), O.dp(p))
    hx = np.zeros(24); hx[0:3] = J[2, 3:6]; hx[3:6] = J[2, 0:3]; hx[12:24] = J[2, 6:18]
    return p[2], hx


def sweep(prob, b, X, U, Defect, reg=0.0, delta=0.1, eps=0.1, sigma=50.0, lam=0.0):
    """One backward sweep + linear rollout at (X, U, Defect) for element b.  Returns dict."""
    hz = prob["horizons"]; dt = prob["dt"]; P = len(hz)
    cont = prob["contacts"][b]
    rb = 0 if prob["ref_x"].shape[0] == 1 else b
    xr_all, ur_all, pf_all = prob["ref_x"][rb], prob["ref_u"][rb], prob["ref_foot"][rb]
    s0 = np.cumsum([0] + [n + 1 for n in hz]); k0 = np.cumsum([0] + list(hz))
    lq = []
    for i in range(P):
        c = cont[i]; cn = cont[i + 1]
        Q, Qf, R, W, D = weights(c)
        Ag = grf_A(c)
        ks = []
        for k in range(hz[i]):
            s, kc = s0[i] + k, k0[i] + k
            x, u = X[s], U[kc]
            A, B = O.hkd_partial(x, u, dt, c.astype(float))
            dx = x - xr_all[s]; du = u - ur_all[s]
            d = (x[12:] - np.tile(x[3:6], 4)) - (pf_all[s] - np.tile(xr_all[s, 3:6], 4))
            lx = dt * Q @ dx + dt * D.T @ W @ d
            lu = dt * R @ du
            lxx = dt * Q + dt * D.T @ W @ D
            luu = dt * R.copy()
            if Ag.shape[0]:
                g = Ag @ u
                with np.errstate(divide="ignore"):
                    d1 = np.where(g > delta, -1.0 / g, (g - 2 * delta) / delta / delta)
                    d2 = np.where(g > delta, 1.0 / g ** 2, 1.0 / delta ** 2)
                lu = lu + dt * (eps * d1) @ Ag
                luu = luu + dt * (Ag.T * (eps * d2)) @ Ag
            ks.append((A, B, lx, lu, lxx, luu))
        s = s0[i] + hz[i]; x = X[s]
        dx = x - xr_all[s]
        d = (x[12:] - np.tile(x[3:6], 4)) - (pf_all[s] - np.tile(xr_all[s, 3:6], 4))
        Phix = Qf @ dx + 20 * D.T @ W @ d
        Phixx = Qf + 20 * D.T @ W @ D
        for l in range(4):
            if c[l] == 0 and cn[l] == 1:
                h, hx = foot_height_grad(x, l)
                Phix = Phix + (sigma * h + lam) * hx
                Phixx = Phixx + (sigma * (1 + h) + lam) * np.outer(hx, hx)
        Px = O.resetmap_partial(x, c, cn) if i < P - 1 else None
        lq.append((ks, Phix, Phixx, Px))
    K = [None] * k0[-1]; dU = [None] * k0[-1]
    G0 = H0 = None
    V0 = [None] * P  # (G[0], H[0]) per phase, SinglePhase.cpp:365
    for i in reversed(range(P)):
        ks, Phix, Phixx, _ = lq[i]
        if i == P - 1:
            G, H = Phix.copy(), Phixx.copy()
        else:
            Px = lq[i][3]
            G, H = Phix + Px.T @ G0, Phixx + Px.T @ H0 @ Px
        for k in reversed(range(hz[i])):
            A, B, lx, lu, lxx, luu = ks[k]
            Gn = G + H @ Defect[s0[i] + k + 1]
            Qx = lx + A.T @ Gn; Qu = lu + B.T @ Gn
            Qxx = lxx + A.T @ H @ A + reg * np.eye(24)
            Quu = luu + B.T @ H @ B + reg * np.eye(24)
            Qux = B.T @ H @ A
            Qi = np.linalg.inv(Quu); Qi = (Qi + Qi.T) / 2; Qxx = (Qxx + Qxx.T) / 2
            dU[k0[i] + k] = -Qi @ Qu
            K[k0[i] + k] = -Qi @ Qux
            G = Qx - Qux.T @ Qi @ Qu
            H = Qxx - Qux.T @ Qi @ Qux
        G0, H0 = G + H @ Defect[s0[i]], H
        V0[i] = (G0, H0)
    # linear rollout (eps = 1)
    dX = np.zeros_like(X); du_all = np.zeros_like(U)
    dV1 = dV2 = 0.0
    dx_init = np.zeros(24)
    for i in range(P):
        ks, Phix, Phixx, _ = lq[i]
        if i > 0:
            dx_init = lq[i - 1][3] @ dX[s0[i - 1] + hz[i - 1]]
        dX[s0[i]] = dx_init + Defect[s0[i]]
        for k in range(hz[i]):
            A, B, lx, lu, lxx, luu = ks[k]
            s, kc = s0[i] + k, k0[i] + k
            du = dU[kc] + K[kc] @ dX[s]
            du_all[kc] = du
            dX[s + 1] = A @ dX[s] + B @ du + Defect[s + 1]
            dV1 += lx @ dX[s] + lu @ du
            dV2 += dX[s] @ lxx @ dX[s] + du @ luu @ du
        xe = dX[s0[i] + hz[i]]
        dV1 += Phix @ xe; dV2 += xe @ Phixx @ xe
    return {"K": np.array(K), "dU": np.array(dU), "dX": dX, "du": du_all, "dV1": dV1, "dV2": dV2,
            "lq": lq, "G0": np.array([v[0] for v in V0]), "H0": np.array([v[1] for v in V0])}


def initial_rollout(prob, b):
    """hybrid_rollout(0) from the warm start: X = Xbar, U = Ubar, Defect = Xsim - X."""
    hz = prob["horizons"]; dt = prob["dt"]; P = len(hz)
    cont = prob["contacts"][b]
    X = prob["Xbar"][b].copy(); U = prob["Ubar"][b].copy()
    s0 = np.cumsum([0] + [n + 1 for n in hz]); k0 = np.cumsum([0] + list(hz))
    Dft = np.zeros_like(X)
    for i in range(P):
        xin = prob["x0"][b] if i == 0 else O.resetmap(X[s0[i] - 1], cont[i - 1], cont[i])
        Dft[s0[i]] = xin - X[s0[i]]
        for k in range(hz[i]):
            xs = O.hkd_step(X[s0[i] + k], U[k0[i] + k], dt, cont[i].astype(float))
            Dft[s0[i] + k + 1] = xs - X[s0[i] + k + 1]
    return X, U, Dft
