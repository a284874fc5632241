"""Synthetic HKD trajectory-optimisation batches.

This is the caller-side problem assembly the reference performs in
``HKDProblem::initialization`` (HKDMPC/HKD-TrajOpt/HKDProblem.cpp:15-111) and
``HKDSinglePhaseReference::get_reference_at_t`` (HKDReference.cpp:8-57), restated for a
batch of independent trajectories with closed-form gait references instead of CSV files:

* reference: constant forward trot at z = 0.25, v_x = 0.1, nominal feet at (±0.2, ±0.14, 0)
  translated with the body (Reference/Data/trot/quad_reference.csv:3-16);
  GRF_r = m g / n_stance on z (scripts/ReferenceGen/generate_reference.m:19-27);
  qJ_r = (0, -0.8, 1.6);
* x0[b] = nominal stance (HKDMPC.cpp:44-54: z = 0.2486, qJ = (0, -0.8, 1.6), stance qdummy =
  forward kinematics) + uniform perturbation (eul ±0.1, pos ±0.03, omega ±0.3, v ±0.3), drawn
  by splitmix64 seeded with 20240807 + b;
* Xbar = reference (HKDProblem.cpp:84-90), Ubar = 0, K = 0 (TrajectoryManagement.cpp:5-35; K is
  returned as None = zero).

Layout (element-major, fp64): contacts [B][P+1][4] (row P = contact after the horizon, which
defines the last phase's touchdown constraint, HKDProblem.cpp:268-310); ref_x/ref_u [Bref][S][24];
ref_foot [Bref][S][12]; S = sum(N_i + 1) state slots, Kc = sum(N_i) control slots.
"""
from __future__ import annotations

import math

import numpy as np

MASS = 8.912           # hkinodyn_casadi.cpp:559
GRAVITY = 9.81         # hkinodyn_casadi.cpp:575
DT = 0.01              # HKDMPC.cpp:28
NOMINAL_Z_REF = 0.25
NOMINAL_Z_X0 = 0.2486
VX_REF = 0.1
QJ_NOMINAL = (0.0, -0.8, 1.6)
FEET_NOMINAL = np.array([[0.2, -0.14, 0.0], [0.2, 0.14, 0.0], [-0.2, -0.14, 0.0], [-0.2, 0.14, 0.0]])
SEED = 20240807

# Gait cycles, legs FR, FL, HR, HL
GAITS = {
    "trot": [(1, 0, 0, 1), (0, 1, 1, 0)],
    "pace": [(1, 0, 1, 0), (0, 1, 0, 1)],
    "bound": [(1, 1, 0, 0), (0, 0, 1, 1)],
    "pronk": [(1, 1, 1, 1), (0, 0, 0, 0)],
    "jump": [(1, 1, 1, 1), (0, 0, 1, 1), (0, 0, 0, 0), (1, 1, 0, 0), (0, 0, 0, 0), (0, 0, 1, 1),
             (0, 0, 0, 0), (1, 1, 1, 1)],
}

_MASK64 = (1 << 64) - 1


def splitmix64(state: int):
    """splitmix64 stream: yields (new_state, value)."""
    state = (state + 0x9E3779B97F4A7C15) & _MASK64
    z = state
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK64
    return state, z ^ (z >> 31)


def uniform_stream(seed: int, n: int) -> np.ndarray:
    """n doubles uniform in [0, 1) from splitmix64 (53-bit mantissa)."""
    out = np.empty(n)
    s = seed & _MASK64
    for i in range(n):
        s, v = splitmix64(s)
        out[i] = (v >> 11) * (1.0 / (1 << 53))
    return out


def _rot_zyx(eul):
    cy, sy = math.cos(eul[0]), math.sin(eul[0])
    cp, sp = math.cos(eul[1]), math.sin(eul[1])
    cr, sr = math.cos(eul[2]), math.sin(eul[2])
    return np.array([[cy * cp, cy * sp * sr - sy * cr, sy * sr + cy * sp * cr],
                     [sy * cp, cy * cr + sy * sp * sr, sy * sp * cr - cy * sr],
                     [-sp, cp * sr, cp * cr]])


def foot_position(leg: int, pos, eul, q) -> np.ndarray:
    """Mini Cheetah forward kinematics (comp_foot_pos_casadi.cpp:46-160)."""
    side = (-1.0, 1.0, -1.0, 1.0)[leg]
    front = (1.0, 1.0, -1.0, -1.0)[leg]
    l_up, l_low, abad = -0.209, -0.195, 0.062
    c0, s0 = math.cos(q[0]), math.sin(q[0])
    c1, s1 = math.cos(q[1]), math.sin(q[1])
    c12, s12 = math.cos(q[1] + q[2]), math.sin(q[1] + q[2])
    pb = np.array([0.19 * front - l_low * s12 - l_up * s1,
                   0.049 * side + abad * side * c0 - l_low * s0 * c12 - l_up * s0 * c1,
                   l_low * c0 * c12 + l_up * c0 * c1 + abad * side * s0])
    return np.asarray(pos, dtype=float) + _rot_zyx(eul) @ pb


def phase_schedule(gait: str, n_phases: int, offset: int = 0):
    cyc = GAITS[gait]
    return [cyc[(offset + i) % len(cyc)] for i in range(n_phases + 1)]


def _reference_slots(contacts_ext, horizons, dt=DT, t0=0):
    """Per-slot reference (x_r, u_r, foot_r) following HKDReference.cpp:24-57.

    The terminal slot of phase i sits at the start time of phase i+1, so its qdummy reference
    uses the next phase's contact (the reference contact at that time).  t0: knot index of the
    first slot (the window start after receding-horizon shifts)."""
    P = len(horizons)
    S = sum(n + 1 for n in horizons)
    ref_x = np.zeros((S, 24))
    ref_u = np.zeros((S, 24))
    ref_f = np.zeros((S, 12))
    s = 0
    t_idx = t0
    for i in range(P):
        for k in range(horizons[i] + 1):
            t = (t_idx + k) * dt
            c = contacts_ext[i] if k < horizons[i] else contacts_ext[i + 1]
            px = VX_REF * t
            body = np.array([0, 0, 0, px, 0, NOMINAL_Z_REF, 0, 0, 0, VX_REF, 0, 0], dtype=float)
            feet = FEET_NOMINAL + np.array([px, 0, 0])
            ref_x[s, :12] = body
            for leg in range(4):
                ref_x[s, 12 + 3 * leg:15 + 3 * leg] = feet[leg] if c[leg] else QJ_NOMINAL
            nst = sum(c)
            for leg in range(4):
                if c[leg]:
                    ref_u[s, 3 * leg + 2] = MASS * GRAVITY / nst
            ref_f[s] = feet.reshape(-1)
            s += 1
        t_idx += horizons[i]
    return ref_x, ref_u, ref_f


def initial_state(b: int, contact0, seed: int = SEED) -> np.ndarray:
    r = uniform_stream(seed + b, 12) * 2.0 - 1.0
    eul = 0.1 * r[0:3]
    pos = np.array([0.0, 0.0, NOMINAL_Z_X0]) + 0.03 * r[3:6]
    om = 0.3 * r[6:9]
    v = 0.3 * r[9:12]
    x = np.zeros(24)
    x[0:3], x[3:6], x[6:9], x[9:12] = eul, pos, om, v
    for leg in range(4):
        if contact0[leg]:
            x[12 + 3 * leg:15 + 3 * leg] = foot_position(leg, pos, eul, QJ_NOMINAL)
        else:
            x[12 + 3 * leg:15 + 3 * leg] = QJ_NOMINAL
    return x


def make_batch(batch: int, n_phases: int = 4, knots: int = 50, gait: str = "trot",
               mixed: bool = False, seed: int = SEED, dt: float = DT, first_element: int = 0,
               jump_layout: bool = False) -> dict:
    """Build a synthetic batch.  mixed=True draws a per-element gait.

    Element b of this batch is global element first_element + b (seed SEED + global index), so
    shards of one global batch built on different ranks are disjoint and reproducible.
    With mixed=True and jump_layout, jump elements run C4's 8 x 25 layout (twice the phases, half
    the knots: the same Kc) beside the others' n_phases x knots — per-element layouts
    (hsddp_set_element_layouts); otherwise every element is on n_phases x knots (jump running the
    first n_phases phases of its cycle)."""
    if mixed and jump_layout and knots % 2 == 0 and 2 * n_phases <= 16:
        names = ["trot", "pace", "bound", "pronk", "jump"]
        pick = (uniform_stream(seed ^ 0x5A5A, first_element + batch)[first_element:] * len(names)).astype(int)
        gaits = [names[i] for i in pick]
        lays = [(g, 2 * n_phases, knots // 2) if g == "jump" else (g, n_phases, knots) for g in gaits]
        return make_layout_batch(lays, seed=seed, dt=dt, first_element=first_element)
    horizons = [knots] * n_phases
    S = sum(n + 1 for n in horizons)
    Kc = sum(horizons)
    if mixed:
        # every gait of SURVEY.md §8(d)'s C4 set; jump runs the first n_phases phases of its cycle
        # (for 4 phases: stance, rear stance, flight, front stance, then flight after the horizon)
        names = ["trot", "pace", "bound", "pronk", "jump"]
        pick = (uniform_stream(seed ^ 0x5A5A, first_element + batch)[first_element:] * len(names)).astype(int)
        gaits = [names[i] for i in pick]
    else:
        gaits = [gait] * batch
    uniq = sorted(set(gaits))
    refs = {g: _reference_slots(phase_schedule(g, n_phases), horizons, dt) for g in uniq}
    contacts = np.zeros((batch, n_phases + 1, 4), dtype=np.int32)
    x0 = np.zeros((batch, 24))
    if len(uniq) == 1:
        ref_x, ref_u, ref_f = (a[None] for a in refs[uniq[0]])
    else:
        ref_x = np.zeros((batch, S, 24)); ref_u = np.zeros((batch, S, 24)); ref_f = np.zeros((batch, S, 12))
    Xbar = np.zeros((batch, S, 24))
    for b in range(batch):
        sched = phase_schedule(gaits[b], n_phases)
        contacts[b] = np.array(sched, dtype=np.int32)
        x0[b] = initial_state(first_element + b, sched[0], seed)
        rx, ru, rf = refs[gaits[b]]
        if len(uniq) > 1:
            ref_x[b], ref_u[b], ref_f[b] = rx, ru, rf
        Xbar[b] = rx
    return {
        "batch": batch, "horizons": horizons, "dt": dt, "S": S, "Kc": Kc, "gaits": gaits,
        "contacts": contacts, "x0": x0, "ref_x": np.ascontiguousarray(ref_x),
        "ref_u": np.ascontiguousarray(ref_u), "ref_foot": np.ascontiguousarray(ref_f),
        "Xbar": Xbar, "Ubar": np.zeros((batch, Kc, 24)),
        "K": None,  # feedback gains default to zero on the device (3.8 GB as a host array at B=4096)
    }


def make_layout_batch(layouts, seed: int = SEED, dt: float = DT, first_element: int = 0) -> dict:
    """A batch whose elements have their own phase layouts: layouts[b] = (gait, n_phases, knots).
    Every element's n_phases * knots must be equal (the handle's Kc).  Arrays use the largest
    layout as the stride (include/hsddp.h, hsddp_set_element_layouts): contacts [B][Pmax+1][4]
    (element b: rows 0 .. P_b), state-slot arrays [B][Smax][..] (element b: its first S_b rows)."""
    batch = len(layouts)
    hz = [[n] * p for _, p, n in layouts]
    Kc = sum(hz[0])
    if any(sum(h) != Kc for h in hz):
        raise ValueError("every element's horizons must sum to the same Kc")
    Pmax = max(len(h) for h in hz)
    Smax = max(sum(n + 1 for n in h) for h in hz)
    contacts = np.zeros((batch, Pmax + 1, 4), dtype=np.int32)
    x0 = np.zeros((batch, 24))
    ref_x = np.zeros((batch, Smax, 24)); ref_u = np.zeros((batch, Smax, 24)); ref_f = np.zeros((batch, Smax, 12))
    refs = {}
    for b, (g, P, n) in enumerate(layouts):
        sched = phase_schedule(g, P)
        contacts[b, :P + 1] = np.array(sched, dtype=np.int32)
        x0[b] = initial_state(first_element + b, sched[0], seed)
        if (g, P, n) not in refs:
            refs[(g, P, n)] = _reference_slots(sched, [n] * P, dt)
        rx, ru, rf = refs[(g, P, n)]
        S_b = rx.shape[0]
        ref_x[b, :S_b], ref_u[b, :S_b], ref_f[b, :S_b] = rx, ru, rf
    return {
        "batch": batch, "horizons": hz[0], "layouts": hz, "dt": dt, "S": Smax, "P": Pmax, "Kc": Kc,
        "gaits": [g for g, _, _ in layouts], "contacts": contacts, "x0": x0, "ref_x": ref_x, "ref_u": ref_u,
        "ref_foot": ref_f, "Xbar": ref_x.copy(), "Ubar": np.zeros((batch, Kc, 24)), "K": None,
    }


def layout_groups(prob: dict) -> dict:
    """Elements of a per-element-layout batch grouped by layout: {tuple(horizons): [b, ...]}."""
    out = {}
    for b, h in enumerate(prob.get("layouts") or [prob["horizons"]] * prob["batch"]):
        out.setdefault(tuple(h), []).append(b)
    return out


def sub_batch(prob: dict, elements, horizons) -> dict:
    """The elements (all of one layout `horizons`) of a per-element-layout batch as an ordinary
    batch of that layout (rows past its S and P dropped)."""
    idx = list(elements)
    P = len(horizons)
    S = sum(n + 1 for n in horizons)
    out = {"batch": len(idx), "horizons": list(horizons), "dt": prob["dt"], "S": S, "Kc": prob["Kc"],
           "contacts": np.ascontiguousarray(prob["contacts"][idx, :P + 1]),
           "x0": np.ascontiguousarray(prob["x0"][idx])}
    for k in ("ref_x", "ref_u", "ref_foot", "Xbar"):
        out[k] = np.ascontiguousarray(prob[k][idx, :S])
    out["Ubar"] = np.ascontiguousarray(prob["Ubar"][idx])
    out["K"] = None
    return out
