"""mpc_oracle.py — TEST INFRASTRUCTURE ONLY.

CPU restatement (plain Python / numpy, one element at a time) of the MPC caller's steps around the
solve in heli-sudoo/HKD-MPC, used by tests/ to check the HIP product path:

  * command extraction — HKDMPCSolver::update_foot_placement / publish_mpc_cmd
    (HKDMPC/HKDMPC.cpp:207-298) into the hkd_command_lcmt fields (lcmtypes/hkd_command_lcmt.lcm).

Layouts follow the product's C-ABI (include/hsddp.h): per element, Xbar [S][24] over state slots
(phase i owns N_i + 1), Ubar [Kc][24] and K [Kc][24][24] over control slots (N_i per phase),
contacts [P+1][4].  The product path never imports this module.
"""
import numpy as np


def phase_offsets(horizons):
    """state / control slot offsets of every phase"""
    s0, k0, s, k = [], [], 0, 0
    for n in horizons:
        s0.append(s); k0.append(k)
        s += n + 1; k += n
    return s0, k0


def foot_placement(Xbar, contacts, horizons, pf_current):
    """HKDMPCSolver::update_foot_placement (HKDMPC.cpp:207-230), one element."""
    s0, _ = phase_offsets(horizons)
    pf = [np.array(pf_current[3 * l:3 * l + 3], dtype=np.float32) for l in range(4)]
    found = [0, 0, 0, 0]
    n_phases = len(horizons)
    for i in range(n_phases - 1):
        ct, ctn = contacts[i], contacts[i + 1]
        for l in range(4):
            if not found[l] and ct[l] == 0 and ctn[l] == 1:
                qd = Xbar[s0[i + 1]][12:24]           # trajectory_ptrs[i + 1]->Xbar[0].tail(12)
                pf[l] = qd[3 * l:3 * l + 3].astype(np.float32)
                found[l] = 1
        if i >= 4:
            break
    return np.concatenate(pf)


def mpc_command(Xbar, Ubar, K, contacts, horizons, nsteps_between_mpc, mpc_time, dt_mpc, durations,
                pf_current, solve_time):
    """HKDMPCSolver::publish_mpc_cmd (HKDMPC.cpp:232-298) after update_foot_placement, one element.
    Returns a dict of the hkd_command_lcmt fields (rows past N_mpcsteps zero)."""
    s0, k0 = phase_offsets(horizons)
    n = nsteps_between_mpc + 7
    cmd = {"N_mpcsteps": n, "mpc_times": np.zeros(10), "hkd_controls": np.zeros((10, 24), np.float32),
           "des_body_state": np.zeros((10, 12), np.float32), "contacts": np.zeros((10, 4), np.int32),
           "statusTimes": np.zeros((10, 4)), "feedback": np.zeros((10, 12, 12), np.float32)}
    k = s = i = 0
    while k < n:
        if s >= horizons[i]:
            s = 0
            i += 1
        cmd["hkd_controls"][k] = Ubar[k0[i] + s].astype(np.float32)
        cmd["des_body_state"][k] = Xbar[s0[i] + s][:12].astype(np.float32)
        cmd["feedback"][k] = K[k0[i] + s][:12, :12].astype(np.float32)
        cmd["mpc_times"][k] = mpc_time + k * dt_mpc
        cmd["contacts"][k] = contacts[i]
        cmd["statusTimes"][k] = durations[i]
        s += 1
        k += 1
    cmd["foot_placement"] = foot_placement(Xbar, contacts, horizons, pf_current)
    cmd["solve_time"] = np.float32(solve_time)
    return cmd


# ---- receding-horizon update ------------------------------------------------------------------
def split_phases(arr, horizons, states):
    """[S][..] (states) or [Kc][..] (controls) -> per-phase lists of rows"""
    out, o = [], 0
    for n in horizons:
        m = n + 1 if states else n
        out.append([np.array(arr[o + j], copy=True) for j in range(m)])
        o += m
    return out


def shift(horizons, shooting, reach_end, Xbar, X, Ubar, K, contact_change):
    """HKDProblem::update (HKDProblem.cpp:117-222) on one element's warm start, as deques of phases.

    Per step: front — pop_front_phase (HKDProblem.h:56-66) when the first phase's end time is not
    after the new start (one knot left), else SinglePhase::pop_front (SinglePhase.cpp:496-501:
    Trajectory::pop_front drops X/Xbar/U/Ubar/K fronts, TrajectoryManagement.cpp:118-148); back — a
    new phase (Trajectory::create_data: zeros, TrajectoryManagement.cpp:4-35; initialization()
    clears SS_set) when the contact changes and is_phase_reach_end.back(), else push_back_default
    (Trajectory::push_back_state(X.back()), TrajectoryManagement.cpp:178-208), marking
    is_phase_reach_end on a change.  Then update_SS_config for all phases but a last one of horizon
    <= 2 and Ubar[0] of the first phase zeroed.  Returns (horizons, shooting, reach_end, Xbar,
    Ubar, K) in the flat slot layout."""
    hz, ss, re = list(horizons), list(shooting), list(reach_end)
    xb, xw = split_phases(Xbar, hz, True), split_phases(X, hz, True)
    ub, kk = split_phases(Ubar, hz, False), split_phases(K, hz, False)
    for cc in contact_change:
        if hz[0] <= 1:                      # approx_leq(phase_end_times.front(), new_start_time)
            for L in (hz, ss, re, xb, xw, ub, kk):
                L.pop(0)
        else:
            for L in (xb[0], xw[0], ub[0], kk[0]):
                L.pop(0)
            hz[0] -= 1
        if cc and re[-1]:
            hz.append(1); ss.append(0); re.append(0)
            xb.append([np.zeros_like(Xbar[0]) for _ in range(2)])
            xw.append([np.zeros_like(Xbar[0]) for _ in range(2)])
            ub.append([np.zeros_like(Ubar[0])])
            kk.append([np.zeros_like(K[0])])
        else:
            last = np.array(xw[-1][-1], copy=True)   # X.back()
            xb[-1].append(last); xw[-1].append(np.array(last, copy=True))
            ub[-1].append(np.zeros_like(Ubar[0])); kk[-1].append(np.zeros_like(K[0]))
            hz[-1] += 1
            if cc:
                re[-1] = 1
    P = len(hz)
    for i in range(P):
        if i < P - 1 or hz[i] > 2:
            ss[i] = hz[i] + 1
    ub[0][0] = np.zeros_like(ub[0][0])
    flat = lambda L: np.array([r for ph in L for r in ph])
    return hz, ss, re, flat(xb), flat(ub), flat(kk)


def shift_working(horizons, reach_end, X, U, Defect, contact_change):
    """The same update on one element's working trajectory, which the reference keeps from tick to
    tick beside the nominal one (a solve whose last line search failed leaves X, U != Xbar, Ubar,
    quirk A2; a later initial rollout that breaks keeps them past the break): Trajectory::pop_front
    drops the front rows of X, U and Defect (TrajectoryManagement.cpp:118-145), push_back_state
    appends X.back() to X, a zero U row and a zero Defect row (:179-207), a new phase starts from
    zeros (Trajectory::create_data).  Returns (X, U, Defect) in the flat slot layout."""
    hz, re = list(horizons), list(reach_end)
    xw, dw, uw = split_phases(X, hz, True), split_phases(Defect, hz, True), split_phases(U, hz, False)
    for cc in contact_change:
        if hz[0] <= 1:
            for L in (hz, re, xw, dw, uw):
                L.pop(0)
        else:
            for L in (xw[0], dw[0], uw[0]):
                L.pop(0)
            hz[0] -= 1
        if cc and re[-1]:
            hz.append(1); re.append(0)
            xw.append([np.zeros_like(X[0]) for _ in range(2)])
            dw.append([np.zeros_like(X[0]) for _ in range(2)])
            uw.append([np.zeros_like(U[0])])
        else:
            xw[-1].append(np.array(xw[-1][-1], copy=True))
            dw[-1].append(np.zeros_like(X[0]))
            uw[-1].append(np.zeros_like(U[0]))
            hz[-1] += 1
            if cc:
                re[-1] = 1
    flat = lambda L: np.array([r for ph in L for r in ph])  # noqa: E731
    return flat(xw), flat(uw), flat(dw)


# ---- the constraint objects through the receding-horizon update --------------------------------
MAX_TD = 4          # touchdown constraints per phase (HSDDP_MAX_TD)
TD_PENDING = 0x10   # a constraint registered by the update whose legs come from the next contact rows


def td_bits(c, cn):
    """legs with contact 0 -> 1 (add_tconstr_one_phase's touchdown_status, HKDProblem.cpp:270-276)"""
    return sum(1 << l for l in range(4) if c[l] == 0 and cn[l] == 1)


def shift_constraints(horizons, reach_end, cons, contact_change, grf_delta, grf_eps, td_sigma, td_lambda,
                      cap=False):
    """HKDProblem::update (HKDProblem.cpp:117-222) on one element's constraint objects, which live on
    in the phases across MPC ticks (HKDProblem::update's reset_params is a no-op, ConstraintsBase.h:
    165-167, 341-348).  cons: reb_delta, reb_eps [Kc][20]; td_mask [P][MAX_TD]; al_sigma, al_lambda
    [P][MAX_TD][4].  Per step: the front knot's ReB row leaves with it (PathConstraintBase::pop_front)
    or the whole first phase is dropped; a pushed-back knot copies the last knot's ReB row
    (PathConstraintBase::push_back, ConstraintsBase.h:147-158); a new phase's GRF constraint starts
    from the initial ReB parameters and carries no touchdown constraint; at every step whose last
    phase has reached its end, add_tconstr_one_phase appends one more touchdown constraint with the
    initial AL parameters (HKDProblem.cpp:199-202) — its legs follow from the next contact rows
    (TD_PENDING, resolve_td).  With "grf_g" / "td_h" in cons, the constraint objects' stored values
    follow too (zero for pushed knots, new phases and new constraints: create_data,
    PathConstraintBase::push_back).  Returns the new cons.  cap: a phase holds at most MAX_TD constraints
    and the later ones are not registered (the device's HSDDP_MAX_TD; "overflow" in the result says
    whether one was dropped) — the reference's lists are unbounded, so without cap that is an error."""
    hz, re = list(horizons), list(reach_end)
    rd = split_phases(cons["reb_delta"], hz, False)
    rs = split_phases(cons["reb_eps"], hz, False)
    # the stored constraint values (optional): GRF g per knot [Kc][20], touchdown h per constraint [P][MAX_TD][4]
    vals = "grf_g" in cons
    gg = split_phases(cons["grf_g"], hz, False) if vals else [[] for _ in hz]
    th = cons["td_h"] if vals else np.zeros((len(hz), MAX_TD, 4))
    td = [list(zip([int(m) for m in cons["td_mask"][i]], [np.array(v) for v in cons["al_sigma"][i]],
                   [np.array(v) for v in cons["al_lambda"][i]], [np.array(v) for v in th[i]])) for i in range(len(hz))]
    init_row = lambda v: np.full(20, v)  # noqa: E731
    overflow = False
    for cc in contact_change:
        if hz[0] <= 1:
            for L in (hz, re, rd, rs, gg, td):
                L.pop(0)
        else:
            rd[0].pop(0); rs[0].pop(0)
            if vals:
                gg[0].pop(0)
            hz[0] -= 1
        if cc and re[-1]:
            hz.append(1); re.append(0)
            rd.append([init_row(grf_delta)]); rs.append([init_row(grf_eps)]); gg.append([np.zeros(20)])
            td.append([(0, np.full(4, td_sigma), np.full(4, td_lambda), np.zeros(4)) for _ in range(MAX_TD)])
        else:
            # PathConstraintBase::push_back: a zero data row, the last knot's ReB parameters
            rd[-1].append(np.array(rd[-1][-1])); rs[-1].append(np.array(rs[-1][-1])); gg[-1].append(np.zeros(20))
            hz[-1] += 1
            if cc:
                re[-1] = 1
        if re[-1]:  # one more touchdown constraint on the last phase, in its first free slot
            slots = td[-1]
            j = next((q for q, s in enumerate(slots) if s[0] == 0), None)
            if j is None and cap:
                overflow = True
                continue
            assert j is not None, "more than MAX_TD touchdown constraints on one phase"
            slots[j] = (TD_PENDING, np.full(4, td_sigma), np.full(4, td_lambda), np.zeros(4))
    flat = lambda L: np.array([r for ph in L for r in ph])  # noqa: E731
    out = {"reb_delta": flat(rd), "reb_eps": flat(rs),
           "td_mask": np.array([[s[0] for s in ph] for ph in td], np.int32),
           "al_sigma": np.array([[s[1] for s in ph] for ph in td]),
           "al_lambda": np.array([[s[2] for s in ph] for ph in td]), "overflow": overflow}
    if vals:
        out["grf_g"] = flat(gg)
        out["td_h"] = np.array([[s[3] for s in ph] for ph in td])
    return out


def resolve_td(cons, contacts):
    """TD_PENDING constraints take the touchdown legs of their phase's contact rows (i -> i + 1)"""
    out = dict(cons)
    m = np.array(cons["td_mask"], copy=True)
    for i in range(m.shape[0]):
        for j in range(m.shape[1]):
            if m[i, j] == TD_PENDING:
                m[i, j] = td_bits(contacts[i], contacts[i + 1])
    out["td_mask"] = m
    return out
