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
