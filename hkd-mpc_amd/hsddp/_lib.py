"""ctypes binding of the C-ABI in include/hsddp.h (libhsddp_amd.so, built in-tree).

The product path has no fallback: if the shared library is missing or no HIP device is present,
every entry point raises.  Import torch (if at all) before this module so the library binds to
the same HIP runtime instance torch loaded.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# HSDDP_LIB selects another in-tree build of the same ABI (kernel A/B measurements)
LIB_PATH = os.environ.get("HSDDP_LIB") or os.path.join(PKG_DIR, "libhsddp_amd.so")

DP = C.POINTER(C.c_double)
IP = C.POINTER(C.c_int)
MAX_PHASES = 16


class Options(C.Structure):
    """Mirror of hsddp_options / HSDDP_OPTION (HSDDP_CompoundTypes.h:18-60)."""
    _fields_ = [(n, C.c_double) for n in ("alpha", "gamma", "update_penalty", "update_relax",
                                          "update_regularization", "update_ReB")] + \
               [(n, C.c_int) for n in ("max_DDP_iter", "max_AL_iter", "max_DDP_iter_runtime",
                                       "max_AL_iter_runtime")] + \
               [(n, C.c_double) for n in ("cost_thresh", "tconstr_thresh", "pconstr_thresh",
                                          "dynamics_feas_thresh", "merit_rho", "merit_scale",
                                          "merit_offset")] + \
               [(n, C.c_int) for n in ("AL_active", "ReB_active", "smooth_active", "MS",
                                       "nsteps_per_node", "no_early_exit")]


class Weights(C.Structure):
    _fields_ = [("q_eul", C.c_double * 3), ("q_pos", C.c_double * 3), ("q_omega", C.c_double * 3),
                ("q_v", C.c_double * 3), ("q_qJ", C.c_double), ("qf_scale", C.c_double * 24),
                ("qf_gain", C.c_double), ("r_grf", C.c_double), ("r_qJd", C.c_double),
                ("foot_w", C.c_double * 3), ("foot_gain", C.c_double),
                ("foot_term_cost", C.c_double), ("foot_term_grad", C.c_double)]


class ConstraintParams(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("grf_delta", "grf_delta_min", "grf_eps", "swing_delta",
                                          "swing_delta_min", "swing_eps", "td_sigma", "td_sigma_max",
                                          "td_lambda", "mu_fric", "ground_height")]


class ProblemDesc(C.Structure):
    _fields_ = [("device", C.c_int), ("batch", C.c_int), ("n_phases", C.c_int),
                ("horizons", C.c_int * MAX_PHASES), ("dt", C.c_double), ("ref_per_element", C.c_int),
                ("weights", Weights), ("cparams", ConstraintParams), ("riccati_fp32", C.c_int)]


class ElementInfo(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("cost", "feas", "merit", "max_tconstr", "max_pconstr")] + \
               [(n, C.c_int) for n in ("iters", "outer_iters", "status", "n_ls_trials")]


class Stats(C.Structure):
    _fields_ = [("inner_iterations", C.c_int), ("outer_iterations", C.c_int), ("ls_trials", C.c_longlong),
                ("element_iterations", C.c_longlong), ("ms_total", C.c_double), ("ms_backward", C.c_double),
                ("ms_lq", C.c_double), ("ms_forward", C.c_double), ("ms_other", C.c_double),
                ("n_backward_launches", C.c_int), ("ms_linear", C.c_double)]


# hsddp_mpc_command (include/hsddp.h) = hkd_command_lcmt (lcmtypes/hkd_command_lcmt.lcm:1-11) as a
# C-aligned numpy record (tests/test_host_logic.py checks size and offsets against the C compiler)
MPC_COMMAND = np.dtype([("N_mpcsteps", np.int32), ("mpc_times", np.float64, (10,)),
                        ("hkd_controls", np.float32, (10, 24)), ("des_body_state", np.float32, (10, 12)),
                        ("contacts", np.int32, (10, 4)), ("statusTimes", np.float64, (10, 4)),
                        ("foot_placement", np.float32, (12,)), ("feedback", np.float32, (10, 12, 12)),
                        ("solve_time", np.float32)], align=True)


# hsddp_quad_state (QuadAugmentedState) and hsddp_phase_plan (include/hsddp.h) as C-aligned records
QUAD_STATE = np.dtype([("body_state", np.float64, (12,)), ("qJ", np.float64, (12,)), ("qJd", np.float64, (12,)),
                       ("foot_placements", np.float64, (12,)), ("grf", np.float64, (12,)),
                       ("torque", np.float64, (12,)), ("contact", np.int32, (4,)), ("status_dur", np.float64, (4,))],
                      align=True)
PHASE_PLAN = np.dtype([("n_phases", np.int32), ("horizons", np.int32, (16,)), ("contacts", np.int32, (17, 4)),
                       ("durations", np.float64, (16, 4)), ("start_times", np.float32, (16,)),
                       ("end_times", np.float32, (16,))], align=True)


class HSDDPError(RuntimeError):
    pass


_lib = None

# every symbol include/hsddp.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "hsddp_last_error", "hsddp_version", "hsddp_default_options", "hsddp_default_weights",
    "hsddp_default_constraint_params", "hsddp_load_settings", "hsddp_load_constraint_params",
    "hsddp_create", "hsddp_destroy", "hsddp_set_options", "hsddp_validate_options", "hsddp_upload_problem",
    "hsddp_upload_warm_start", "hsddp_solve", "hsddp_solve_begin", "hsddp_iterate", "hsddp_solve_end", "hsddp_download_trajectory", "hsddp_download_working",
    "hsddp_download_element_info", "hsddp_download_solver_info", "hsddp_download_lq",
    "hsddp_download_terminal", "hsddp_set_value_export", "hsddp_download_value", "hsddp_synchronize", "hsddp_device_bytes", "hsddp_hkd_dynamics",
    "hsddp_hkd_dynamics_partial", "hsddp_hkd_foot_position", "hsddp_hkd_foot_jacobian",
    "hsddp_hkd_resetmap", "hsddp_hkd_resetmap_partial", "hsddp_device_alloc", "hsddp_device_free",
    "hsddp_memcpy_h2d", "hsddp_memcpy_d2h", "hsddp_device_synchronize", "hsddp_extract_commands",
    "hsddp_shift", "hsddp_get_layout", "hsddp_update_problem", "hsddp_load_quad_reference",
    "hsddp_plan_phases", "hsddp_set_reference_table", "hsddp_build_references", "hsddp_download_references", "hsddp_advance",
    "hsddp_get_phase_info", "hsddp_hkd_running_cost", "hsddp_hkd_terminal_cost", "hsddp_hkd_grf_constraint",
    "hsddp_hkd_touchdown_constraint", "hsddp_set_element_layouts",
    "hsddp_shift_elements", "hsddp_get_element_layouts", "hsddp_extract_commands_device",
    "hsddp_set_layout", "hsddp_upload_constraint_params", "hsddp_download_constraint_params",
    "hsddp_download_constraint_values",
    "hsddp_extract_commands_async", "hsddp_commands_wait",
]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise HSDDPError(f"{LIB_PATH} not built: run __graft_entry__.build() (or make -C hkd-mpc_amd/csrc)")
    L = C.CDLL(LIB_PATH)
    L.hsddp_last_error.restype = C.c_char_p
    L.hsddp_version.restype = C.c_char_p
    L.hsddp_device_bytes.restype = C.c_size_t
    L.hsddp_device_bytes.argtypes = [C.c_void_p]
    L.hsddp_create.argtypes = [C.POINTER(ProblemDesc), C.POINTER(C.c_void_p)]
    L.hsddp_destroy.argtypes = [C.c_void_p]
    L.hsddp_set_options.argtypes = [C.c_void_p, C.POINTER(Options)]
    if hasattr(L, "hsddp_download_lq"):
        L.hsddp_download_lq.argtypes = [C.c_void_p] + [C.c_void_p] * 7
        L.hsddp_download_terminal.argtypes = [C.c_void_p] + [C.c_void_p] * 4
        L.hsddp_set_value_export.argtypes = [C.c_void_p, C.c_int]
        L.hsddp_download_value.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    if hasattr(L, "hsddp_download_solver_info"):
        L.hsddp_download_solver_info.argtypes = [C.c_void_p, C.c_int] + [C.c_void_p] * 5
    if hasattr(L, "hsddp_validate_options"):  # (older A/B builds lack it)
        L.hsddp_validate_options.argtypes = [C.POINTER(Options)]
    L.hsddp_upload_problem.argtypes = [C.c_void_p, IP, DP, DP, DP, DP]
    L.hsddp_upload_warm_start.argtypes = [C.c_void_p, DP, DP, DP]
    L.hsddp_solve.argtypes = [C.c_void_p, C.POINTER(Stats)]
    L.hsddp_solve_begin.argtypes = [C.c_void_p]
    L.hsddp_iterate.argtypes = [C.c_void_p, C.c_int, C.POINTER(Stats)]
    L.hsddp_solve_end.argtypes = [C.c_void_p]
    L.hsddp_download_trajectory.argtypes = [C.c_void_p, DP, DP, DP]
    L.hsddp_download_working.argtypes = [C.c_void_p, DP, DP, DP, DP, DP]
    L.hsddp_download_element_info.argtypes = [C.c_void_p, C.POINTER(ElementInfo)]
    L.hsddp_synchronize.argtypes = [C.c_void_p]
    L.hsddp_load_settings.argtypes = [C.c_char_p, C.POINTER(Options)]
    L.hsddp_load_constraint_params.argtypes = [C.c_char_p, C.POINTER(ConstraintParams)]
    for f in ("hsddp_hkd_dynamics",):
        getattr(L, f).argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_double, C.c_void_p, C.c_int, C.c_void_p]
    L.hsddp_hkd_dynamics_partial.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_double, C.c_void_p,
                                             C.c_void_p, C.c_int, C.c_void_p]
    L.hsddp_hkd_foot_position.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.hsddp_hkd_foot_jacobian.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.hsddp_hkd_resetmap.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    L.hsddp_hkd_resetmap_partial.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
    V = C.c_void_p
    L.hsddp_hkd_running_cost.argtypes = [V] * 6 + [C.POINTER(Weights), C.c_double, C.c_int] + [V] * 5 + [C.c_int, V]
    L.hsddp_hkd_terminal_cost.argtypes = [V] * 4 + [C.POINTER(Weights), C.c_int] + [V] * 3 + [C.c_int, V]
    L.hsddp_hkd_grf_constraint.argtypes = [V, V, C.c_double, V, V, C.c_int, V]
    L.hsddp_hkd_touchdown_constraint.argtypes = [V, V, V, C.c_double, V, V, C.c_int, V]
    L.hsddp_set_element_layouts.argtypes = [V, IP, IP]
    L.hsddp_shift_elements.argtypes = [V, C.c_int, IP]
    L.hsddp_get_element_layouts.argtypes = [V, IP, IP, IP, IP]
    L.hsddp_device_alloc.restype = C.c_void_p
    L.hsddp_device_alloc.argtypes = [C.c_size_t, C.c_int]
    L.hsddp_device_free.argtypes = [C.c_void_p]
    L.hsddp_memcpy_h2d.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.hsddp_memcpy_d2h.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.hsddp_device_synchronize.argtypes = [C.c_int]
    L.hsddp_shift.argtypes = [C.c_void_p, C.c_int, IP]
    L.hsddp_load_quad_reference.argtypes = [C.c_char_p, C.c_int, C.POINTER(C.c_float), C.c_void_p, C.c_int]
    L.hsddp_plan_phases.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_float, C.c_float, C.c_float, C.c_void_p]
    L.hsddp_set_reference_table.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_float]
    L.hsddp_build_references.argtypes = [C.c_void_p, IP, C.c_int, C.c_void_p, C.c_float]
    L.hsddp_download_references.argtypes = [C.c_void_p, DP, DP, DP]
    L.hsddp_advance.argtypes = [C.c_void_p, C.c_int, C.c_float, C.c_float, DP, IP]
    L.hsddp_get_phase_info.argtypes = [C.c_void_p, IP, DP]
    L.hsddp_get_layout.argtypes = [C.c_void_p, IP, IP, IP, IP]
    L.hsddp_update_problem.argtypes = [C.c_void_p, IP, DP, DP, DP, DP]
    L.hsddp_extract_commands.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double, C.c_void_p, C.c_int,
                                         C.c_void_p, C.c_int, C.c_float, C.c_void_p]
    L.hsddp_extract_commands_device.argtypes = L.hsddp_extract_commands.argtypes
    L.hsddp_set_layout.argtypes = [V, C.c_int, IP, IP, IP]
    L.hsddp_upload_constraint_params.argtypes = [V] * 6
    L.hsddp_download_constraint_params.argtypes = [V] * 6
    L.hsddp_download_constraint_values.argtypes = [V] * 3
    L.hsddp_extract_commands_async.argtypes = [V, C.c_int, C.c_double, C.c_double, V, C.c_int, V, C.c_int, C.c_float,
                                               C.POINTER(C.c_int)]
    L.hsddp_commands_wait.argtypes = [V, C.c_int, C.POINTER(C.c_void_p)]
    _lib = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        raise HSDDPError(f"hsddp error {rc}: {lib().hsddp_last_error().decode()}")


def dp(a: np.ndarray):
    if a.dtype != np.float64 or not a.flags.c_contiguous:
        raise TypeError("expected a C-contiguous float64 array")
    return a.ctypes.data_as(DP)


def ip(a: np.ndarray):
    if a.dtype != np.int32 or not a.flags.c_contiguous:
        raise TypeError("expected a C-contiguous int32 array")
    return a.ctypes.data_as(IP)
