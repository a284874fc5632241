// hsddp_mpc.h — kernel interface of the MPC-side steps around the solve (hsddp_mpc.hip).
#pragma once

#include "hsddp_internal.h"

struct hsddp_mpc_command;

namespace hsddp {

// publish_mpc_cmd's knot walk resolved on the host (horizons are shared by the batch)
struct CmdArgs {
    int n;                         // N_mpcsteps
    int kc[10], xs[10], ph[10];    // control slot, state slot and phase of command row k
    double mpc_time, dt_mpc;
    const double *durations;       // [Bd][P][4] device, or null
    int dur_per_elem;
    const float *feet;             // [Bf][12] device, or null
    int feet_per_elem;
    float solve_time;
};

// receding-horizon gather: new slot <- old slot (labels as hsddp_api.cpp ShiftPhase)
struct ShiftArgs {
    int S_old, S_new, Kc;
    const int *smap, *cmap;   // [n_maps][S_new], [n_maps][Kc] device
    const int *map_id;        // [B] map of each element (null: one map for the batch)
    int fp32, zero_u0;
    // [3][B][S_old][24] staging (the state rows' element stride changes, S_new != S_old): the
    // nominal X, working X and working Defect rows are copied here first, and the gathers read them
    // from here — written in place at the new stride, element b's rows would overlap the old rows
    // of its neighbours in a buffer another element still reads (every element picks its own
    // buffers); null: the strides agree and every element's rows stay inside its own region
    double *stage;
};
// the new Xbar / Ubar rows into every element's third buffer, which becomes its nominal one; the
// working rows (X, U, Defect) follow into the same buffer when they are the nominal ones, else into
// the old nominal buffer (read by then), which becomes the working one; the new compact K rows into K_new
void launch_shift_gather(int B, const ShiftArgs &a, const Bufs &d, void *K_new, hipStream_t st);
// constraint objects through the shift: ReB rows by control-slot source (rmap: old slot, -1 =
// initial), the stored GRF values' table by control-slot source (cmap: old slot, -1 = a new knot,
// whose zero values are its zero working row's), touchdown constraints by phase source (pmap: old
// phase, -1 = new) plus nadd appended pending ones per new phase (zero residual: TD_STALE);
// overflow counts phases past MTD constraints
struct ShiftParamArgs {
    int Kc, P_old, P_new;
    const int *rmap, *cmap;   // [n_maps][Kc]
    const int *pmap, *nadd;   // [n_maps][MAXP]
    const int *map_id;        // [B] (null: one map)
    double reb_delta0, reb_eps0, td_sigma0, td_lambda0;
    int *overflow;
};
struct ShiftParamOut {
    double *reb_delta, *reb_eps, *al_sigma, *al_lambda, *cf_u;
    int *td_mask, *cf_flag;
};
void launch_shift_params(int B, const ShiftParamArgs &a, const Bufs &d, const ShiftParamOut &o, hipStream_t st);

// reference sample table on the device: [n][RT_W] doubles per sample
constexpr int RT_BODY = 0, RT_QJ = 12, RT_QJD = 24, RT_FOOT = 36, RT_GRF = 48, RT_C = 60, RT_W = 64;
struct RefArgs {
    const double *table;   // [n][RT_W]
    int n;
    const int *start;      // [Bw] window start sample per element (Bw = Bref)
    const int *slot_idx;   // [n_maps][S] sample offset of each state slot within the window
    const int *map_id;     // [B] slot map of each element (per-element layouts), or null: map 0
};
void launch_build_refs(const Params &p, const Bufs &d, int Bref, const RefArgs &a, hipStream_t st);

void launch_extract_commands(const Params &p, const Bufs &d, const CmdArgs &a, hsddp_mpc_command *out,
                             hipStream_t st);

}  // namespace hsddp
