// hsddp_api.cpp — C-ABI of the batched HS-DDP solver (include/hsddp.h): handle, device memory,
// the per-element-masked solve loop (MultiPhaseDDP::solve, MultiPhaseDDP.cpp:232-428) and the
// INFO-file loaders (loadHSDDPSetting, HSDDP_CompoundTypes.h:62-87; loadConstrintParameters,
// HKDProblem.h:70-90).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/hsddp.h"
#include "hsddp_internal.h"
#include "hsddp_mpc.h"

using namespace hsddp;

static thread_local std::string g_err;

static int fail(int code, const std::string &msg)
{
    g_err = msg;
    return code;
}

extern "C" int hsddp_ref_fail(int code, const char *msg) { return fail(code, msg); }

#define HIPCHK(expr)                                                                                 \
    do {                                                                                             \
        hipError_t e_ = (expr);                                                                      \
        if (e_ != hipSuccess) return fail(HSDDP_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

extern "C" const char *hsddp_last_error(void) { return g_err.c_str(); }
extern "C" const char *hsddp_version(void) { return "hsddp-mi355x 0.1 (gfx950, fp64)"; }

// ---- options / parameters ----------------------------------------------------------------
extern "C" void hsddp_default_options(hsddp_options *o)
{
    // HSDDP_OPTION in-class defaults (HSDDP_CompoundTypes.h:20-45)
    o->alpha = 0.1; o->gamma = 0.1; o->update_penalty = 8; o->update_relax = 0.1;
    o->update_regularization = 2; o->update_ReB = 7;
    o->max_DDP_iter = 3; o->max_AL_iter = 2; o->max_DDP_iter_runtime = 1; o->max_AL_iter_runtime = 2;
    o->cost_thresh = 1e-3; o->tconstr_thresh = 1e-3; o->pconstr_thresh = 1e-3; o->dynamics_feas_thresh = 1e-3;
    o->merit_rho = 1e4; o->merit_scale = 0.2; o->merit_offset = 10;
    o->AL_active = 1; o->ReB_active = 1; o->smooth_active = 0; o->MS = 1; o->nsteps_per_node = 1;
    o->no_early_exit = 0;
}

extern "C" void hsddp_default_weights(hsddp_hkd_weights *w)
{
    const double qe[3] = {1, 4, 5}, qp[3] = {1, 1, 30}, qo[3] = {.2, .2, .2}, qv[3] = {4, 1, .5};
    const double sc[24] = {1, 1, 2, 1, 1, 20, .3, .3, .3, 1, 3, 1, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01};
    for (int i = 0; i < 3; ++i) { w->q_eul[i] = qe[i]; w->q_pos[i] = qp[i]; w->q_omega[i] = qo[i]; w->q_v[i] = qv[i]; }
    w->q_qJ = 0.2;
    for (int i = 0; i < 24; ++i) w->qf_scale[i] = sc[i];
    w->qf_gain = 20; w->r_grf = 0.2; w->r_qJd = 0.1;
    w->foot_w[0] = 3; w->foot_w[1] = 1; w->foot_w[2] = 0; w->foot_gain = 20;
    w->foot_term_cost = 10; w->foot_term_grad = 20;
}

extern "C" void hsddp_default_constraint_params(hsddp_constraint_params *cp)
{
    // settings/constraint_params.info values; mu = 0.7 (HKDConstraints.h:17); ground height 0
    cp->grf_delta = 0.1; cp->grf_delta_min = 0.1; cp->grf_eps = 0.1;
    cp->swing_delta = 1.0; cp->swing_delta_min = 0.5; cp->swing_eps = 0.01;
    cp->td_sigma = 50; cp->td_sigma_max = 1e4; cp->td_lambda = 0;
    cp->mu_fric = 0.7; cp->ground_height = 0.0;
}

// Minimal Boost.PropertyTree INFO reader: `key value` pairs, `key { ... }` children, ';' comments,
// optional double quotes.  Produces dotted paths ("ddp.alpha").
static int parse_info(const char *path, std::map<std::string, std::string> &out)
{
    std::ifstream f(path);
    if (!f) return fail(HSDDP_ERR_IO, std::string("cannot open ") + path);
    std::vector<std::string> stack;
    std::string line, last_key;
    while (std::getline(f, line)) {
        // strip comment (outside quotes)
        bool q = false;
        for (size_t i = 0; i < line.size(); ++i) {
            if (line[i] == '"') q = !q;
            if (line[i] == ';' && !q) { line.resize(i); break; }
        }
        std::vector<std::string> tok;
        std::string cur;
        q = false;
        for (char ch : line) {
            if (ch == '"') { q = !q; continue; }
            if (!q && (std::isspace((unsigned char)ch) || ch == '{' || ch == '}')) {
                if (!cur.empty()) { tok.push_back(cur); cur.clear(); }
                if (ch == '{' || ch == '}') tok.push_back(std::string(1, ch));
                continue;
            }
            cur += ch;
        }
        if (!cur.empty()) tok.push_back(cur);
        size_t i = 0;
        while (i < tok.size()) {
            if (tok[i] == "{") {
                stack.push_back(last_key);
                ++i;
                continue;
            }
            if (tok[i] == "}") {
                if (stack.empty()) return fail(HSDDP_ERR_IO, std::string("unbalanced '}' in ") + path);
                stack.pop_back();
                ++i;
                continue;
            }
            std::string key = tok[i++];
            std::string val;
            if (i < tok.size() && tok[i] != "{" && tok[i] != "}") val = tok[i++];
            std::string full;
            for (auto &s : stack) full += s + ".";
            full += key;
            out[full] = val;
            last_key = key;
        }
    }
    if (!stack.empty()) return fail(HSDDP_ERR_IO, std::string("unbalanced '{' in ") + path);
    return HSDDP_OK;
}

static int get_num(const std::map<std::string, std::string> &m, const std::string &k, double &v)
{
    auto it = m.find(k);
    if (it == m.end()) return fail(HSDDP_ERR_IO, "No such node (" + k + ")"); // ptree_bad_path
    char *end = nullptr;
    v = std::strtod(it->second.c_str(), &end);
    if (end == it->second.c_str() || *end) return fail(HSDDP_ERR_IO, "conversion of data failed (" + k + ")");
    return HSDDP_OK;
}
static int get_int(const std::map<std::string, std::string> &m, const std::string &k, int &v)
{
    auto it = m.find(k);
    if (it == m.end()) return fail(HSDDP_ERR_IO, "No such node (" + k + ")");
    char *end = nullptr;
    long x = std::strtol(it->second.c_str(), &end, 10);
    if (end == it->second.c_str() || *end) return fail(HSDDP_ERR_IO, "conversion of data failed (" + k + ")");
    v = (int)x;
    return HSDDP_OK;
}
static int get_bool(const std::map<std::string, std::string> &m, const std::string &k, int &v)
{
    auto it = m.find(k);
    if (it == m.end()) return fail(HSDDP_ERR_IO, "No such node (" + k + ")");
    const std::string &s = it->second;
    if (s == "true" || s == "1") v = 1;
    else if (s == "false" || s == "0") v = 0;
    else return fail(HSDDP_ERR_IO, "conversion of data failed (" + k + ")");
    return HSDDP_OK;
}

extern "C" int hsddp_load_settings(const char *path, hsddp_options *o)
{
    if (!path || !o) return fail(HSDDP_ERR_ARG, "null argument");
    std::map<std::string, std::string> m;
    int rc = parse_info(path, m);
    if (rc) return rc;
    hsddp_options t = *o;
    // exactly the keys loadHSDDPSetting reads (HSDDP_CompoundTypes.h:70-86); update_regularization and
    // smooth_active are not read, so they keep the caller's values (quirk A1).
#define N_(k) if ((rc = get_num(m, "ddp." #k, t.k))) return rc
#define I_(k) if ((rc = get_int(m, "ddp." #k, t.k))) return rc
#define B_(k) if ((rc = get_bool(m, "ddp." #k, t.k))) return rc
    N_(alpha); N_(gamma); N_(update_penalty); N_(update_relax); N_(update_ReB);
    I_(max_DDP_iter); I_(max_AL_iter); I_(max_DDP_iter_runtime); I_(max_AL_iter_runtime);
    N_(cost_thresh); N_(tconstr_thresh); N_(pconstr_thresh); N_(dynamics_feas_thresh);
    N_(merit_rho); N_(merit_scale); N_(merit_offset);
    B_(AL_active); B_(ReB_active); B_(MS); I_(nsteps_per_node);
#undef N_
#undef I_
#undef B_
    *o = t;
    return HSDDP_OK;
}

extern "C" int hsddp_load_constraint_params(const char *path, hsddp_constraint_params *cp)
{
    if (!path || !cp) return fail(HSDDP_ERR_ARG, "null argument");
    std::map<std::string, std::string> m;
    int rc = parse_info(path, m);
    if (rc) return rc;
    hsddp_constraint_params t = *cp;
    if ((rc = get_num(m, "GRF_ReB.delta", t.grf_delta)) || (rc = get_num(m, "GRF_ReB.delta_min", t.grf_delta_min)) ||
        (rc = get_num(m, "GRF_ReB.eps", t.grf_eps)) || (rc = get_num(m, "Swing_ReB.delta", t.swing_delta)) ||
        (rc = get_num(m, "Swing_ReB.delta_min", t.swing_delta_min)) || (rc = get_num(m, "Swing_ReB.eps", t.swing_eps)) ||
        (rc = get_num(m, "TD_AL.sigma", t.td_sigma)) || (rc = get_num(m, "TD_AL.lambda", t.td_lambda)) ||
        (rc = get_num(m, "TD_AL.sigma_max", t.td_sigma_max)))
        return rc;
    *cp = t;
    return HSDDP_OK;
}

// ---- handle ----------------------------------------------------------------------------------
struct hsddp_handle_t {
    // the slot costs / |Defect|^2 of the last rollout (k_rollout's per-slot outputs) belong to the
    // working trajectory under the current cost parameters: k_lq need not recompute them
    bool slots_fresh = false;
    // every per-knot ReB (delta, eps) still equals the descriptor's initial pair, so the kernels may
    // read the two scalars (Params::reb_uniform) when the schedule keeps them there
    bool reb_at_init = true;
    hsddp_problem_desc desc;
    hsddp_options opt;
    Params p;
    Bufs d;
    hipStream_t stream = nullptr;
    int *host_counter = nullptr;                // [16]: k_count's activity counts, stat sums, the graphs' counts
    std::vector<hipEvent_t> events;             // the stats timer's pool (reused, destroyed with the handle)
    // hsddp_solve's inner iteration + activity count as replayed hipGraphs (early-exit mode), keyed
    // by the launch arguments they froze; a small cache so the receding-horizon tick's recurring
    // layouts and swapped warm-start buffers find theirs again (round-robin eviction)
    struct IterGraph {
        hipGraphExec_t exec = nullptr;
        Params p;
        Bufs d;
        double alpha = 0;
        int par = 0;  // which host count slot (host_counter[8 + 4 * par + 1]) its copy fills
    } iter_graph[8];
    int iter_graph_next = 0;
    // hsddp_advance's shift without its own synchronisation: the host rows its pageable copies read
    // stay here until the advance synchronises, and the touchdown-overflow flag is read then
    std::vector<std::vector<int>> shift_keep;
    bool shift_overflow_pending = false;
    size_t scratch_reserved = 0;  // scratch bytes the pending shift's maps occupy (build_refs goes after)
    hipEvent_t iter_done[2] = {nullptr, nullptr};  // recorded after each replay, by parity
    std::vector<void *> allocs;
    size_t bytes = 0;
    int Bref = 1;
    bool have_problem = false;
    std::vector<int> contacts;  // host copy [B][P+1][4]: maps the compact K rows to controls
    bool contacts_current = false;  // `contacts` belong to the current layout (not stale after a shift)
    void *scratch = nullptr;    // device staging for the MPC-side calls (grown on demand)
    size_t scratch_bytes = 0;
    // receding-horizon state (HKDProblemData, HKDProblem.h:20-66): is_phase_reach_end per phase,
    // state-slot capacity (a shift keeps Kc and may add phases), and the second set of compact gain
    // rows the shift gathers into (allocated by the first shift; the new Xbar / Ubar rows go to each
    // element's third trajectory buffer)
    std::vector<int> reach_end;
    size_t S_cap = 0;
    void *spare_K = nullptr;
    // ... and of the constraint parameters the phases carry (ReB per knot, touchdown constraints)
    double *spare_reb_delta = nullptr, *spare_reb_eps = nullptr, *spare_al_sigma = nullptr, *spare_al_lambda = nullptr;
    int *spare_td_mask = nullptr;
    double *spare_cf_u = nullptr;
    int *spare_cf_flag = nullptr;
    double *shift_stage = nullptr;  // [3][B][S_cap][24] (ShiftArgs::stage), at the first stride-changing shift
    bool need_inputs = false;   // a shift changed the layout: update_problem before solving
    double *ref_table = nullptr;  // reference samples [n][RT_W] (hsddp_set_reference_table)
    int ref_n = 0;
    float ref_dt = 0;
    bool refs_on_device = false;  // references built by hsddp_build_references for this layout
    bool ref_cols_stale = true;   // Bufs::ref_t behind the reference rows (refreshed by begin_launches)
    // reference-driven MPC state (hsddp_advance): the table's samples on the host (contacts and
    // durations are read there), each reference element's window start, the window length and
    // the simulation step of the last hsddp_build_references, QuadReference::t_cur, and the
    // contact durations of every element's phases [B][P][4] (HKDProblemData::contact_durations)
    std::vector<hsddp_quad_state> table_host;
    std::vector<int> win_start;
    int win_len = 0;
    float dt_sim = 0, t_cur = 0;
    std::vector<double> durations;
    int retry_cap_alloc = 0, retry_m_alloc = 0;  // parallel regularisation retry scratch (k_riccati_retry)
    float *hist = nullptr;  // solver-info history [B][p.hcap][4] (grown by ensure_history)
    // per-element layouts (hsddp_set_element_layouts): host copies of Bufs::lay; empty = the handle's
    std::vector<Layout> lays;
    std::vector<int> reach_el;  // [B][16] is_phase_reach_end per element (with per-element layouts)
    double *value0 = nullptr;  // G[0], H[0] per phase [B][16][600] (hsddp_set_value_export)
    // asynchronous command extraction (hsddp_extract_commands_async): two device record buffers, two
    // pinned host buffers, a copy stream and per buffer the event of its last copy
    hsddp_mpc_command *cmd_dev[2] = {nullptr, nullptr}, *cmd_host[2] = {nullptr, nullptr};
    hipStream_t copy_stream = nullptr;
    hipEvent_t cmd_ready[2] = {nullptr, nullptr}, cmd_copied[2] = {nullptr, nullptr};
    char *cmd_in_host[2] = {nullptr, nullptr};  // pinned staging of each ticket's durations / feet
    size_t cmd_in_bytes[2] = {0, 0};
    int cmd_next = 0;
};

// device staging area of at least `bytes` (contents not preserved when it grows)
static int scratch(hsddp_handle h, size_t bytes, char **out)
{
    if (bytes > h->scratch_bytes) {
        if (h->scratch) hipFree(h->scratch);
        h->scratch = nullptr;
        h->scratch_bytes = 0;
        hipError_t e = hipMalloc(&h->scratch, bytes);
        if (e != hipSuccess) return fail(HSDDP_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
        h->scratch_bytes = bytes;
    }
    *out = (char *)h->scratch;
    return HSDDP_OK;
}

// the layout of element b: the handle's, or its own (hsddp_set_element_layouts)
static Layout layout_of(hsddp_handle h, size_t b)
{
    if (!h->lays.empty()) return h->lays[b];
    const Params &p = h->p;
    Layout L{};
    L.P = p.P; L.S = p.S; L.has_tail = p.has_tail;
    for (int i = 0; i < p.P; ++i) { L.N[i] = p.N[i]; L.s0[i] = p.s0[i]; L.k0[i] = p.k0[i]; L.ss[i] = p.ss[i]; }
    return L;
}

// phase of control slot kc in a layout
static int phase_of_control(const Layout &L, int kc)
{
    int i = 0;
    while (i + 1 < L.P && kc >= L.k0[i + 1]) ++i;
    return i;
}

// control u of compact gain row q at control slot k of element b (KCW layout, hsddp_internal.h)
static int coupled_control(hsddp_handle h, size_t b, size_t k, int q)
{
    const Params &p = h->p;
    const int i = phase_of_control(layout_of(h, b), (int)k);
    const int c = h->contacts[(b * (p.P + 1) + i) * 4 + q / 3];
    return c ? q : 12 + q;
}

template <typename T>
static int dalloc(hsddp_handle h, T *&ptr, size_t n)
{
    void *p = nullptr;
    size_t sz = n * sizeof(T);
    if (sz == 0) sz = 16;
    hipError_t e = hipMalloc(&p, sz);
    if (e != hipSuccess) return fail(HSDDP_ERR_ALLOC, std::string("hipMalloc: ") + hipGetErrorString(e));
    // zeroed on the handle's stream once it exists: the null stream is not ordered with a
    // non-blocking stream, so a null-stream memset of a buffer allocated mid-solve (the shift's
    // spares) could land after the kernel that fills it
    if (h->stream) hipMemsetAsync(p, 0, sz, h->stream);
    else {
        hipMemset(p, 0, sz);
        hipStreamSynchronize(nullptr);
    }
    h->allocs.push_back(p);
    h->bytes += sz;
    ptr = (T *)p;
    return HSDDP_OK;
}

static void fill_params(hsddp_handle h)
{
    h->slots_fresh = false;
    Params &p = h->p;
    const hsddp_problem_desc &ds = h->desc;
    const hsddp_options &o = h->opt;
    p.dt = ds.dt;
    p.dt_m = ds.dt / hkd::kMass;
    {
        const char *tr = std::getenv("HSDDP_TRACE");
        p.trace = (tr && tr[0] == '1') ? 1 : 0;
    }
    p.mu = ds.cparams.mu_fric;
    p.grf_delta = ds.cparams.grf_delta; p.grf_delta_min = ds.cparams.grf_delta_min; p.grf_eps = ds.cparams.grf_eps;
    p.td_sigma = ds.cparams.td_sigma; p.td_sigma_max = ds.cparams.td_sigma_max; p.td_lambda = ds.cparams.td_lambda;
    p.ground = ds.cparams.ground_height;
    const hsddp_hkd_weights &w = ds.weights;
    for (int j = 0; j < 3; ++j) { p.qbase[j] = w.q_eul[j]; p.qbase[3 + j] = w.q_pos[j]; p.qbase[6 + j] = w.q_omega[j]; p.qbase[9 + j] = w.q_v[j]; }
    p.q_qJ = w.q_qJ;
    for (int j = 0; j < 24; ++j) p.qf_scale[j] = w.qf_scale[j];
    p.qf_gain = w.qf_gain; p.r_grf = w.r_grf; p.r_qJd = w.r_qJd;
    for (int j = 0; j < 3; ++j) p.foot_w[j] = w.foot_w[j];
    p.foot_gain = w.foot_gain; p.foot_term_cost = w.foot_term_cost; p.foot_term_grad = w.foot_term_grad;
    p.alpha = o.alpha; p.gamma = o.gamma; p.update_penalty = o.update_penalty; p.update_relax = o.update_relax;
    p.update_regularization = o.update_regularization; p.update_ReB = o.update_ReB;
    p.cost_thresh = o.cost_thresh; p.tconstr_thresh = o.tconstr_thresh; p.pconstr_thresh = o.pconstr_thresh;
    p.feas_thresh = o.dynamics_feas_thresh; p.merit_scale = o.merit_scale; p.merit_offset = o.merit_offset;
    p.AL_active = o.AL_active; p.ReB_active = o.ReB_active; p.no_early_exit = o.no_early_exit;
    p.ms0 = o.MS ? 0 : 1;  // single shooting (MultiPhaseDDP.cpp:326-329; SinglePhase.cpp:214)
    // With update_ReB = update_relax = 1 (the shipped settings) update_REB_params leaves every
    // (delta, eps) at its initial value (ConstraintsBase.h:168-183): the kernels then read the two
    // scalars instead of the per-knot arrays.
    p.reb_uniform = o.update_ReB == 1.0 && o.update_relax == 1.0 && p.grf_delta >= p.grf_delta_min && h->reb_at_init;
    p.grf_inv_delta = 1.0 / p.grf_delta;
    p.grf_log_delta = std::log(p.grf_delta);
    // attempts of backward_sweep_regularized after the first, at most (from mu = 0: 1e-3, then
    // x update_regularization while <= 1e2); the parallel retry holds that many per deferred element
    int M = 0;
    if (o.update_regularization > 1) {
        double mu = 0;
        for (;;) {
            mu = std::fmax(mu * o.update_regularization, 1e-03);
            if (mu > 1e2) break;
            if (++M > 64) { M = 0; break; }
        }
    }
    p.retry_m = M;
    // value export writes G[0], H[0] from the sweep that succeeds: the in-kernel retry loop only.
    // Below 4 elements (C1: one robot) the retries run in k_riccati too: the retry and select
    // launches (≈ 10 µs of a 340 µs inner iteration at B = 1) cost more than the rare sequential
    // retry of a lone element saves.
    p.retry_cap = (M > 0 && M <= h->retry_m_alloc && !p.store_value && p.B >= 4) ? h->retry_cap_alloc : 0;
}

// the solver-info history holds every entry one solve with the handle's options can push: the
// initial one and one per inner iteration (MultiPhaseDDP.cpp:277-280, 368-371)
static int ensure_history(hsddp_handle h)
{
    const long need = 1 + (long)std::max(0, h->opt.max_AL_iter) * std::max(0, h->opt.max_DDP_iter);
    if (h->hist && need <= h->p.hcap) return HSDDP_OK;
    const int cap = (int)std::min<long>(std::max<long>(need, 16), 1 << 20);
    float *nh = nullptr;
    HIPCHK(hipMalloc(&nh, (size_t)h->p.B * cap * 4 * sizeof(float)));
    HIPCHK(hipMemset(nh, 0, (size_t)h->p.B * cap * 4 * sizeof(float)));
    HIPCHK(hipStreamSynchronize(nullptr));  // (null-stream work is not ordered with h->stream)
    if (h->hist) {
        HIPCHK(hipStreamSynchronize(h->stream));
        hipFree(h->hist);
        h->bytes -= (size_t)h->p.B * h->p.hcap * 4 * sizeof(float);
    }
    h->hist = nh;
    h->d.hist = nh;
    h->p.hcap = cap;
    h->bytes += (size_t)h->p.B * cap * 4 * sizeof(float);
    return HSDDP_OK;
}

extern "C" int hsddp_create(const hsddp_problem_desc *desc, hsddp_handle *out)
{
    if (!desc || !out) return fail(HSDDP_ERR_ARG, "null argument");
    if (desc->batch < 1 || desc->n_phases < 1 || desc->n_phases > HSDDP_MAX_PHASES || !(desc->dt > 0))
        return fail(HSDDP_ERR_ARG, "invalid batch / n_phases / dt");
    for (int i = 0; i < desc->n_phases; ++i)
        if (desc->horizons[i] < 1) return fail(HSDDP_ERR_ARG, "phase horizons must be >= 1");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1)
        return fail(HSDDP_ERR_DEVICE, "no HIP device available (the solver has no CPU fallback)");
    if (desc->device < 0 || desc->device >= ndev) return fail(HSDDP_ERR_DEVICE, "device ordinal out of range");
    HIPCHK(hipSetDevice(desc->device));
    hsddp_handle h = new hsddp_handle_t();
    h->desc = *desc;
    hsddp_default_options(&h->opt);
    Params &p = h->p;
    p.B = desc->batch;
    p.P = desc->n_phases;
    int s = 0, k = 0;
    for (int i = 0; i < p.P; ++i) {
        p.N[i] = desc->horizons[i]; p.s0[i] = s; p.k0[i] = k;
        s += p.N[i] + 1; k += p.N[i];
    }
    p.S = s; p.Kc = k;
    p.ref_per_element = desc->ref_per_element ? 1 : 0;
    p.fp32 = desc->riccati_fp32 ? 1 : 0;
    h->Bref = p.ref_per_element ? p.B : 1;
    fill_params(h);
    for (int i = 0; i < p.P; ++i) p.ss[i] = p.N[i] + 1;  // every knot a shooting state (HKDProblem.cpp:104)
    p.has_tail = 0;
    h->reach_end.assign(p.P, 0);  // HKDProblem.cpp:56-57 compares a contact with itself (quirk A15)
    // State-slot buffers hold Kc + HSDDP_MAX_PHASES slots (a receding-horizon shift keeps Kc and can
    // add phases, S = Kc + P); per-phase buffers hold HSDDP_MAX_PHASES phases.
    h->S_cap = (size_t)p.Kc + HSDDP_MAX_PHASES;
    const size_t B = p.B, S = h->S_cap, Kc = p.Kc, P = HSDDP_MAX_PHASES, Br = h->Bref;
    Bufs &d = h->d;
    int *contacts; double *x0, *rx, *ru, *rf;
    int rc = 0;
    if ((rc = dalloc(h, contacts, B * (P + 1) * 4)) || (rc = dalloc(h, x0, B * NX)) || (rc = dalloc(h, rx, Br * S * NX)) ||
        (rc = dalloc(h, ru, Br * S * NX)) || (rc = dalloc(h, rf, Br * S * 12)) || (rc = dalloc(h, d.ref_t, REF_COLS * Br * S)) ||
        (rc = dalloc(h, d.X3, 3 * B * S * NX)) ||
        (rc = dalloc(h, d.D3, 3 * B * S * NX)) || (rc = dalloc(h, d.U3, 3 * B * Kc * NX)) || (rc = dalloc(h, d.sel, B)) ||
        (rc = dalloc(h, d.cf_u, B * Kc * 12)) || (rc = dalloc(h, d.cf_flag, B * Kc)) ||
        (rc = dalloc(h, d.dX, B * S * NX)) ||
        (rc = dalloc(h, d.dU, B * Kc * NX)) ||
        (rc = dalloc(h, d.du, B * Kc * NX)) || (rc = dalloc(h, d.dbg, B * 16)) ||
        (p.fp32 ? ((rc = dalloc(h, d.K32, B * Kc * KCW)) || (rc = dalloc(h, d.lq32, B * Kc * LQW32)) ||
                   (rc = dalloc(h, d.def32, B * S * NX)))
                : ((rc = dalloc(h, d.K, B * Kc * KCW)) || (rc = dalloc(h, d.lq, B * Kc * LQW)))) ||
        (rc = dalloc(h, d.term, B * P * TW)) || (rc = dalloc(h, d.reb_delta, B * Kc * 20)) ||
        (rc = dalloc(h, d.reb_eps, B * Kc * 20)) || (rc = dalloc(h, d.al_sigma, B * P * MTD * 4)) ||
        (rc = dalloc(h, d.al_lambda, B * P * MTD * 4)) || (rc = dalloc(h, d.td_mask, B * P * MTD)) ||
        (rc = dalloc(h, d.term_h, B * P * 4)) ||
        (rc = dalloc(h, d.slot_cost, B * S)) || (rc = dalloc(h, d.slot_feas, B * S)) || (rc = dalloc(h, d.slot_viol, B * S)) ||
        (rc = dalloc(h, d.slot_div, B * S)) || (rc = dalloc(h, d.el, B)) || (rc = dalloc(h, d.counter, 8)) || (rc = dalloc(h, d.ls_live, LS_LIVE)) ||
        (rc = dalloc(h, (Layout *&)d.lay, B)) || (rc = dalloc(h, (int *&)d.pairs, 2 * B + 2))) {
        hsddp_destroy(h);
        return rc;
    }
    d.contacts = contacts; d.x0 = x0; d.ref_x = rx; d.ref_u = ru; d.ref_foot = rf;
    d.ref_tw = Br * S;
    d.xs3 = B * S * NX;  // (S = S_cap here)
    d.us3 = B * Kc * NX;
    d.rows3 = (int)(B * S);
    d.urows3 = (int)(B * Kc);
    {   // parallel regularisation retries: p.retry_m attempts for each of up to `cap` deferred elements
        // per launch (HSDDP_SEQUENTIAL_RETRY=1 keeps every retry inside k_riccati: a diagnostic for
        // tests).  Scratch per deferred element: M attempts x (Kc gain rows + Kc dU rows), 8.5 MB at the
        // metric's horizon in fp64 (17 x 200 x 312 x 8 B).  The cap is 128 elements within a 256 MiB
        // budget (30 at the metric's horizon; device_bytes counts it): the oracle's jump solves defer a
        // few elements of 4096 per iteration, and deferrals past the cap run the same retries inside
        // k_riccati.  HSDDP_RETRY_CAP=n lowers the cap (a diagnostic: tests use it to send deferrals
        // past the cap into the in-kernel loop).
        const char *seq = std::getenv("HSDDP_SEQUENTIAL_RETRY");
        const char *capenv = std::getenv("HSDDP_RETRY_CAP");
        const size_t per_elem = (size_t)std::max(1, p.retry_m) * Kc * (KCW * (p.fp32 ? 4 : 8) + NX * 8 + 4);
        size_t cap = std::min<size_t>(std::min<size_t>(128, B), std::max<size_t>(2, ((size_t)256 << 20) / per_elem));
        if (capenv && std::atoi(capenv) > 0) cap = std::min<size_t>(cap, (size_t)std::atoi(capenv));
        const size_t M = (seq && seq[0] == '1') ? 0 : p.retry_m, n = cap * M;
        if (M > 0) {
            void *rk;
            if ((rc = dalloc(h, d.retry_list, cap)) || (rc = dalloc(h, d.retry_count, 1)) ||
                (rc = dalloc(h, d.retry_flag, n)) || (rc = dalloc(h, d.retry_dU, n * Kc * NX)) ||
                (rc = dalloc(h, d.retry_dv, n)) ||
                (rc = p.fp32 ? dalloc(h, (float *&)rk, n * Kc * KCW) : dalloc(h, (double *&)rk, n * Kc * KCW))) {
                hsddp_destroy(h);
                return rc;
            }
            d.retry_K = rk;
            h->retry_cap_alloc = (int)cap;
            h->retry_m_alloc = (int)M;
            fill_params(h);
        }
    }
    if (hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void **)&h->host_counter, 16 * sizeof(int), 0) != hipSuccess) {
        hsddp_destroy(h);
        return fail(HSDDP_ERR_DEVICE, "stream / pinned allocation failed");
    }
    if ((rc = ensure_history(h))) {
        hsddp_destroy(h);
        return rc;
    }
    launch_init_params(p, d, h->stream);
    launch_reset_elements(p, d, h->stream);
    if (hipStreamSynchronize(h->stream) != hipSuccess) {
        hsddp_destroy(h);
        return fail(HSDDP_ERR_DEVICE, "kernel launch failed at create (is the library built for this GPU?)");
    }
    *out = h;
    return HSDDP_OK;
}

extern "C" int hsddp_destroy(hsddp_handle h)
{
    if (!h) return HSDDP_OK;
    hipSetDevice(h->desc.device);
    if (h->stream) hipStreamSynchronize(h->stream);
    for (void *p : h->allocs) hipFree(p);
    if (h->scratch) hipFree(h->scratch);
    if (h->ref_table) hipFree(h->ref_table);
    if (h->hist) hipFree(h->hist);
    if (h->value0) hipFree(h->value0);

    for (auto &g : h->iter_graph)
        if (g.exec) hipGraphExecDestroy(g.exec);
    for (hipEvent_t e : h->iter_done)
        if (e) hipEventDestroy(e);
    if (h->host_counter) hipHostFree(h->host_counter);
    if (h->copy_stream) hipStreamSynchronize(h->copy_stream);
    for (int q = 0; q < 2; ++q) {
        if (h->cmd_dev[q]) hipFree(h->cmd_dev[q]);
        if (h->cmd_host[q]) hipHostFree(h->cmd_host[q]);
        if (h->cmd_ready[q]) hipEventDestroy(h->cmd_ready[q]);
        if (h->cmd_copied[q]) hipEventDestroy(h->cmd_copied[q]);
        if (h->cmd_in_host[q]) hipHostFree(h->cmd_in_host[q]);
    }
    if (h->copy_stream) hipStreamDestroy(h->copy_stream);
    for (hipEvent_t e : h->events) hipEventDestroy(e);
    if (h->stream) hipStreamDestroy(h->stream);
    delete h;
    return HSDDP_OK;
}

extern "C" int hsddp_validate_options(const hsddp_options *o)
{
    if (!o) return fail(HSDDP_ERR_ARG, "null argument");
    if (!(o->alpha > 0 && o->alpha < 1)) return fail(HSDDP_ERR_ARG, "alpha must lie in (0, 1)");
    if (o->max_AL_iter < 0 || o->max_DDP_iter < 0) return fail(HSDDP_ERR_ARG, "negative iteration budget");
    // backward_sweep_regularized (MultiPhaseDDP.cpp:150-167) raises mu = max(mu * factor, 1e-3)
    // until a sweep succeeds or mu > 1e2.  A factor <= 1 never gets there (the reference spins
    // forever on the first failed sweep) and a factor barely above 1 takes thousands of sweeps per
    // failure; both are refused rather than left to hang a GPU wave.
    if (!(o->update_regularization > 1))
        return fail(HSDDP_ERR_ARG, "update_regularization must exceed 1 (the regularisation schedule would never end)");
    int m = 0;
    for (double mu = 0;; ++m) {
        mu = std::fmax(mu * o->update_regularization, 1e-03);
        if (mu > 1e2) break;
        if (m >= HSDDP_MAX_REG_ATTEMPTS)
            return fail(HSDDP_ERR_ARG, "update_regularization too close to 1: more than HSDDP_MAX_REG_ATTEMPTS "
                                       "regularisation retries per failed sweep");
    }
    return HSDDP_OK;
}

extern "C" int hsddp_set_options(hsddp_handle h, const hsddp_options *o)
{
    if (!h || !o) return fail(HSDDP_ERR_ARG, "null argument");
    int rc = hsddp_validate_options(o);
    if (rc) return rc;
    // the solver-info history must hold every entry of the new budget (1 + outer x inner)
    if (1 + (long)std::max(0, o->max_AL_iter) * std::max(0, o->max_DDP_iter) > (1L << 20))
        return fail(HSDDP_ERR_ARG, "max_AL_iter * max_DDP_iter exceeds the solver-info history (2^20 entries)");
    const hsddp_options old = h->opt;
    h->opt = *o;
    if ((rc = ensure_history(h))) {  // allocation failed: the handle keeps its previous options
        h->opt = old;
        return rc;
    }
    fill_params(h);
    return HSDDP_OK;
}

// install per-element layouts: device records, sweep pairs (equal layouts share a wave), strides
static int set_layouts(hsddp_handle h, const std::vector<Layout> &lays)
{
    h->slots_fresh = false;
    Params &p = h->p;
    const int B = p.B;
    int Pmax = 0, Smax = 0, tail = 0;
    for (auto &L : lays) { Pmax = std::max(Pmax, L.P); Smax = std::max(Smax, L.S); tail |= L.has_tail; }
    std::map<std::vector<int>, std::vector<int>> groups;
    for (int b = 0; b < B; ++b) {
        std::vector<int> key(lays[b].N, lays[b].N + lays[b].P);
        key.push_back(-1);
        key.insert(key.end(), lays[b].ss, lays[b].ss + lays[b].P);
        groups[key].push_back(b);
    }
    std::vector<int> pairs;
    for (auto &g : groups)
        for (size_t j = 0; j < g.second.size(); j += 2) {
            pairs.push_back(g.second[j]);
            pairs.push_back(j + 1 < g.second.size() ? g.second[j + 1] : -1);
        }
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipMemcpy((void *)h->d.lay, lays.data(), B * sizeof(Layout), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy((void *)h->d.pairs, pairs.data(), pairs.size() * sizeof(int), hipMemcpyHostToDevice));
    h->lays = lays;
    p.elem_layout = 1;
    p.n_pairs = (int)pairs.size() / 2;
    p.P = Pmax;  // strides of the per-phase and per-slot buffers
    p.S = Smax;
    p.has_tail = tail;
    for (int i = 0; i < HSDDP_MAX_PHASES; ++i) { p.N[i] = 0; p.s0[i] = 0; p.k0[i] = 0; p.ss[i] = 0; }
    return HSDDP_OK;
}

extern "C" int hsddp_set_element_layouts(hsddp_handle h, const int *n_phases, const int *horizons)
{
    if (!h || !n_phases || !horizons) return fail(HSDDP_ERR_ARG, "null argument");
    Params &p = h->p;
    const int B = p.B;
    if (B > 1 && h->Bref == 1)  // a shared reference is laid out for one layout
        return fail(HSDDP_ERR_ARG, "per-element layouts need per-element references (ref_per_element = 1)");
    std::vector<Layout> lays(B);
    for (int b = 0; b < B; ++b) {
        Layout &L = lays[b];
        L = Layout{};
        L.P = n_phases[b];
        if (L.P < 1 || L.P > HSDDP_MAX_PHASES) return fail(HSDDP_ERR_ARG, "element n_phases must lie in 1..16");
        int s = 0, k = 0;
        for (int i = 0; i < L.P; ++i) {
            const int N = horizons[(size_t)b * HSDDP_MAX_PHASES + i];
            if (N < 1) return fail(HSDDP_ERR_ARG, "phase horizons must be >= 1");
            L.N[i] = N; L.s0[i] = s; L.k0[i] = k; L.ss[i] = N + 1;
            s += N + 1; k += N;
        }
        if (k != p.Kc) return fail(HSDDP_ERR_ARG, "every element's horizons must sum to the handle's Kc");
        L.S = s;
    }
    int rc = set_layouts(h, lays);
    if (rc) return rc;
    h->reach_el.assign((size_t)B * HSDDP_MAX_PHASES, 0);  // HKDProblem.cpp:56-57 (quirk A15)
    h->have_problem = false;  // inputs of the new layouts next (hsddp_upload_problem)
    h->contacts_current = false;
    h->refs_on_device = false;
    h->ref_cols_stale = true;
    return HSDDP_OK;
}

// the layout of every element: n_phases [B], horizons / shooting / reach_end [B][16] (any NULL)
extern "C" int hsddp_get_element_layouts(hsddp_handle h, int *n_phases, int *horizons, int *shooting, int *reach_end)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    for (size_t b = 0; b < (size_t)h->p.B; ++b) {
        const Layout L = layout_of(h, b);
        if (n_phases) n_phases[b] = L.P;
        for (int i = 0; i < HSDDP_MAX_PHASES; ++i) {
            const bool in = i < L.P;
            if (horizons) horizons[b * HSDDP_MAX_PHASES + i] = in ? L.N[i] : 0;
            if (shooting) shooting[b * HSDDP_MAX_PHASES + i] = in ? L.ss[i] : 0;
            if (reach_end)
                reach_end[b * HSDDP_MAX_PHASES + i] =
                    in ? (h->lays.empty() ? h->reach_end[i] : h->reach_el[b * HSDDP_MAX_PHASES + i]) : 0;
        }
    }
    return HSDDP_OK;
}

static int h2d(void *dst, const void *src, size_t bytes, hipStream_t st)
{
    HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, st));
    return HSDDP_OK;
}

// contacts, x0 and references of the current layout to the device
static int upload_inputs(hsddp_handle h, const int *contacts, const double *x0, const double *ref_x,
                         const double *ref_u, const double *ref_foot)
{
    if (!h || !x0) return fail(HSDDP_ERR_ARG, "null argument");
    const bool keep_refs = !ref_x && !ref_u && !ref_foot;
    if (!keep_refs && (!ref_x || !ref_u || !ref_foot)) return fail(HSDDP_ERR_ARG, "references: all three or none");
    if (keep_refs && !h->refs_on_device)
        return fail(HSDDP_ERR_ARG, "no device references for this layout (hsddp_build_references)");
    if (!h->lays.empty() && h->Bref == 1 && h->p.B > 1)  // a shared reference is laid out for one layout
        return fail(HSDDP_ERR_ARG, "per-element layouts need per-element references (desc.ref_per_element = 1)");
    HIPCHK(hipSetDevice(h->desc.device));
    const Params &p = h->p;
    const size_t B = p.B, S = p.S, P = p.P, Br = h->Bref;
    // contacts NULL: the handle's own (those hsddp_advance derived for this layout)
    const std::vector<int> own = contacts ? std::vector<int>() : h->contacts;
    if (!contacts) {
        if (!h->contacts_current || own.size() != B * (P + 1) * 4)
            return fail(HSDDP_ERR_ARG, "no contacts of this layout on the handle");
        contacts = own.data();
    }
    for (size_t q = 0; q < B * (P + 1) * 4; ++q)
        if (contacts[q] != 0 && contacts[q] != 1) return fail(HSDDP_ERR_ARG, "contacts must be 0/1");
    int rc;
    if ((rc = h2d((void *)h->d.contacts, contacts, B * (P + 1) * 4 * sizeof(int), h->stream)) ||
        (rc = h2d((void *)h->d.x0, x0, B * NX * sizeof(double), h->stream)))
        return rc;
    if (!keep_refs &&
        ((rc = h2d((void *)h->d.ref_x, ref_x, Br * S * NX * sizeof(double), h->stream)) ||
         (rc = h2d((void *)h->d.ref_u, ref_u, Br * S * NX * sizeof(double), h->stream)) ||
         (rc = h2d((void *)h->d.ref_foot, ref_foot, Br * S * 12 * sizeof(double), h->stream))))
        return rc;
    if (!keep_refs) {
        h->refs_on_device = false;
        h->ref_cols_stale = true;
    }
    h->contacts.assign(contacts, contacts + B * (P + 1) * 4);
    h->contacts_current = true;
    return HSDDP_OK;
}

extern "C" int hsddp_upload_problem(hsddp_handle h, const int *contacts, const double *x0, const double *ref_x,
                                    const double *ref_u, const double *ref_foot)
{
    int rc = upload_inputs(h, contacts, x0, ref_x, ref_u, ref_foot);
    if (rc) return rc;
    const Params &p = h->p;
    const size_t B = p.B, S = p.S, Br = h->Bref;
    // default warm start: Xbar = X = reference (HKDProblem.cpp:84-90), Ubar = U = 0, K = 0
    HIPCHK(hipMemsetAsync(h->d.sel, 0, B * sizeof(int), h->stream));  // nominal and working rows in buffer 0
    if (Br == 1) launch_broadcast(h->d.X3, h->d.ref_x, S * NX, B, h->stream);
    else HIPCHK(hipMemcpyAsync(h->d.X3, h->d.ref_x, B * S * NX * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
    HIPCHK(hipMemsetAsync(h->d.U3, 0, B * p.Kc * NX * sizeof(double), h->stream));
    if (p.fp32) HIPCHK(hipMemsetAsync(h->d.K32, 0, B * p.Kc * KCW * sizeof(float), h->stream));
    else HIPCHK(hipMemsetAsync(h->d.K, 0, B * p.Kc * KCW * sizeof(double), h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    h->have_problem = true;
    h->need_inputs = false;
    return hsddp_upload_warm_start(h, nullptr, nullptr, nullptr);
}

static int reset_working(hsddp_handle h, bool params);

extern "C" int hsddp_update_problem(hsddp_handle h, const int *contacts, const double *x0, const double *ref_x,
                                    const double *ref_u, const double *ref_foot)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    int rc = upload_inputs(h, contacts, x0, ref_x, ref_u, ref_foot);
    if (rc) return rc;
    h->need_inputs = false;
    // keeps Xbar / Ubar / K, the working trajectory (X, U, Defect) and the constraint objects —
    // their ReB / AL parameters (HKDProblem::update's reset_params is a no-op, ConstraintsBase.h:
    // 165-167,341-348) and stored values — as the reference's objects live on into the next tick;
    // resets the per-element solver state; touchdown constraints added by the shift take their legs
    // from the new contact rows
    return reset_working(h, false);
}

// params (a new problem: hsddp_upload_warm_start): the working trajectory restarts at the warm
// start (X = Xbar, U = Ubar, Defect = 0), the ReB / AL parameters and touchdown constraints return
// to their initial values and the constraint values to zero — else all of them are kept.  Either
// way dX = du = dU = 0 (the next initial rollout multiplies them by eps = 0), the per-element solver
// state is cleared and pending touchdown masks are resolved from the contact rows.
static int reset_working(hsddp_handle h, bool params)
{
    const Params &p = h->p;
    const size_t B = p.B, S = p.S, Kc = p.Kc;
    Bufs &d = h->d;
    if (params) launch_reset_working(p, d, h->stream);  // X = Xbar, U = Ubar (one buffer), Defect = 0
    // dX, du, dU: a new problem's are zero.  Between solves the initial rollout (eps = 0) does not
    // read them (fma_step / add_step) and the sweep and linear rollout rewrite them before any
    // trial, so an update keeps them (474 MB of memsets at B = 4096 saved per MPC tick) — except dX
    // with single shooting, which no linear rollout writes: the trials read it (zero, as in a
    // problem that never ran multiple shooting; the reference's is never written there either)
    if (params || p.ms0) HIPCHK(hipMemsetAsync(d.dX, 0, B * S * NX * sizeof(double), h->stream));
    if (params) {
        HIPCHK(hipMemsetAsync(d.du, 0, B * Kc * NX * sizeof(double), h->stream));
        HIPCHK(hipMemsetAsync(d.dU, 0, B * Kc * NX * sizeof(double), h->stream));
    }
    if (params) {
        launch_init_params(p, d, h->stream);
        h->reb_at_init = true;
        fill_params(h);
    }
    launch_resolve_td(p, d, h->stream);
    launch_reset_elements(p, d, h->stream);
    HIPCHK(hipStreamSynchronize(h->stream));
    h->slots_fresh = false;
    return HSDDP_OK;
}

extern "C" int hsddp_upload_warm_start(hsddp_handle h, const double *Xbar, const double *Ubar, const double *K)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    h->slots_fresh = false;
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    HIPCHK(hipSetDevice(h->desc.device));
    const Params &p = h->p;
    const size_t B = p.B, S = p.S, Kc = p.Kc;
    Bufs &d = h->d;
    int rc;
    launch_normalize(p, d, h->stream);  // every element's nominal rows in buffer 0
    if (Xbar && (rc = h2d(d.X3, Xbar, B * S * NX * sizeof(double), h->stream))) return rc;
    if (Ubar && (rc = h2d(d.U3, Ubar, B * Kc * NX * sizeof(double), h->stream))) return rc;
    if (K) { // keep the 12 coupled rows of each knot's gain (KCW layout, hsddp_internal.h)
        std::vector<double> kc(B * Kc * KCW);
        for (size_t b = 0; b < B; ++b)
            for (size_t k = 0; k < Kc; ++k)
                for (int q = 0; q < 12; ++q) {
                    const int u = coupled_control(h, b, k, q);
                    std::memcpy(&kc[((b * Kc + k) * 12 + q) * NX], K + ((b * Kc + k) * NX + u) * NX, NX * sizeof(double));
                }
        if (p.fp32) {
            std::vector<float> k32(kc.begin(), kc.end());
            if ((rc = h2d(d.K32, k32.data(), B * Kc * KCW * sizeof(float), h->stream))) return rc;
            HIPCHK(hipStreamSynchronize(h->stream));
        } else if ((rc = h2d(d.K, kc.data(), B * Kc * KCW * sizeof(double), h->stream))) {
            return rc;
        }
        HIPCHK(hipStreamSynchronize(h->stream));
    }
    return reset_working(h, true);
}

static_assert(MTD == HSDDP_MAX_TD, "touchdown constraint slots");

extern "C" int hsddp_upload_constraint_params(hsddp_handle h, const double *reb_delta, const double *reb_eps,
                                              const int *td_legs, const double *al_sigma, const double *al_lambda)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    const Params &p = h->p;
    const size_t nr = (size_t)p.B * p.Kc * 20, nt = (size_t)p.B * p.P * MTD;
    if (td_legs)
        for (size_t q = 0; q < nt; ++q)
            if (td_legs[q] < 0 || td_legs[q] > 15) return fail(HSDDP_ERR_ARG, "td_legs entries are 4-bit leg masks");
    HIPCHK(hipSetDevice(h->desc.device));
    const Bufs &d = h->d;
    int rc;
    if ((reb_delta && (rc = h2d(d.reb_delta, reb_delta, nr * sizeof(double), h->stream))) ||
        (reb_eps && (rc = h2d(d.reb_eps, reb_eps, nr * sizeof(double), h->stream))) ||
        (td_legs && (rc = h2d(d.td_mask, td_legs, nt * sizeof(int), h->stream))) ||
        (al_sigma && (rc = h2d(d.al_sigma, al_sigma, nt * 4 * sizeof(double), h->stream))) ||
        (al_lambda && (rc = h2d(d.al_lambda, al_lambda, nt * 4 * sizeof(double), h->stream))))
        return rc;
    HIPCHK(hipStreamSynchronize(h->stream));
    if (reb_delta || reb_eps) {  // the uniform-ReB shortcut holds only while every knot has the initial pair
        bool at = true;
        for (size_t q = 0; q < nr && at; ++q)
            at = (!reb_delta || reb_delta[q] == p.grf_delta) && (!reb_eps || reb_eps[q] == p.grf_eps);
        h->reb_at_init = at && h->reb_at_init;
        if (at && reb_delta && reb_eps) h->reb_at_init = true;
        fill_params(h);
    }
    h->slots_fresh = false;  // the running / terminal costs change with the parameters
    return HSDDP_OK;
}

extern "C" int hsddp_download_constraint_params(hsddp_handle h, double *reb_delta, double *reb_eps, int *td_legs,
                                                double *al_sigma, double *al_lambda)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    const Params &p = h->p;
    const size_t nr = (size_t)p.B * p.Kc * 20, nt = (size_t)p.B * p.P * MTD;
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const Bufs &d = h->d;
    if (reb_delta) HIPCHK(hipMemcpy(reb_delta, d.reb_delta, nr * sizeof(double), hipMemcpyDeviceToHost));
    if (reb_eps) HIPCHK(hipMemcpy(reb_eps, d.reb_eps, nr * sizeof(double), hipMemcpyDeviceToHost));
    if (td_legs) {
        HIPCHK(hipMemcpy(td_legs, d.td_mask, nt * sizeof(int), hipMemcpyDeviceToHost));
        for (size_t q = 0; q < nt; ++q) td_legs[q] &= 15;  // (legs only: TD_STALE is the device's)
    }
    if (al_sigma) HIPCHK(hipMemcpy(al_sigma, d.al_sigma, nt * 4 * sizeof(double), hipMemcpyDeviceToHost));
    if (al_lambda) HIPCHK(hipMemcpy(al_lambda, d.al_lambda, nt * 4 * sizeof(double), hipMemcpyDeviceToHost));
    return HSDDP_OK;
}

// The stored constraint values, formed on the host from what the device keeps (hsddp_internal.h):
// a knot's GRF values from its cf_u forces where cf_flag is set, else from its working control row;
// a touchdown constraint's residual is 0 while TD_STALE, else its phase end's (term_h, written by
// the last rollout or divergence fix-up from the working X_i[N]).
extern "C" int hsddp_download_constraint_values(hsddp_handle h, double *grf_g, double *td_h)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    if (grf_g && !h->contacts_current) return fail(HSDDP_ERR_ARG, "no contacts of this layout on the handle");
    const Params &p = h->p;
    const size_t B = p.B, Kc = p.Kc, P = p.P;
    int rc;
    std::vector<ElemState> el(B);
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipMemcpy(el.data(), h->d.el, B * sizeof(ElemState), hipMemcpyDeviceToHost));
    if (grf_g) {
        std::vector<double> U(B * Kc * NX), cfu(B * Kc * 12);
        std::vector<int> cff(B * Kc);
        if ((rc = hsddp_download_working(h, nullptr, U.data(), nullptr, nullptr, nullptr))) return rc;
        HIPCHK(hipMemcpy(cfu.data(), h->d.cf_u, cfu.size() * sizeof(double), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(cff.data(), h->d.cf_flag, cff.size() * sizeof(int), hipMemcpyDeviceToHost));
        std::fill(grf_g, grf_g + B * Kc * 20, 0.0);
        for (size_t b = 0; b < B; ++b) {
            const Layout L = layout_of(h, b);
            for (int i = 0; i < L.P; ++i)
                for (int k = 0; k < L.N[i]; ++k) {
                    const size_t q = b * Kc + L.k0[i] + k;
                    const double *f = (el[b].ovr && cff[q]) ? &cfu[q * 12] : &U[q * NX];
                    for (int l = 0; l < 4; ++l) {
                        if (!h->contacts[(b * (P + 1) + i) * 4 + l]) continue;
                        const double *fl = f + 3 * l;
                        double *g = grf_g + q * 20 + 5 * l;  // GRFConstraint rows (HKDConstraints.cpp:15-22)
                        g[0] = fl[2];
                        g[1] = -fl[0] + p.mu * fl[2];
                        g[2] = fl[0] + p.mu * fl[2];
                        g[3] = -fl[1] + p.mu * fl[2];
                        g[4] = fl[1] + p.mu * fl[2];
                    }
                }
        }
    }
    if (td_h) {
        std::vector<int> mask(B * P * MTD);
        std::vector<double> th(B * P * 4);
        HIPCHK(hipMemcpy(mask.data(), h->d.td_mask, mask.size() * sizeof(int), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(th.data(), h->d.term_h, th.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (size_t b = 0; b < B; ++b)
            for (size_t i = 0; i < P; ++i)
                for (int j = 0; j < MTD; ++j) {
                    const int m = mask[(b * P + i) * MTD + j];
                    for (int l = 0; l < 4; ++l)
                        td_h[((b * P + i) * MTD + j) * 4 + l] =
                            ((m >> l) & 1) && !(m & TD_STALE) ? th[(b * P + i) * 4 + l] : 0.0;
                }
    }
    return HSDDP_OK;
}

// ---- solve --------------------------------------------------------------------------------------
namespace {
struct Timer {
    hipStream_t st;
    bool on;
    std::vector<hipEvent_t> *pool;  // the handle's events, handed out in order (no create / destroy per launch)
    size_t used = 0;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[5];  // lq, riccati, forward, other, linear
    // the last end() event, when nothing was launched since: the next begin() reuses it (an event
    // record costs the stream a ~5 us gap, and adjacent end / begin pairs were two)
    hipEvent_t pend = nullptr;
    hipEvent_t next()
    {
        if (used == pool->size()) {
            hipEvent_t e;
            hipEventCreate(&e);
            pool->push_back(e);
        }
        return (*pool)[used++];
    }
    void begin(int cat, hipEvent_t &e0)
    {
        if (!on) return;
        (void)cat;
        if (pend) {
            e0 = pend;
            pend = nullptr;
            return;
        }
        e0 = next();
        hipEventRecord(e0, st);
    }
    // launches outside the timed categories follow: the next begin() records its own event
    void cut() { pend = nullptr; }
    void end(int cat, hipEvent_t e0)
    {
        if (!on) return;
        hipEvent_t e1 = next();
        hipEventRecord(e1, st);
        ev[cat].push_back({e0, e1});
        pend = e1;
    }
    double total(int cat)
    {
        double t = 0;
        for (auto &pr : ev[cat]) {
            float ms = 0;
            hipEventElapsedTime(&ms, pr.first, pr.second);
            t += ms;
        }
        ev[cat].clear();
        return t;
    }
};
}  // namespace

static int count_active(hsddp_handle h, int which, int &n)
{
    HIPCHK(hipMemsetAsync(h->d.counter, 0, 4 * sizeof(int), h->stream));
    launch_count(h->p, h->d, which, h->stream);
    HIPCHK(hipMemcpyAsync(h->host_counter, h->d.counter, 4 * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    n = h->host_counter[which];
    return HSDDP_OK;
}

// The solve is split so a caller can time a fixed number of inner iterations:
//   hsddp_solve_begin  = initial hybrid_rollout(0) + update_nominal + compute_cost (MultiPhaseDDP.cpp:257-260)
//                        and the first outer-iteration prologue (:284-303)
//   hsddp_iterate      = n inner iterations (:304-381) for every still-active element
//   hsddp_solve_end    = outer epilogue: AL / ReB updates and tests (:383-408)
// hsddp_solve runs the complete reference loop with per-element early exits.
static int solve_check(hsddp_handle h)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    if (h->need_inputs) return fail(HSDDP_ERR_ARG, "the layout changed (hsddp_shift): call hsddp_update_problem first");
    HIPCHK(hipSetDevice(h->desc.device));
    return HSDDP_OK;
}

static std::vector<double> ls_steps(double alpha)
{
    // line-search step sizes exactly as `while (eps > 1e-3) { ...; eps *= alpha; }` evaluates them
    std::vector<double> trials;
    for (double eps = 1; eps > 1e-3; eps *= alpha) trials.push_back(eps);
    return trials;
}

// Bufs::ref_t refreshed from the reference rows if an upload changed them since (before any
// launch that reads the references; never inside a graph capture)
static void sync_ref_columns(hsddp_handle h)
{
    if (!h->ref_cols_stale) return;
    launch_ref_columns(h->p, h->d, h->Bref, h->stream);
    h->ref_cols_stale = false;
}

static void begin_launches(hsddp_handle h)
{
    if (h->p.trace) hipMemsetAsync(h->d.dbg, 0, (size_t)h->p.B * 16 * sizeof(unsigned long long), h->stream);
    sync_ref_columns(h);
    launch_reset_elements(h->p, h->d, h->stream);
    launch_rollout(h->p, h->d, 0.0, 0, 1, -1, h->stream);
    launch_decide(h->p, h->d, 0.0, 0, 1, -1, h->stream);
    h->slots_fresh = true;
}

static void iteration_launches(hsddp_handle h, const std::vector<double> &trials, Timer &tm)
{
    const Params &p = h->p;
    const Bufs &d = h->d;
    hipStream_t st = h->stream;
    hipEvent_t e0;
    tm.begin(0, e0);
    {   // every path to here ran a rollout on the working trajectory (the initial one or the last
        // line-search trial, quirk A2) unless the cost parameters changed since (slots_fresh)
        Params pl = p;
        pl.lq_slots = h->slots_fresh ? 0 : 1;
        launch_lq(pl, d, st);
    }
    tm.end(0, e0);
    tm.begin(1, e0);
    launch_riccati(p, d, st);
    tm.end(1, e0);
    // the linear rollout with multiple shooting only (MultiPhaseDDP.cpp:326-329); with single
    // shooting the sweep forms dV and the merit (k_riccati's DV instantiation)
    if (!p.ms0) {
        tm.begin(4, e0);
        launch_lin_rollout(p, d, st);
        tm.end(4, e0);
    }
    tm.begin(2, e0);
    for (size_t t = 0; t < trials.size(); ++t) {
        launch_rollout(p, d, trials[t], t + 1 == trials.size(), 0, (int)t, st);
        launch_decide(p, d, trials[t], t + 1 == trials.size(), 0, (int)t, st);
    }
    tm.end(2, e0);
    h->slots_fresh = true;
}

// One early-exit inner iteration of hsddp_solve (MultiPhaseDDP.cpp:304-381 and the `n == 0` test)
// replayed from a hipGraph: the ~15 launches, the count kernel and the pinned read-back of the
// activity count go to the device as one submission.  At B = 1 (BASELINE config 1) the iteration's
// kernels are a few microseconds each and the host's per-launch cost was the critical path.  The
// graph freezes the launch arguments (Params, Bufs, the step sizes): it is re-captured whenever
// they differ from the ones it was built with.  The per-phase timers are not recorded in this mode
// (hsddp_stats carries ms_total only); HSDDP_NO_GRAPH=1 restores launch-by-launch issue.
static bool graphs_enabled()
{
    const char *e = std::getenv("HSDDP_NO_GRAPH");  // read per solve: a test switches it in-process
    return !(e && *e && *e != '0');
}

static int graph_launch(hsddp_handle h, const std::vector<double> &trials, int par)
{
    Params pl = h->p;
    pl.lq_slots = h->slots_fresh ? 0 : 1;
    hsddp_handle_t::IterGraph *hit = nullptr;
    for (auto &c : h->iter_graph)
        if (c.exec && c.par == par && !std::memcmp(&c.p, &pl, sizeof(Params)) &&
            !std::memcmp(&c.d, &h->d, sizeof(Bufs)) && c.alpha == h->opt.alpha)
            hit = &c;
    if (!hit) {
        auto &g = h->iter_graph[h->iter_graph_next];
        h->iter_graph_next = (h->iter_graph_next + 1) % 8;
        if (g.exec) {
            // the victim may be the iteration queued last (still on the stream): drain the stream
            // before its exec goes away (evictions are rare: 8 keys cover an MPC tick's recurring ones)
            HIPCHK(hipStreamSynchronize(h->stream));
            HIPCHK(hipGraphExecDestroy(g.exec));
        }
        g.exec = nullptr;
        HIPCHK(hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal));
        Timer off{h->stream, false, &h->events};
        iteration_launches(h, trials, off);
        launch_count(h->p, h->d, 1, h->stream);  // (k_lq's first terminal task zeroed the counts)
        hipError_t e = hipMemcpyAsync(h->host_counter + 8 + 4 * par, h->d.counter, 4 * sizeof(int), hipMemcpyDeviceToHost,
                               h->stream);
        hipGraph_t graph = nullptr;
        const hipError_t ec = hipStreamEndCapture(h->stream, &graph);
        if (e == hipSuccess) e = ec;
        if (e == hipSuccess) e = hipGraphInstantiate(&g.exec, graph, nullptr, nullptr, 0);
        if (graph) hipGraphDestroy(graph);
        if (e != hipSuccess) {
            g.exec = nullptr;
            return fail(HSDDP_ERR_DEVICE, std::string("iteration graph: ") + hipGetErrorString(e));
        }
        std::memcpy(&g.p, &pl, sizeof(Params));
        std::memcpy(&g.d, &h->d, sizeof(Bufs));
        g.alpha = h->opt.alpha;
        g.par = par;
        hit = &g;
    }
    if (!h->iter_done[par]) HIPCHK(hipEventCreateWithFlags(&h->iter_done[par], hipEventDisableTiming));
    HIPCHK(hipGraphLaunch(hit->exec, h->stream));
    HIPCHK(hipEventRecord(h->iter_done[par], h->stream));
    h->slots_fresh = true;
    return HSDDP_OK;
}

static int graph_wait(hsddp_handle h, int par, int &n_active)
{
    HIPCHK(hipEventSynchronize(h->iter_done[par]));
    n_active = h->host_counter[8 + 4 * par + 1];
    return HSDDP_OK;
}

static void outer_end_launches(hsddp_handle h, Timer &tm)
{
    hipEvent_t e0;
    tm.begin(3, e0);
    // update_REB_params moves per-knot (delta, eps) unless they stay uniform: the running costs change
    if (h->opt.ReB_active && !h->p.reb_uniform) {
        h->slots_fresh = false;
        h->reb_at_init = false;
    }
    if (h->opt.ReB_active) launch_reb_update(h->p, h->d, h->stream);
    launch_outer_end(h->p, h->d, h->stream);
    tm.end(3, e0);
}

static int finish_stats(hsddp_handle h, Timer &tm, hipEvent_t e0, hsddp_stats *stats, int iters, int outers, int nbwd)
{
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(h->stream));
    if (!stats) return HSDDP_OK;
    hipEvent_t e1;
    hipEventCreate(&e1);
    hipEventRecord(e1, h->stream);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
    stats->ms_total = ms;
    stats->ms_lq = tm.total(0);
    stats->ms_backward = tm.total(1);
    stats->ms_forward = tm.total(2);
    stats->ms_other = tm.total(3);
    stats->ms_linear = tm.total(4);
    stats->inner_iterations = iters;
    stats->outer_iterations = outers;
    stats->n_backward_launches = nbwd;
    // the two sums on the device (a copy of every element's state would be ~0.6 MB per call)
    HIPCHK(hipMemsetAsync(h->d.counter + 4, 0, 2 * sizeof(int), h->stream));
    launch_stat_sums(h->p, h->d, h->stream);
    HIPCHK(hipMemcpyAsync(h->host_counter + 4, h->d.counter + 4, 2 * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    stats->ls_trials = h->host_counter[4];
    stats->element_iterations = h->host_counter[5];
    return HSDDP_OK;
}

static hipEvent_t start_stats(hsddp_handle h, hsddp_stats *stats)
{
    if (!stats) return nullptr;
    memset(stats, 0, sizeof(*stats));
    hipEvent_t e0;
    hipEventCreate(&e0);
    hipEventRecord(e0, h->stream);
    return e0;
}

extern "C" int hsddp_solve(hsddp_handle h, hsddp_stats *stats)
{
    int rc = solve_check(h);
    if (rc) return rc;
    Timer tm{h->stream, stats != nullptr, &h->events};
    hipEvent_t e0 = start_stats(h, stats);
    const std::vector<double> trials = ls_steps(h->opt.alpha);
    begin_launches(h);
    int iters = 0, outers = 0, nbwd = 0;
    const bool checks = !h->opt.no_early_exit;
    const bool graph = checks && graphs_enabled();
    for (int ou = 0; ou < h->opt.max_AL_iter; ++ou) {
        tm.cut();
        launch_outer_begin(h->p, h->d, h->stream);
        outers++;
        for (int in = 0; in < h->opt.max_DDP_iter; ++in) {
            if (graph) {
                // iteration `in` was launched by the step before (or here, for the first); the next
                // one is queued before waiting for this one's count, so the GPU never waits on the
                // host's round trip.  When the count comes back 0 the queued iteration finds every
                // element inner_done / done and returns at once (the kernels' own early exits), as
                // the reference's loop would not have run it; it is never queued past max_DDP_iter.
                int n = 0;
                tm.cut();
                if (in == 0 && (rc = graph_launch(h, trials, 0))) return rc;
                if (in + 1 < h->opt.max_DDP_iter && (rc = graph_launch(h, trials, (in + 1) & 1))) return rc;
                if ((rc = graph_wait(h, in & 1, n))) return rc;
                iters++;
                nbwd++;
                if (n == 0) break;
                continue;
            }
            iteration_launches(h, trials, tm);
            iters++;
            nbwd++;
            if (checks) {
                int n = 0;
                tm.cut();
                if ((rc = count_active(h, 1, n))) return rc;
                if (n == 0) break;
            }
        }
        outer_end_launches(h, tm);
        if (checks) {
            int n = 0;
            tm.cut();
            if ((rc = count_active(h, 2, n))) return rc;
            if (n == 0) break;
        }
    }
    return finish_stats(h, tm, e0, stats, iters, outers, nbwd);
}

extern "C" int hsddp_solve_begin(hsddp_handle h)
{
    int rc = solve_check(h);
    if (rc) return rc;
    begin_launches(h);
    launch_outer_begin(h->p, h->d, h->stream);
    HIPCHK(hipGetLastError());
    return HSDDP_OK;
}

extern "C" int hsddp_iterate(hsddp_handle h, int n, hsddp_stats *stats)
{
    int rc = solve_check(h);
    if (rc) return rc;
    if (n < 0) return fail(HSDDP_ERR_ARG, "negative iteration count");
    Timer tm{h->stream, stats != nullptr, &h->events};
    hipEvent_t e0 = start_stats(h, stats);
    const std::vector<double> trials = ls_steps(h->opt.alpha);
    sync_ref_columns(h);  // (references uploaded after hsddp_solve_begin)
    for (int i = 0; i < n; ++i) iteration_launches(h, trials, tm);
    return finish_stats(h, tm, e0, stats, n, 0, n);
}

extern "C" int hsddp_solve_end(hsddp_handle h)
{
    int rc = solve_check(h);
    if (rc) return rc;
    Timer tm{h->stream, false, &h->events};
    outer_end_launches(h, tm);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(h->stream));
    return HSDDP_OK;
}

static int d2h(void *dst, const void *src, size_t bytes)
{
    if (!dst) return HSDDP_OK;
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return HSDDP_OK;
}

extern "C" int hsddp_download_trajectory(hsddp_handle h, double *Xbar, double *Ubar, double *K)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const size_t B = h->p.B, S = h->p.S, Kc = h->p.Kc;
    int rc;
    launch_normalize(h->p, h->d, h->stream);  // nominal rows in buffer 0
    HIPCHK(hipStreamSynchronize(h->stream));
    if ((rc = d2h(Xbar, h->d.X3, B * S * NX * 8)) || (rc = d2h(Ubar, h->d.U3, B * Kc * NX * 8)))
        return rc;
    if (K && h->need_inputs)
        return fail(HSDDP_ERR_ARG, "the layout changed (hsddp_shift): call hsddp_update_problem before downloading K");
    if (K) { // expand the coupled rows; the decoupled controls' rows are exactly zero
        std::vector<double> kc(B * Kc * KCW);
        if (h->p.fp32) {
            std::vector<float> k32(B * Kc * KCW);
            if ((rc = d2h(k32.data(), h->d.K32, B * Kc * KCW * 4))) return rc;
            std::copy(k32.begin(), k32.end(), kc.begin());
        } else if ((rc = d2h(kc.data(), h->d.K, B * Kc * KCW * 8))) {
            return rc;
        }
        std::memset(K, 0, B * Kc * NN * sizeof(double));
        for (size_t b = 0; b < B; ++b)
            for (size_t k = 0; k < Kc; ++k)
                for (int q = 0; q < 12; ++q) {
                    const int u = coupled_control(h, b, k, q);
                    std::memcpy(K + ((b * Kc + k) * NX + u) * NX, &kc[((b * Kc + k) * 12 + q) * NX], NX * sizeof(double));
                }
    }
    return HSDDP_OK;
}

// diagnostic builds (-DHSDDP_STAMPS=1): per-element in-kernel stamp sums [B][16]; not in hsddp.h
extern "C" int hsddp_debug_stamps(hsddp_handle h, unsigned long long *out)
{
    if (!h || !out) return fail(HSDDP_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    HIPCHK(hipMemcpy(out, h->d.dbg, h->p.B * 16 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return HSDDP_OK;
}

extern "C" int hsddp_download_working(hsddp_handle h, double *X, double *U, double *Defect, double *dX, double *dU)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const size_t B = h->p.B, S = h->p.S, Kc = h->p.Kc;
    int rc;
    if ((rc = d2h(dX, h->d.dX, B * S * NX * 8)) || (rc = d2h(dU, h->d.dU, B * Kc * NX * 8)))
        return rc;
    if (X || U || Defect) {  // each element's working rows from the buffer sel names
        std::vector<int> sel(B);
        HIPCHK(hipMemcpy(sel.data(), h->d.sel, B * sizeof(int), hipMemcpyDeviceToHost));
        for (int q = 0; q < 3; ++q) {
            std::vector<double> xb(X ? B * S * NX : 0), ub(U ? B * Kc * NX : 0), db(Defect ? B * S * NX : 0);
            if ((rc = d2h(X ? xb.data() : nullptr, h->d.X3 + q * h->d.xs3, B * S * NX * 8)) ||
                (rc = d2h(U ? ub.data() : nullptr, h->d.U3 + q * h->d.us3, B * Kc * NX * 8)) ||
                (rc = d2h(Defect ? db.data() : nullptr, h->d.D3 + q * h->d.xs3, B * S * NX * 8)))
                return rc;
            for (size_t b = 0; b < B; ++b) {
                if (((sel[b] >> 2) & 3) != q) continue;
                if (X) std::copy(xb.begin() + b * S * NX, xb.begin() + (b + 1) * S * NX, X + b * S * NX);
                if (U) std::copy(ub.begin() + b * Kc * NX, ub.begin() + (b + 1) * Kc * NX, U + b * Kc * NX);
                if (Defect) std::copy(db.begin() + b * S * NX, db.begin() + (b + 1) * S * NX, Defect + b * S * NX);
            }
        }
    }
    return HSDDP_OK;
}

extern "C" int hsddp_download_references(hsddp_handle h, double *ref_x, double *ref_u, double *ref_foot)
{
    if (!h || !ref_x || !ref_u || !ref_foot) return fail(HSDDP_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const size_t Br = h->Bref, S = h->p.S;
    int rc;
    if ((rc = d2h(ref_x, h->d.ref_x, Br * S * NX * 8)) || (rc = d2h(ref_u, h->d.ref_u, Br * S * NX * 8)) ||
        (rc = d2h(ref_foot, h->d.ref_foot, Br * S * 12 * 8)))
        return rc;
    return HSDDP_OK;
}

extern "C" int hsddp_download_element_info(hsddp_handle h, hsddp_element_info *info)
{
    if (!h || !info) return fail(HSDDP_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    std::vector<ElemState> el(h->p.B);
    HIPCHK(hipMemcpy(el.data(), h->d.el, h->p.B * sizeof(ElemState), hipMemcpyDeviceToHost));
    for (int b = 0; b < h->p.B; ++b) {
        const ElemState &e = el[b];
        info[b].cost = e.cost; info[b].feas = e.feas; info[b].merit = e.merit;
        info[b].max_tconstr = e.max_t; info[b].max_pconstr = e.max_p;
        info[b].iters = e.iters; info[b].outer_iters = e.outer_iters; info[b].status = e.status;
        info[b].n_ls_trials = e.n_ls;
    }
    return HSDDP_OK;
}

extern "C" int hsddp_download_solver_info(hsddp_handle h, int capacity, float *cost, float *dyn_feas,
                                          float *eqn_feas, float *ineq_feas, int *count)
{
    if (!h || capacity < 0) return fail(HSDDP_ERR_ARG, "null handle or negative capacity");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const int B = h->p.B, hc = h->p.hcap;
    std::vector<ElemState> el(B);
    HIPCHK(hipMemcpy(el.data(), h->d.el, B * sizeof(ElemState), hipMemcpyDeviceToHost));
    std::vector<float> hv((size_t)B * hc * 4);
    HIPCHK(hipMemcpy(hv.data(), h->d.hist, hv.size() * sizeof(float), hipMemcpyDeviceToHost));
    float *outs[4] = {cost, dyn_feas, eqn_feas, ineq_feas};
    for (int b = 0; b < B; ++b) {
        const int n = std::min(el[b].hist_n, std::min(hc, capacity));
        if (count) count[b] = n;
        for (int f = 0; f < 4; ++f) {
            if (!outs[f]) continue;
            float *o = outs[f] + (size_t)b * capacity;
            for (int k = 0; k < capacity; ++k) o[k] = k < n ? hv[((size_t)b * hc + k) * 4 + f] : 0.0f;
        }
    }
    return HSDDP_OK;
}

// ---- the reference Trajectory's derived fields (TrajectoryManagement.h:49-81) ---------------
// The device keeps the LQ model of a knot in the compact record (hsddp_internal.h); these host
// routines expand it to the reference's dense blocks for callers that read them.


extern "C" int hsddp_download_lq(hsddp_handle h, double *A, double *Bm, double *l, double *lx, double *lu,
                                 double *lxx, double *luu)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const Params &p = h->p;
    const size_t B = p.B, Kc = p.Kc, S = p.S, W = p.fp32 ? LQW32 : LQW;
    std::vector<double> rec(B * Kc * W), cost(B * S);
    if (p.fp32) {
        std::vector<float> r32(B * Kc * W);
        HIPCHK(hipMemcpy(r32.data(), h->d.lq32, r32.size() * sizeof(float), hipMemcpyDeviceToHost));
        for (size_t q = 0; q < rec.size(); ++q) rec[q] = r32[q];
    } else {
        HIPCHK(hipMemcpy(rec.data(), h->d.lq, rec.size() * sizeof(double), hipMemcpyDeviceToHost));
    }
    if (l) HIPCHK(hipMemcpy(cost.data(), h->d.slot_cost, cost.size() * sizeof(double), hipMemcpyDeviceToHost));
    const double dt = p.dt;
    for (size_t b = 0; b < B; ++b)
        for (size_t kc = 0; kc < Kc; ++kc) {
            const double *r = rec.data() + (b * Kc + kc) * W;
            const int i = phase_of_control(layout_of(h, b), (int)kc);
            const int *c = h->contacts.data() + (b * (p.P + 1) + i) * 4;
            const size_t o = (b * Kc + kc);
            if (A) {  // A = I + S (hkd_model.h: Se, Sw, dt at (3 + a, 9 + a))
                double *a = A + o * NN;
                std::fill(a, a + NN, 0.0);
                for (int j = 0; j < NX; ++j) a[j * NX + j] = 1.0;
                for (int rr = 0; rr < 3; ++rr)
                    for (int q = 0; q < 5; ++q) a[rr * NX + hkd::se_col(q)] += r[LQ_SE + 5 * rr + q];
                for (int q = 0; q < 3; ++q) a[(3 + q) * NX + 9 + q] += dt;
                for (int rr = 0; rr < 3; ++rr)
                    for (int q = 0; q < 17; ++q) a[(6 + rr) * NX + hkd::sw_col(q)] += r[sw_at(rr, q)];
            }
            if (Bm) {
                double *bb = Bm + o * NN;
                std::fill(bb, bb + NN, 0.0);
                for (int rr = 0; rr < 3; ++rr)
                    for (int q = 0; q < 12; ++q) bb[(6 + rr) * NX + q] = r[bw_at(rr, q)];
                for (int lg = 0; lg < 4; ++lg)
                    for (int a = 0; a < 3; ++a) {
                        bb[(9 + a) * NX + 3 * lg + a] = dt * c[lg] / hkd::kMass;
                        bb[(12 + 3 * lg + a) * NX + 12 + 3 * lg + a] = dt * (1.0 - c[lg]);
                    }
            }
            if (l) l[o] = cost[b * S + kc + i];
            if (lx) for (int j = 0; j < NX; ++j) lx[o * NX + j] = r[LQ_LX + j];
            if (lu) for (int j = 0; j < NX; ++j) lu[o * NX + j] = r[LQ_LU + j];
            if (lxx) {  // dt Q + dt D^T Qfoot D (HKDCost.cpp:22-37; constant per phase)
                double *m = lxx + o * NN;
                std::fill(m, m + NN, 0.0);
                for (int j = 0; j < NX; ++j)
                    m[j * NX + j] = dt * (j < 12 ? p.qbase[j] : p.q_qJ * (1 - c[(j - 12) / 3]));
                for (int lg = 0; lg < 4; ++lg)
                    for (int a = 0; a < 3; ++a) {
                        const double w = c[lg] ? dt * (p.foot_gain * p.foot_w[a]) : 0.0;
                        const int pa = 3 + a, qa = 12 + 3 * lg + a;
                        m[pa * NX + pa] += w; m[qa * NX + qa] += w;
                        m[pa * NX + qa] -= w; m[qa * NX + pa] -= w;
                    }
            }
            if (luu) {  // dt R + dt ReB Hessian of the stance legs' GRF rows (SinglePhase.cpp:380-394)
                double *m = luu + o * NN;
                std::fill(m, m + NN, 0.0);
                for (int j = 0; j < NX; ++j) m[j * NX + j] = dt * (j < 12 ? p.r_grf : p.r_qJd);
                static const int ix[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
                for (int lg = 0; lg < 4; ++lg)
                    for (int a = 0; a < 3; ++a)
                        for (int e = 0; e < 3; ++e) m[(3 * lg + a) * NX + 3 * lg + e] += r[LQ_RB + 6 * lg + ix[a][e]];
            }
        }
    return HSDDP_OK;
}

extern "C" int hsddp_download_terminal(hsddp_handle h, double *Phi, double *Phix, double *Phixx, double *Px)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const Params &p = h->p;
    const size_t B = p.B, P = p.P;
    std::vector<double> term(B * P * TW), cost(B * p.S);
    HIPCHK(hipMemcpy(term.data(), h->d.term, term.size() * sizeof(double), hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(cost.data(), h->d.slot_cost, cost.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (size_t b = 0; b < B; ++b) {
        const Layout L = layout_of(h, b);
        for (size_t i = 0; i < P; ++i) {
            const double *t = term.data() + (b * P + i) * TW;
            const size_t o = b * P + i;
            if ((int)i >= L.P) {  // past this element's phases
                if (Phi) Phi[o] = 0;
                if (Phix) std::fill(Phix + o * NX, Phix + (o + 1) * NX, 0.0);
                if (Phixx) std::fill(Phixx + o * NN, Phixx + (o + 1) * NN, 0.0);
                if (Px) std::fill(Px + o * NN, Px + (o + 1) * NN, 0.0);
                continue;
            }
            if (Phi) Phi[o] = cost[b * p.S + L.s0[i] + L.N[i]];
            if (Phix) std::copy(t + TM_PHIX, t + TM_PHIX + NX, Phix + o * NX);
            if (Phixx) std::copy(t + TM_PHIXX, t + TM_PHIXX + NN, Phixx + o * NN);
            if (Px) {
                if ((int)i + 1 < L.P) std::copy(t + TM_PX, t + TM_PX + NN, Px + o * NN);
                else std::fill(Px + o * NN, Px + (o + 1) * NN, 0.0);  // no reset after the last phase
            }
        }
    }
    return HSDDP_OK;
}

extern "C" int hsddp_set_value_export(hsddp_handle h, int on)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    HIPCHK(hipSetDevice(h->desc.device));
    if (on && !h->value0) {
        const size_t n = (size_t)h->p.B * HSDDP_MAX_PHASES * (NX + NN);
        HIPCHK(hipMalloc(&h->value0, n * sizeof(double)));
        HIPCHK(hipMemset(h->value0, 0, n * sizeof(double)));
        HIPCHK(hipStreamSynchronize(nullptr));
        h->bytes += n * sizeof(double);
        h->d.value0 = h->value0;
    }
    h->p.store_value = on ? 1 : 0;
    fill_params(h);
    return HSDDP_OK;
}

extern "C" int hsddp_download_value(hsddp_handle h, double *G, double *H)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    if (!h->value0 || !h->p.store_value) return fail(HSDDP_ERR_ARG, "value export is off (hsddp_set_value_export)");
    HIPCHK(hipSetDevice(h->desc.device));
    HIPCHK(hipStreamSynchronize(h->stream));
    const size_t B = h->p.B, P = h->p.P;
    std::vector<double> v(B * P * (NX + NN));
    HIPCHK(hipMemcpy(v.data(), h->value0, v.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (size_t o = 0; o < B * P; ++o) {
        // phases past the element's own layout (per-element layouts, or left from before a shift) are zero
        const bool live = (int)(o % P) < layout_of(h, o / P).P;
        const double *s = v.data() + o * (NX + NN);
        if (G) { if (live) std::copy(s, s + NX, G + o * NX); else std::fill(G + o * NX, G + (o + 1) * NX, 0.0); }
        if (H) { if (live) std::copy(s + NX, s + NX + NN, H + o * NN); else std::fill(H + o * NN, H + (o + 1) * NN, 0.0); }
    }
    return HSDDP_OK;
}

extern "C" int hsddp_synchronize(hsddp_handle h)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    HIPCHK(hipStreamSynchronize(h->stream));
    return HSDDP_OK;
}

extern "C" size_t hsddp_device_bytes(hsddp_handle h) { return h ? h->bytes : 0; }

// ---- model primitives ------------------------------------------------------------------------
static int check_launch()
{
    HIPCHK(hipGetLastError());
    return HSDDP_OK;
}

extern "C" int hsddp_hkd_dynamics(const double *x, const double *u, const double *c, double dt, double *xn, int n,
                                  void *stream)
{
    if (!x || !u || !c || !xn || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_dynamics(x, u, c, dt, xn, n, (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_dynamics_partial(const double *x, const double *u, const double *c, double dt, double *A,
                                          double *B, int n, void *stream)
{
    if (!x || !u || !c || !A || !B || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_partial(x, u, c, dt, A, B, n, (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_foot_position(const double *x, const int *leg, double *p, int n, void *stream)
{
    if (!x || !leg || !p || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_foot(x, leg, p, nullptr, n, (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_foot_jacobian(const double *x, const int *leg, double *J, int n, void *stream)
{
    if (!x || !leg || !J || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_foot(x, leg, nullptr, J, n, (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_resetmap(const double *x, const int *c, const int *cn, double *xn, int n, void *stream)
{
    if (!x || !c || !cn || !xn || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_reset(x, c, cn, xn, nullptr, n, (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_resetmap_partial(const double *x, const int *c, const int *cn, double *Px, int n,
                                          void *stream)
{
    if (!x || !c || !cn || !Px || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_reset(x, c, cn, nullptr, Px, n, (hipStream_t)stream);
    return check_launch();
}

// weights / dt of a plugin primitive in the solver's parameter block (the kernels share the
// solver's cost helpers)
static Params plugin_params(const hsddp_hkd_weights &w, double dt)
{
    Params p{};
    p.dt = dt;
    for (int j = 0; j < 3; ++j) { p.qbase[j] = w.q_eul[j]; p.qbase[3 + j] = w.q_pos[j]; p.qbase[6 + j] = w.q_omega[j]; p.qbase[9 + j] = w.q_v[j]; }
    p.q_qJ = w.q_qJ;
    for (int j = 0; j < 24; ++j) p.qf_scale[j] = w.qf_scale[j];
    p.qf_gain = w.qf_gain; p.r_grf = w.r_grf; p.r_qJd = w.r_qJd;
    for (int j = 0; j < 3; ++j) p.foot_w[j] = w.foot_w[j];
    p.foot_gain = w.foot_gain; p.foot_term_cost = w.foot_term_cost; p.foot_term_grad = w.foot_term_grad;
    return p;
}
extern "C" int hsddp_hkd_running_cost(const double *x, const double *u, const int *c, const double *xr, const double *ur,
                                      const double *pf, const hsddp_hkd_weights *w, double dt, int terms, double *l,
                                      double *lx, double *lu, double *lxx, double *luu, int n, void *stream)
{
    if (!x || !u || !c || !xr || !ur || !pf || !w || n < 0 || (terms & ~3)) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_running_cost(plugin_params(*w, dt), x, u, c, xr, ur, pf, terms, l, lx, lu, lxx, luu, n,
                                     (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_terminal_cost(const double *x, const int *c, const double *xr, const double *pf,
                                       const hsddp_hkd_weights *w, int terms, double *Phi, double *Phix, double *Phixx,
                                       int n, void *stream)
{
    if (!x || !c || !xr || !pf || !w || n < 0 || (terms & ~3)) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_terminal_cost(plugin_params(*w, 0.0), x, c, xr, pf, terms, Phi, Phix, Phixx, n,
                                      (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_grf_constraint(const double *u, const int *c, double mu, double *g, double *gu, int n,
                                        void *stream)
{
    if (!u || !c || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_grf(u, c, mu, g, gu, n, (hipStream_t)stream);
    return check_launch();
}
extern "C" int hsddp_hkd_touchdown_constraint(const double *x, const int *c, const int *cn, double ground, double *h,
                                              double *hx, int n, void *stream)
{
    if (!x || !c || !cn || n < 0) return fail(HSDDP_ERR_ARG, "bad argument");
    if (n) launch_model_touchdown(x, c, cn, ground, h, hx, n, (hipStream_t)stream);
    return check_launch();
}

extern "C" void *hsddp_device_alloc(size_t bytes, int device)
{
    if (hipSetDevice(device) != hipSuccess) { g_err = "hipSetDevice failed"; return nullptr; }
    void *p = nullptr;
    if (hipMalloc(&p, bytes ? bytes : 16) != hipSuccess) { g_err = "hipMalloc failed"; return nullptr; }
    return p;
}
extern "C" int hsddp_device_free(void *p)
{
    HIPCHK(hipFree(p));
    return HSDDP_OK;
}
extern "C" int hsddp_memcpy_h2d(void *dst, const void *src, size_t bytes)
{
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return HSDDP_OK;
}
extern "C" int hsddp_memcpy_d2h(void *dst, const void *src, size_t bytes)
{
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return HSDDP_OK;
}
extern "C" int hsddp_device_synchronize(int device)
{
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipDeviceSynchronize());
    return HSDDP_OK;
}

// ---- MPC command extraction (HKDMPCSolver::update_foot_placement + publish_mpc_cmd) ----------
static int extract_commands(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                            const double *status_durations, int durations_per_element, const float *foot_placements,
                            int feet_per_element, float solve_time, hsddp_mpc_command *out, bool out_on_device,
                            int ticket = -1);

extern "C" int hsddp_extract_commands(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                                      const double *status_durations, int durations_per_element,
                                      const float *foot_placements, int feet_per_element, float solve_time,
                                      hsddp_mpc_command *out)
{
    return extract_commands(h, nsteps_between_mpc, mpc_time, dt_mpc, status_durations, durations_per_element,
                            foot_placements, feet_per_element, solve_time, out, false);
}

extern "C" int hsddp_extract_commands_device(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                                             const double *status_durations, int durations_per_element,
                                             const float *foot_placements, int feet_per_element, float solve_time,
                                             void *out_device)
{
    return extract_commands(h, nsteps_between_mpc, mpc_time, dt_mpc, status_durations, durations_per_element,
                            foot_placements, feet_per_element, solve_time, (hsddp_mpc_command *)out_device, true);
}

// ticket >= 0 (asynchronous form): the records go to device buffer `ticket` and from there to its
// pinned host buffer on the copy stream; out is unused
static int extract_commands(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                            const double *status_durations, int durations_per_element, const float *foot_placements,
                            int feet_per_element, float solve_time, hsddp_mpc_command *out, bool out_on_device,
                            int ticket)
{
    if (!h || (!out && ticket < 0)) return fail(HSDDP_ERR_ARG, "null argument");
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    const Params &p = h->p;
    CmdArgs a{};
    a.n = nsteps_between_mpc + 7;  // HKDMPC.cpp:232-233
    if (nsteps_between_mpc < 1 || a.n > HSDDP_CMD_STEPS || a.n > p.Kc)
        return fail(HSDDP_ERR_ARG, "nsteps_between_mpc + 7 must fit the command (10 rows) and the horizon");
    // the knot walk of publish_mpc_cmd (HKDMPC.cpp:239-246): s runs over phase i's controls (per-
    // element layouts: each workgroup walks its element's own)
    if (h->lays.empty())
        for (int k = 0, i = 0, s = 0; k < a.n; ++k, ++s) {
            if (s >= p.N[i]) { s = 0; ++i; }
            a.kc[k] = p.k0[i] + s;
            a.xs[k] = p.s0[i] + s;
            a.ph[k] = i;
        }
    a.mpc_time = mpc_time;
    a.dt_mpc = dt_mpc;
    a.solve_time = solve_time;
    a.dur_per_elem = durations_per_element ? 1 : 0;
    a.feet_per_elem = feet_per_element ? 1 : 0;
    HIPCHK(hipSetDevice(h->desc.device));
    const size_t B = p.B;
    const size_t cmd_bytes = (B * sizeof(hsddp_mpc_command) + 255) / 256 * 256;
    const size_t dur_bytes = status_durations ? ((a.dur_per_elem ? B : 1) * p.P * 4 * sizeof(double) + 255) / 256 * 256 : 0;
    const size_t feet_bytes = foot_placements ? (a.feet_per_elem ? B : 1) * 12 * sizeof(float) : 0;
    char *buf;
    int rc;
    if ((rc = scratch(h, cmd_bytes + dur_bytes + feet_bytes, &buf))) return rc;
    hsddp_mpc_command *dcmd = ticket >= 0 ? h->cmd_dev[ticket] : out_on_device ? out : (hsddp_mpc_command *)buf;
    const size_t dur_len = (a.dur_per_elem ? B : 1) * p.P * 4 * sizeof(double);
    const void *dur_src = status_durations, *feet_src = foot_placements;
    if (ticket >= 0 && (status_durations || foot_placements)) {
        // the call returns before the kernel runs and the caller may release its (pageable) inputs:
        // they are copied into this ticket's pinned staging first, and the H2D copies read from
        // there — nothing waits for the handle's stream.  The staging's previous copies (two
        // extractions ago) finished before that extraction's kernel, whose event is long past.
        char *&pin = h->cmd_in_host[ticket];
        if (h->cmd_in_bytes[ticket] < dur_bytes + feet_bytes) {
            HIPCHK(hipEventSynchronize(h->cmd_ready[ticket]));
            if (pin) hipHostFree(pin);
            pin = nullptr;
            h->cmd_in_bytes[ticket] = 0;
            HIPCHK(hipHostMalloc((void **)&pin, dur_bytes + feet_bytes, 0));
            h->cmd_in_bytes[ticket] = dur_bytes + feet_bytes;
        } else {
            HIPCHK(hipEventSynchronize(h->cmd_ready[ticket]));
        }
        if (status_durations) std::memcpy(pin, status_durations, dur_len);
        if (foot_placements) std::memcpy(pin + dur_bytes, foot_placements, feet_bytes);
        dur_src = pin;
        feet_src = pin + dur_bytes;
    }
    if (status_durations) {
        a.durations = (const double *)(buf + cmd_bytes);
        if ((rc = h2d((void *)a.durations, dur_src, dur_len, h->stream))) return rc;
    }
    if (foot_placements) {
        a.feet = (const float *)(buf + cmd_bytes + dur_bytes);
        if ((rc = h2d((void *)a.feet, feet_src, feet_bytes, h->stream))) return rc;
    }
    if (ticket >= 0)  // the buffer's previous copy (two extractions ago) has left it
        HIPCHK(hipStreamWaitEvent(h->stream, h->cmd_copied[ticket], 0));
    launch_extract_commands(p, h->d, a, dcmd, h->stream);
    HIPCHK(hipGetLastError());
    if (ticket >= 0) {  // D2H on the copy stream, behind the kernel: the handle's stream moves on
        HIPCHK(hipEventRecord(h->cmd_ready[ticket], h->stream));
        HIPCHK(hipStreamWaitEvent(h->copy_stream, h->cmd_ready[ticket], 0));
        HIPCHK(hipMemcpyAsync(h->cmd_host[ticket], dcmd, B * sizeof(hsddp_mpc_command), hipMemcpyDeviceToHost,
                              h->copy_stream));
        HIPCHK(hipEventRecord(h->cmd_copied[ticket], h->copy_stream));
        return HSDDP_OK;
    }
    if (!out_on_device) HIPCHK(hipMemcpyAsync(out, dcmd, B * sizeof(hsddp_mpc_command), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(hipStreamSynchronize(h->stream));
    return HSDDP_OK;
}

extern "C" int hsddp_extract_commands_async(hsddp_handle h, int nsteps_between_mpc, double mpc_time, double dt_mpc,
                                            const double *status_durations, int durations_per_element,
                                            const float *foot_placements, int feet_per_element, float solve_time,
                                            int *ticket)
{
    if (!h || !ticket) return fail(HSDDP_ERR_ARG, "null argument");
    HIPCHK(hipSetDevice(h->desc.device));
    const size_t bytes = (size_t)h->p.B * sizeof(hsddp_mpc_command);
    if (!h->copy_stream) {  // first use: two record buffers on each side, the copy stream, events
        HIPCHK(hipStreamCreateWithFlags(&h->copy_stream, hipStreamNonBlocking));
        for (int q = 0; q < 2; ++q) {
            HIPCHK(hipMalloc((void **)&h->cmd_dev[q], bytes));
            HIPCHK(hipHostMalloc((void **)&h->cmd_host[q], bytes, 0));
            HIPCHK(hipEventCreateWithFlags(&h->cmd_ready[q], hipEventDisableTiming));
            HIPCHK(hipEventCreateWithFlags(&h->cmd_copied[q], hipEventDisableTiming));
            HIPCHK(hipEventRecord(h->cmd_copied[q], h->copy_stream));
        }
    }
    const int t = h->cmd_next;
    const int rc = extract_commands(h, nsteps_between_mpc, mpc_time, dt_mpc, status_durations, durations_per_element,
                                    foot_placements, feet_per_element, solve_time, nullptr, false, t);
    if (rc) return rc;
    h->cmd_next ^= 1;
    *ticket = t;
    return HSDDP_OK;
}

extern "C" int hsddp_commands_wait(hsddp_handle h, int ticket, const hsddp_mpc_command **records)
{
    if (!h || !records) return fail(HSDDP_ERR_ARG, "null argument");
    if (ticket < 0 || ticket > 1 || !h->copy_stream) return fail(HSDDP_ERR_ARG, "no such extraction ticket");
    HIPCHK(hipEventSynchronize(h->cmd_copied[ticket]));
    *records = h->cmd_host[ticket];
    return HSDDP_OK;
}

// ---- receding-horizon shift (HKDProblem::update, HKDProblem.cpp:117-222) ----------------------
namespace {
// one phase of the layout being shifted; slot labels name where each value comes from:
// state  >= 0: old Xbar slot, -1: zero, <= -2: old (working) X slot -2 - label;
// control >= 0: old control slot (Ubar and K), -1: zero
struct ShiftPhase {
    int N, ss, reach;
    std::vector<int> xs, us;
    int src = -1;         // the old phase it continues (-1: added by this shift)
    int add = 0;          // touchdown constraints appended by this shift (add_tconstr_one_phase)
    std::vector<int> rs;  // per control slot: the old slot its ReB parameters come from (-1: initial)
};
}  // namespace

// HKDProblem::update's phase bookkeeping (HKDProblem.cpp:117-222) of one layout for n_steps steps,
// step j with contact-change flag cc[j * cstride]: the phases afterwards, each with the old slots
// its new slots come from (labels: >= 0 old slot, -2 - s old X row s, -1 zero)
static int shift_phases(const Layout &L, const int *reach, int n_steps, const int *cc, size_t cstride,
                        std::vector<ShiftPhase> &ph)
{
    ph.assign(L.P, ShiftPhase{});
    for (int i = 0; i < L.P; ++i) {
        ph[i].N = L.N[i]; ph[i].ss = L.ss[i]; ph[i].reach = reach[i];
        ph[i].src = i;
        for (int k = 0; k <= L.N[i]; ++k) ph[i].xs.push_back(L.s0[i] + k);
        for (int k = 0; k < L.N[i]; ++k) ph[i].us.push_back(L.k0[i] + k);
        ph[i].rs = ph[i].us;
    }
    for (int j = 0; j < n_steps; ++j) {
        const int change = cc[(size_t)j * cstride];
        // front: a first phase of one knot shrinks to a point and is removed (pop_front_phase,
        // HKDProblem.h:56-66); otherwise its first knot is dropped (SinglePhase::pop_front,
        // SinglePhase.cpp:496-501)
        if (ph.front().N <= 1) {
            if (ph.size() == 1) return fail(HSDDP_ERR_ARG, "shift would remove the only phase");
            ph.erase(ph.begin());
        } else {
            ShiftPhase &f = ph.front();
            f.xs.erase(f.xs.begin());
            f.us.erase(f.us.begin());
            f.rs.erase(f.rs.begin());
            f.N--;
        }
        // back: a contact change after the last phase reached its end starts a new phase of one
        // knot with a zero trajectory (Trajectory::create_data); otherwise the last phase grows by
        // push_back_default: X.back() copied into X and Xbar, zero control and gain
        // (SinglePhase.cpp:485-490, TrajectoryManagement.cpp:163-190)
        ShiftPhase &l = ph.back();
        if (change && l.reach) {
            if ((int)ph.size() >= HSDDP_MAX_PHASES) return fail(HSDDP_ERR_ARG, "shift exceeds HSDDP_MAX_PHASES phases");
            ShiftPhase n;
            n.N = 1; n.ss = 0; n.reach = 0;
            n.xs = {-1, -1};
            n.us = {-1};
            n.rs = {-1};  // a new GRF constraint: initial ReB parameters (HKDProblem.cpp:255-263)
            ph.push_back(n);
        } else {
            const int last = l.xs.back();
            l.xs.push_back(last >= 0 ? -2 - last : last);
            l.us.push_back(-1);
            l.rs.push_back(l.rs.back());  // PathConstraintBase::push_back copies params.back()
            l.N++;
            if (change) l.reach = 1;
        }
        // add_tconstr_one_phase on a last phase that has reached its end, at every step
        // (HKDProblem.cpp:199-202): one more touchdown constraint with initial AL parameters
        if (ph.back().reach) ph.back().add++;
    }
    // update_SS_config after the steps (HKDProblem.cpp:203-217): every phase but a last one of
    // horizon <= 2 gets all its states as shooting states
    const int P = (int)ph.size();
    for (int i = 0; i < P; ++i)
        if (i < P - 1 || ph[i].N > 2) ph[i].ss = ph[i].N + 1;
    for (int i = 0; i < P - 1; ++i)
        if (ph[i].ss < ph[i].N + 1) return fail(HSDDP_ERR_UNSUPPORTED, "non-shooting states outside the last phase");
    return HSDDP_OK;
}

// the receding-horizon shift of every element: cc[b * bstride + j * sstride] is element b's flag of
// step j.  Elements with equal (layout, reach flags, step flags) share one slot map; when every
// element ends on one layout the handle keeps (or returns to) the shared layout.  A phase that would
// carry more than HSDDP_MAX_TD touchdown constraints keeps the first ones (the shift is otherwise
// complete): HSDDP_ERR_UNSUPPORTED, or, with `overflow`, *overflow = 1 and HSDDP_OK (hsddp_advance
// finishes the step and reports it then).  defer: no synchronisation (one layout for the batch;
// the flag is read by hsddp_advance).
static int shift_impl(hsddp_handle h, int n_steps, const int *cc, size_t bstride, size_t sstride, bool defer = false,
                      int *overflow = nullptr)
{
    if (!h || (n_steps > 0 && !cc)) return fail(HSDDP_ERR_ARG, "null argument");
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    if (n_steps < 0) return fail(HSDDP_ERR_ARG, "n_steps must be >= 0");
    h->slots_fresh = false;
    Params &p = h->p;
    const size_t B = p.B;
    const bool elem = !h->lays.empty();
    // per unique key: the new phases and slot maps
    std::map<std::vector<int>, int> keys;
    std::vector<std::vector<ShiftPhase>> phs;
    std::vector<int> map_id(B);
    // the handle's shared layout shifted by one set of flags (hsddp_shift): one key for the batch
    // (a per-element key and map lookup cost ≈ 1 µs an element: 4 ms of host time at B = 4096)
    const size_t nkey = (!elem && bstride == 0) ? std::min<size_t>(B, 1) : B;
    for (size_t b = 0; b < nkey; ++b) {
        const Layout L = layout_of(h, b);
        const int *reach = elem ? &h->reach_el[b * HSDDP_MAX_PHASES] : h->reach_end.data();
        std::vector<int> key(L.N, L.N + L.P);
        key.push_back(-1);
        key.insert(key.end(), L.ss, L.ss + L.P);
        key.insert(key.end(), reach, reach + L.P);
        for (int j = 0; j < n_steps; ++j) key.push_back(cc[b * bstride + j * sstride]);
        auto it = keys.find(key);
        if (it == keys.end()) {
            std::vector<ShiftPhase> ph;
            int rc = shift_phases(L, reach, n_steps, cc + b * bstride, sstride, ph);
            if (rc) return rc;
            it = keys.emplace(key, (int)phs.size()).first;
            phs.push_back(ph);
        }
        map_id[b] = it->second;
    }
    const int nk = (int)phs.size();
    if (nk > 1 && h->Bref == 1 && B > 1)  // checked before any device work: the handle stays usable
        return fail(HSDDP_ERR_ARG, "the elements' shifts diverge into per-element layouts, which need per-element "
                                   "references (ref_per_element = 1)");
    std::vector<Layout> nl(nk);
    int Snew = 0, Pnew = 0;
    for (int q = 0; q < nk; ++q) {
        Layout &L = nl[q];
        L = Layout{};
        L.P = (int)phs[q].size();
        int s = 0, k = 0;
        for (int i = 0; i < L.P; ++i) {
            L.N[i] = phs[q][i].N; L.s0[i] = s; L.k0[i] = k; L.ss[i] = phs[q][i].ss;
            s += L.N[i] + 1; k += L.N[i];
            if (L.ss[i] < L.N[i] + 1) L.has_tail = 1;
        }
        L.S = s;
        if (k != p.Kc || (size_t)s > h->S_cap) return fail(HSDDP_ERR_ARG, "shifted layout exceeds the handle's capacity");
        Snew = std::max(Snew, s);
        Pnew = std::max(Pnew, L.P);
    }
    // slot maps [nk][Snew] (padding rows: zero) and [nk][Kc]; constraint-parameter maps: ReB source
    // per control slot [nk][Kc], phase source and appended touchdown constraints [nk][16]
    std::vector<int> smap((size_t)nk * Snew, -1), cmap((size_t)nk * p.Kc), rmap((size_t)nk * p.Kc);
    std::vector<int> pmap((size_t)nk * HSDDP_MAX_PHASES, -1), nadd((size_t)nk * HSDDP_MAX_PHASES, 0);
    for (int q = 0; q < nk; ++q) {
        size_t s = 0, k = 0, r = 0;
        for (size_t i = 0; i < phs[q].size(); ++i) {
            const auto &f = phs[q][i];
            for (int v : f.xs) smap[(size_t)q * Snew + s++] = v;
            for (int v : f.us) cmap[(size_t)q * p.Kc + k++] = v;
            for (int v : f.rs) rmap[(size_t)q * p.Kc + r++] = v;
            pmap[(size_t)q * HSDDP_MAX_PHASES + i] = f.src;
            nadd[(size_t)q * HSDDP_MAX_PHASES + i] = f.add;
        }
    }
    HIPCHK(hipSetDevice(h->desc.device));
    Bufs &d = h->d;
    int rc;
    if (!h->spare_K) {  // (the new Xbar / Ubar rows go to each element's third buffer)
        void *sk;
        if (p.fp32) { float *k32; if ((rc = dalloc(h, k32, B * p.Kc * KCW))) return rc; sk = k32; }
        else { double *k64; if ((rc = dalloc(h, k64, B * p.Kc * KCW))) return rc; sk = k64; }
        h->spare_K = sk;
    }
    if (!h->spare_reb_delta) {
        if ((rc = dalloc(h, h->spare_reb_delta, B * p.Kc * 20)) || (rc = dalloc(h, h->spare_reb_eps, B * p.Kc * 20)) ||
            (rc = dalloc(h, h->spare_al_sigma, B * HSDDP_MAX_PHASES * MTD * 4)) ||
            (rc = dalloc(h, h->spare_al_lambda, B * HSDDP_MAX_PHASES * MTD * 4)) ||
            (rc = dalloc(h, h->spare_td_mask, B * HSDDP_MAX_PHASES * MTD)) ||
            (rc = dalloc(h, h->spare_cf_u, B * p.Kc * 12)) || (rc = dalloc(h, h->spare_cf_flag, B * p.Kc)))
            return rc;
    }
    char *buf;
    const size_t nmaps = smap.size() + cmap.size() + rmap.size() + pmap.size() + nadd.size();
    if ((rc = scratch(h, (nmaps + (nk > 1 ? B : 0)) * sizeof(int), &buf))) return rc;
    int *dsm = (int *)buf, *dcm = dsm + smap.size(), *drm = dcm + cmap.size(), *dpm = drm + rmap.size(),
        *dna = dpm + pmap.size(), *did = dna + nadd.size();
    if ((rc = h2d(dsm, smap.data(), smap.size() * sizeof(int), h->stream)) ||
        (rc = h2d(dcm, cmap.data(), cmap.size() * sizeof(int), h->stream)) ||
        (rc = h2d(drm, rmap.data(), rmap.size() * sizeof(int), h->stream)) ||
        (rc = h2d(dpm, pmap.data(), pmap.size() * sizeof(int), h->stream)) ||
        (rc = h2d(dna, nadd.data(), nadd.size() * sizeof(int), h->stream)) ||
        (nk > 1 && (rc = h2d(did, map_id.data(), B * sizeof(int), h->stream))))
        return rc;
    // the constraint parameters first (they read the old layout's strides)
    ShiftParamArgs pa;
    pa.Kc = p.Kc; pa.P_old = p.P; pa.P_new = Pnew;
    pa.rmap = drm; pa.cmap = dcm; pa.pmap = dpm; pa.nadd = dna;
    pa.map_id = nk > 1 ? did : nullptr;
    pa.reb_delta0 = p.grf_delta; pa.reb_eps0 = p.grf_eps; pa.td_sigma0 = p.td_sigma; pa.td_lambda0 = p.td_lambda;
    pa.overflow = d.counter + 6;
    HIPCHK(hipMemsetAsync(d.counter + 6, 0, sizeof(int), h->stream));
    ShiftParamOut po;
    po.reb_delta = h->spare_reb_delta; po.reb_eps = h->spare_reb_eps; po.al_sigma = h->spare_al_sigma;
    po.al_lambda = h->spare_al_lambda; po.td_mask = h->spare_td_mask; po.cf_u = h->spare_cf_u;
    po.cf_flag = h->spare_cf_flag;
    launch_shift_params(p.B, pa, d, po, h->stream);
    HIPCHK(hipMemcpyAsync(h->host_counter + 6, d.counter + 6, sizeof(int), hipMemcpyDeviceToHost, h->stream));
    ShiftArgs a;
    a.S_old = p.S; a.S_new = Snew; a.Kc = p.Kc;
    a.smap = dsm; a.cmap = dcm;
    a.map_id = nk > 1 ? did : nullptr;
    a.fp32 = p.fp32;
    a.zero_u0 = 1;  // trajectory_ptrs.front()->Ubar[0].setZero() (HKDProblem.cpp:219)
    a.stage = nullptr;
    if (Snew != p.S) {
        if (!h->shift_stage && (rc = dalloc(h, h->shift_stage, 3 * B * h->S_cap * NX))) return rc;
        a.stage = h->shift_stage;
    }
    launch_shift_gather(p.B, a, d, h->spare_K, h->stream);  // (working rows and sel too)
    HIPCHK(hipGetLastError());
    // defer (hsddp_advance, one layout for the batch): the caller's host work runs under the gather;
    // everything after it is ordered on the handle's stream
    const bool async = defer && nk == 1;
    if (!async) HIPCHK(hipStreamSynchronize(h->stream));
    std::swap(d.reb_delta, h->spare_reb_delta);
    std::swap(d.reb_eps, h->spare_reb_eps);
    std::swap(d.al_sigma, h->spare_al_sigma);
    std::swap(d.al_lambda, h->spare_al_lambda);
    std::swap(d.td_mask, h->spare_td_mask);
    std::swap(d.cf_u, h->spare_cf_u);
    std::swap(d.cf_flag, h->spare_cf_flag);
    const bool td_overflow = !async && h->host_counter[6] != 0;
    if (p.fp32) { float *t = d.K32; d.K32 = (float *)h->spare_K; h->spare_K = t; }
    else { double *t = d.K; d.K = (double *)h->spare_K; h->spare_K = t; }
    // the new layouts
    if (nk == 1) {  // one layout for the batch: the handle's own
        const Layout &L = nl[0];
        p.P = L.P;
        p.has_tail = L.has_tail;
        h->reach_end.resize(L.P);
        for (int i = 0; i < L.P; ++i) {
            p.N[i] = L.N[i]; p.s0[i] = L.s0[i]; p.k0[i] = L.k0[i]; p.ss[i] = L.ss[i];
            h->reach_end[i] = phs[0][i].reach;
        }
        p.S = L.S;
        p.elem_layout = 0;
        h->lays.clear();
        h->reach_el.clear();
        h->desc.n_phases = L.P;
        for (int i = 0; i < L.P; ++i) h->desc.horizons[i] = L.N[i];
    } else {
        std::vector<Layout> lays(B);
        std::vector<int> reach(B * HSDDP_MAX_PHASES, 0);
        for (size_t b = 0; b < B; ++b) {
            lays[b] = nl[map_id[b]];
            for (int i = 0; i < lays[b].P; ++i) reach[b * HSDDP_MAX_PHASES + i] = phs[map_id[b]][i].reach;
        }
        if ((rc = set_layouts(h, lays))) return rc;
        h->reach_el = reach;
    }
    h->need_inputs = true;
    h->refs_on_device = false;  // built for the old layout
    h->ref_cols_stale = true;
    h->contacts_current = false;
    if (async) {
        h->shift_overflow_pending = true;
        h->scratch_reserved = ((nmaps + (nk > 1 ? B : 0)) * sizeof(int) + 255) & ~(size_t)255;
        for (std::vector<int> *v : {&smap, &cmap, &rmap, &pmap, &nadd}) h->shift_keep.push_back(std::move(*v));
    }
    if (td_overflow) {  // the shift itself is complete; the constraints past HSDDP_MAX_TD were not added
        if (overflow) *overflow = 1;
        else return fail(HSDDP_ERR_UNSUPPORTED, "a phase would carry more than HSDDP_MAX_TD touchdown constraints");
    }
    return HSDDP_OK;
}

extern "C" int hsddp_shift(hsddp_handle h, int n_steps, const int *contact_change)
{
    return shift_impl(h, n_steps, contact_change, 0, 1);
}

extern "C" int hsddp_shift_elements(hsddp_handle h, int n_steps, const int *contact_change)
{
    return shift_impl(h, n_steps, contact_change, h ? (size_t)n_steps : 0, 1);
}

extern "C" int hsddp_get_layout(hsddp_handle h, int *n_phases, int *horizons, int *shooting, int *reach_end)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    if (!h->lays.empty()) return fail(HSDDP_ERR_UNSUPPORTED, "per-element layouts: hsddp_get_element_layouts");
    const Params &p = h->p;
    if (n_phases) *n_phases = p.P;
    for (int i = 0; i < p.P; ++i) {
        if (horizons) horizons[i] = p.N[i];
        if (shooting) shooting[i] = p.ss[i];
        if (reach_end) reach_end[i] = h->reach_end[i];
    }
    return HSDDP_OK;
}

// The caller's own receding-horizon bookkeeping applied to a live handle (the C++ facade's
// MultiPhaseDDP after HKDProblem::update, HKDProblem.cpp:117-222): a new shared layout of the same
// Kc, with each phase's shooting states SS_set = {0 .. shooting[i] - 1} (SinglePhase.h:161-164).
// Host only; the inputs and warm start of the new layout are uploaded next.
extern "C" int hsddp_set_layout(hsddp_handle h, int n_phases, const int *horizons, const int *shooting,
                                const int *reach_end)
{
    if (!h || !horizons) return fail(HSDDP_ERR_ARG, "null argument");
    if (n_phases < 1 || n_phases > HSDDP_MAX_PHASES) return fail(HSDDP_ERR_ARG, "n_phases must lie in 1..16");
    Params &p = h->p;
    int s = 0, k = 0, tail = 0;
    for (int i = 0; i < n_phases; ++i) {
        const int N = horizons[i], ss = shooting ? shooting[i] : N + 1;
        if (N < 1) return fail(HSDDP_ERR_ARG, "phase horizons must be >= 1");
        if (ss < 0 || ss > N + 1) return fail(HSDDP_ERR_ARG, "shooting states must lie in 0 .. N_i + 1");
        // the knot-parallel rollout simulates non-shooting states after the shooting ones, and only
        // in the last phase (the one HKDProblem::update leaves with horizon <= 2)
        if (ss < N + 1 && i < n_phases - 1)
            return fail(HSDDP_ERR_UNSUPPORTED, "non-shooting states outside the last phase");
        tail |= ss < N + 1;
        s += N + 1;
        k += N;
    }
    if (k != p.Kc) return fail(HSDDP_ERR_ARG, "the layout's horizons must sum to the handle's Kc");
    if ((size_t)s > h->S_cap) return fail(HSDDP_ERR_ARG, "layout exceeds the handle's state-slot capacity");
    h->slots_fresh = false;
    s = k = 0;
    for (int i = 0; i < HSDDP_MAX_PHASES; ++i) {
        const bool in = i < n_phases;
        p.N[i] = in ? horizons[i] : 0;
        p.s0[i] = in ? s : 0;
        p.k0[i] = in ? k : 0;
        p.ss[i] = in ? (shooting ? shooting[i] : horizons[i] + 1) : 0;
        if (in) { s += horizons[i] + 1; k += horizons[i]; }
    }
    p.P = n_phases;
    p.S = s;
    p.has_tail = tail;
    p.elem_layout = 0;
    h->lays.clear();
    h->reach_el.clear();
    h->reach_end.assign(n_phases, 0);
    if (reach_end)
        for (int i = 0; i < n_phases; ++i) h->reach_end[i] = reach_end[i] ? 1 : 0;
    h->desc.n_phases = n_phases;
    for (int i = 0; i < HSDDP_MAX_PHASES; ++i) h->desc.horizons[i] = i < n_phases ? horizons[i] : 0;
    h->have_problem = false;  // inputs of the new layout next (hsddp_upload_problem)
    h->need_inputs = false;
    h->contacts_current = false;
    h->refs_on_device = false;
    h->ref_cols_stale = true;
    return HSDDP_OK;
}

// ---- batched reference construction ------------------------------------------------------------
extern "C" int hsddp_set_reference_table(hsddp_handle h, const hsddp_quad_state *table, int n, float dt_ref)
{
    if (!h || !table || n < 1) return fail(HSDDP_ERR_ARG, "null / empty table");
    if (!(dt_ref > 0)) return fail(HSDDP_ERR_ARG, "dt_ref must be > 0");
    HIPCHK(hipSetDevice(h->desc.device));
    std::vector<double> t((size_t)n * RT_W, 0.0);
    for (int i = 0; i < n; ++i) {
        double *q = &t[(size_t)i * RT_W];
        const hsddp_quad_state &s = table[i];
        for (int j = 0; j < 12; ++j) {
            q[RT_BODY + j] = s.body_state[j]; q[RT_QJ + j] = s.qJ[j]; q[RT_QJD + j] = s.qJd[j];
            q[RT_FOOT + j] = s.foot_placements[j]; q[RT_GRF + j] = s.grf[j];
        }
        for (int l = 0; l < 4; ++l) q[RT_C + l] = s.contact[l];
    }
    if (h->ref_table) { hipFree(h->ref_table); h->ref_table = nullptr; }
    HIPCHK(hipMalloc((void **)&h->ref_table, t.size() * sizeof(double)));
    HIPCHK(hipMemcpy(h->ref_table, t.data(), t.size() * sizeof(double), hipMemcpyHostToDevice));
    h->ref_n = n;
    h->ref_dt = dt_ref;
    h->table_host.assign(table, table + n);
    h->win_start.clear();
    return HSDDP_OK;
}

// sample index of relative time t in a window of sz + 1 samples (QuadReference.cpp:65-79, 86-99)
static int ref_sample(float t, float dt, int sz)
{
    int k = (int)std::floor(t / dt);
    if (t - k * dt > 0.5 * dt) k++;
    return k > sz ? sz : k;
}

static int build_refs(hsddp_handle h, const int *window_start, int window_len, const float *phase_start_times,
                      float dt_sim, bool initial);

extern "C" int hsddp_build_references(hsddp_handle h, const int *window_start, int window_len,
                                      const float *phase_start_times, float dt_sim)
{
    if (h) h->slots_fresh = false;  // new reference rows: the running costs change
    return build_refs(h, window_start, window_len, phase_start_times, dt_sim, true);
}

// initial: a new problem (not an hsddp_advance step): QuadReference's clock restarts and every
// phase's contact duration is read at its start time, as HKDProblem::initialization does
// (get_contact_duration_at_t at t = 0 and at each phase end, HKDProblem.cpp:38,63)
static int build_refs(hsddp_handle h, const int *window_start, int window_len, const float *phase_start_times,
                      float dt_sim, bool initial)
{
    if (!h || !window_start) return fail(HSDDP_ERR_ARG, "null argument");
    if (!h->ref_table) return fail(HSDDP_ERR_ARG, "no reference table (hsddp_set_reference_table)");
    if (window_len < 1 || !(dt_sim > 0)) return fail(HSDDP_ERR_ARG, "window_len >= 1 and dt_sim > 0 required");
    const Params &p = h->p;
    const int Br = h->Bref;
    const bool elem = !h->lays.empty();
    for (int b = 0; b < Br; ++b)
        if (window_start[b] < 0 || window_start[b] >= h->ref_n) return fail(HSDDP_ERR_ARG, "window start outside the table");
    if (elem && phase_start_times)
        return fail(HSDDP_ERR_ARG, "per-element layouts: the phase start times follow each element's own float clock (NULL)");
    // slot times as the reference forms them: t_offset (float, phase start relative to the first
    // phase) + k dt (double), passed on as float (SinglePhase.cpp:243-287; set_time_offset,
    // HKDProblem.cpp:103,208), snapped to a sample (QuadReference.cpp:60-76); per layout
    auto starts_of = [&](const Layout &L) {
        std::vector<float> start(L.P);
        if (phase_start_times) {
            for (int i = 0; i < L.P; ++i) start[i] = phase_start_times[i] - phase_start_times[0];
        } else {  // the float clock of HKDProblem::initialization (t += dt_sim per knot)
            float t = 0.0f;
            for (int i = 0; i < L.P; ++i) {
                start[i] = t;
                for (int k = 0; k < L.N[i]; ++k) t += dt_sim;
            }
        }
        return start;
    };
    const int sz = window_len - 1;
    // one slot map per distinct layout ([n_maps][S], padding slots repeat the last sample)
    std::map<std::vector<int>, int> keys;
    std::vector<int> idx, map_id(elem ? p.B : 0);
    std::vector<std::vector<float>> map_starts;
    for (int b = 0; b < (elem ? p.B : 1); ++b) {
        const Layout L = layout_of(h, b);
        std::vector<int> key(L.N, L.N + L.P);
        auto it = keys.find(key);
        if (it == keys.end()) {
            const std::vector<float> start = starts_of(L);
            std::vector<int> row(p.S, 0);
            for (int i = 0; i < L.P; ++i)
                for (int k = 0; k <= L.N[i]; ++k) {
                    const float t = (float)((double)start[i] + k * (double)dt_sim);
                    int q = (int)std::floor(t / h->ref_dt);
                    if (t - q * h->ref_dt > 0.5 * h->ref_dt) q++;
                    row[L.s0[i] + k] = q > sz ? sz : q;
                }
            for (int sl = L.S; sl < p.S; ++sl) row[sl] = row[L.S - 1];
            it = keys.emplace(key, (int)map_starts.size()).first;
            idx.insert(idx.end(), row.begin(), row.end());
            map_starts.push_back(start);
        }
        if (elem) map_id[b] = it->second;
    }
    HIPCHK(hipSetDevice(h->desc.device));
    char *buf;
    int rc;
    if ((rc = scratch(h, h->scratch_reserved + (Br + idx.size() + map_id.size()) * sizeof(int), &buf))) return rc;
    buf += h->scratch_reserved;  // (after a pending shift's maps: hsddp_advance)
    int *dstart = (int *)buf, *didx = dstart + Br, *dmap = didx + idx.size();
    if ((rc = h2d(dstart, window_start, Br * sizeof(int), h->stream)) ||
        (rc = h2d(didx, idx.data(), idx.size() * sizeof(int), h->stream)) ||
        (elem && (rc = h2d(dmap, map_id.data(), map_id.size() * sizeof(int), h->stream))))
        return rc;
    RefArgs a{h->ref_table, h->ref_n, dstart, didx, elem ? dmap : nullptr};
    launch_build_refs(p, h->d, Br, a, h->stream);
    h->ref_cols_stale = false;  // (k_build_refs writes the entry-major copy too)
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(h->stream));
    h->refs_on_device = true;
    h->win_start.assign(window_start, window_start + Br);
    h->win_len = window_len;
    h->dt_sim = dt_sim;
    if (initial) {
        h->t_cur = 0;
        h->durations.assign((size_t)p.B * p.P * 4, 0.0);
        for (int b = 0; b < p.B; ++b) {
            const std::vector<float> &start = map_starts[elem ? map_id[b] : 0];
            for (int i = 0; i < (int)start.size(); ++i) {
                const int k = std::min(window_start[Br == 1 ? 0 : b] + ref_sample(start[i], h->ref_dt, sz), h->ref_n - 1);
                for (int l = 0; l < 4; ++l) h->durations[((size_t)b * p.P + i) * 4 + l] = h->table_host[k].status_dur[l];
            }
        }
    }
    return HSDDP_OK;
}

// ---- reference-driven receding-horizon step -------------------------------------------------------
// HKDProblem::update (HKDProblem.cpp:117-222) with the contacts read from the reference table:
// per simulation step the window advances (QuadReference::step, QuadReference.cpp:33-47), the
// contact at the new horizon end (get_contact_at_t(new_end - new_start)) decides whether the last
// phase grows or a new phase starts, and a last phase that has reached its end gets the touchdown
// constraint / reset map towards the contact at plan_duration + dt_mpc (add_tconstr_one_phase,
// :199-202, 268-308).  Then the shifted warm start (hsddp_shift), the new layout's references
// (build_refs) and the new contacts and x0 (hsddp_update_problem).
static int advance_impl(hsddp_handle h, int n_steps, float plan_duration, float dt_mpc, const double *x0,
                        int *contact_change, int &overflow)
{
    if (!h->have_problem) return fail(HSDDP_ERR_ARG, "upload the problem first");
    if (h->need_inputs) return fail(HSDDP_ERR_ARG, "the previous shift awaits hsddp_update_problem");
    if (h->win_start.empty() || h->table_host.empty())
        return fail(HSDDP_ERR_ARG, "references not built from a table (hsddp_build_references)");
    if (n_steps < 0) return fail(HSDDP_ERR_ARG, "n_steps must be >= 0");
    const Params &p = h->p;
    const int B = p.B, Br = h->Bref, sz = h->win_len - 1;
    const bool elem = !h->lays.empty();
    const float dt = h->ref_dt, dts = h->dt_sim;
    // HSDDP_ADVANCE_TIMING=1: wall time of the advance's stages to stderr (a diagnostic)
    static const bool timing = std::getenv("HSDDP_ADVANCE_TIMING") != nullptr;
    using clk = std::chrono::steady_clock;
    clk::time_point tmark = clk::now();
    double tstage[6] = {0, 0, 0, 0, 0, 0};
    auto stage = [&](int q) {
        if (!timing) return;
        const clk::time_point t = clk::now();
        tstage[q] = std::chrono::duration<double, std::micro>(t - tmark).count();
        tmark = t;
    };
    auto leq = [](float a, float b) { return a < b || std::abs(a - b) <= 1e-6f; };
    int adv = 0;  // samples per simulation step
    for (int i = 1; leq(i * dt, dts); ++i) adv++;
    // QuadReference::step for every step: the window starts and the clock (shared by the batch)
    const int P0 = p.P;  // stride of the current contact rows [B][P0 + 1][4] and durations [B][P0][4]
    std::vector<std::vector<int>> wsj(n_steps);  // window starts at each step
    std::vector<float> relj(n_steps);            // new_end - new_start at each step
    std::vector<int> ws(h->win_start);
    float t_cur = h->t_cur;
    for (int j = 0; j < n_steps; ++j) {
        for (int a = 0; a < adv; ++a) {
            t_cur += dt;
            for (int &w : ws) w++;
        }
        for (int &w : ws)
            if (w >= h->ref_n) return fail(HSDDP_ERR_ARG, "the reference window ran past the table");
        wsj[j] = ws;
        relj[j] = (t_cur + plan_duration) - t_cur;  // new_end_time - new_start_time
    }
    auto sample_w = [&](const std::vector<int> &w, int b, float t) -> const hsddp_quad_state & {
        const int k = w[Br == 1 ? 0 : b] + ref_sample(t, dt, sz);
        return h->table_host[std::min(k, h->ref_n - 1)];
    };
    // HKDProblem::update's bookkeeping (HKDProblem.cpp:126-202) of every element over the steps: its
    // phases as sources — an old phase (index >= 0) or the sample a new phase starts from (step j:
    // -1 - j) — the step flags and where its next-contact row comes from
    struct Track {
        std::vector<int> hz, reach, src, flags;
        int P_old = 0;                       // the element's phases before the steps
        int next_kind = 0, next_step = -1;  // row P: 0 old row, 1 contact at relj, 2 at plan + dt_mpc
    };
    // with the handle's shared layout and window, an element whose contact rows equal element 0's
    // tracks exactly as element 0 does (the MPC batch of one gait): its bookkeeping is element 0's
    std::vector<int> rep(B);
    for (int b = 0; b < B; ++b) {
        const size_t n = (size_t)(P0 + 1) * 4;
        rep[b] = (b > 0 && !elem && Br == 1 &&
                  std::equal(h->contacts.begin() + (size_t)b * n, h->contacts.begin() + (size_t)(b + 1) * n, h->contacts.begin()))
                     ? 0 : b;
    }
    std::vector<Track> tr(B);
    for (int b = 0; b < B; ++b) {
        if (rep[b] != b) continue;
        Track &T = tr[b];
        const Layout L = layout_of(h, b);
        const int *reach0 = elem ? &h->reach_el[(size_t)b * HSDDP_MAX_PHASES] : h->reach_end.data();
        T.hz.assign(L.N, L.N + L.P);
        T.P_old = L.P;
        T.reach.assign(reach0, reach0 + L.P);
        for (int i = 0; i < L.P; ++i) T.src.push_back(i);
        T.flags.assign(n_steps, 0);
        auto phase_contact = [&](int sc, int l) {
            return sc >= 0 ? h->contacts[((size_t)b * (P0 + 1) + sc) * 4 + l]
                           : sample_w(wsj[-1 - sc], b, relj[-1 - sc]).contact[l];
        };
        for (int j = 0; j < n_steps; ++j) {
            if (T.hz.front() <= 1) {  // pop_front_phase (HKDProblem.h:56-66)
                if (T.hz.size() == 1) return fail(HSDDP_ERR_ARG, "advance would remove the only phase");
                T.hz.erase(T.hz.begin());
                T.reach.erase(T.reach.begin());
                T.src.erase(T.src.begin());
            } else {
                T.hz.front()--;
            }
            const int *nc = sample_w(wsj[j], b, relj[j]).contact;
            int cc = 0;
            for (int l = 0; l < 4; ++l) cc |= nc[l] != phase_contact(T.src.back(), l);
            if (cc && T.reach.back()) {
                if ((int)T.hz.size() >= HSDDP_MAX_PHASES) return fail(HSDDP_ERR_ARG, "advance exceeds HSDDP_MAX_PHASES phases");
                T.hz.push_back(1);
                T.reach.push_back(0);
                T.src.push_back(-1 - j);
                T.next_kind = 1;  // a new phase carries no terminal constraint (identity reset)
                T.next_step = j;
            } else {
                T.hz.back()++;
                if (cc) T.reach.back() = 1;
            }
            if (T.reach.back()) { T.next_kind = 2; T.next_step = j; }
            T.flags[j] = cc;
        }
    }
    // the shift: one set of flags for the batch when it agrees (the shared layout stays shared),
    // else every element's own (per-element layouts; they need per-element references)
    bool agree = !elem;
    for (int b = 1; b < B && agree; ++b) agree = tr[rep[b]].flags == tr[0].flags;
    stage(0);
    int rc;
    if (agree) {
        if ((rc = shift_impl(h, n_steps, tr[0].flags.data(), 0, 1, true, &overflow))) return rc;
    } else {
        if (B > 1 && Br == 1)
            return fail(HSDDP_ERR_UNSUPPORTED, "elements disagree on a contact change, which takes per-element layouts "
                                               "and per-element references (ref_per_element = 1)");
        std::vector<int> cc((size_t)B * n_steps);
        for (int b = 0; b < B; ++b)
            std::copy(tr[rep[b]].flags.begin(), tr[rep[b]].flags.end(), cc.begin() + (size_t)b * n_steps);
        // (hsddp_shift_elements, with a touchdown overflow reported after the rest of the step)
        if ((rc = shift_impl(h, n_steps, cc.data(), (size_t)n_steps, 1, false, &overflow))) return rc;
    }
    stage(1);
    for (int b = 0; b < B; ++b) {
        const Layout L = layout_of(h, b);
        const int *re = h->lays.empty() ? h->reach_end.data() : &h->reach_el[(size_t)b * HSDDP_MAX_PHASES];
        const Track &T = tr[rep[b]];
        if (L.P != (int)T.hz.size() || !std::equal(T.hz.begin(), T.hz.end(), L.N) ||
            !std::equal(T.reach.begin(), T.reach.end(), re))
            return fail(HSDDP_ERR_ARG, "internal: advance and shift disagree on the layout");
    }
    stage(2);
    const int P = p.P;  // the new stride (the largest layout's with per-element layouts)
    std::vector<int> contacts((size_t)B * (P + 1) * 4, 0);
    std::vector<double> dur((size_t)B * P * 4, 0.0);
    for (int b = 0; b < B; ++b) {
        const Track &T = tr[rep[b]];
        const int Pb = (int)T.hz.size();
        auto phase_contact = [&](int sc, int l) {
            return sc >= 0 ? h->contacts[((size_t)b * (P0 + 1) + sc) * 4 + l]
                           : sample_w(wsj[-1 - sc], b, relj[-1 - sc]).contact[l];
        };
        for (int i = 0; i < Pb; ++i) {
            const int sc = T.src[i];
            const double *dv = sc >= 0 ? &h->durations[((size_t)b * P0 + sc) * 4]
                                       : sample_w(wsj[-1 - sc], b, relj[-1 - sc]).status_dur;
            for (int l = 0; l < 4; ++l) {
                contacts[((size_t)b * (P + 1) + i) * 4 + l] = phase_contact(sc, l);
                dur[((size_t)b * P + i) * 4 + l] = dv[l];
            }
        }
        for (int l = 0; l < 4; ++l)
            contacts[((size_t)b * (P + 1) + Pb) * 4 + l] =
                T.next_kind == 0 ? h->contacts[((size_t)b * (P0 + 1) + T.P_old) * 4 + l]
                : T.next_kind == 1 ? sample_w(wsj[T.next_step], b, relj[T.next_step]).contact[l]
                                   : sample_w(wsj[T.next_step], b, plan_duration + dt_mpc).contact[l];
    }
    stage(3);
    if ((rc = build_refs(h, ws.data(), h->win_len, nullptr, dts, false))) return rc;
    stage(4);
    if (x0) {
        if ((rc = hsddp_update_problem(h, contacts.data(), x0, nullptr, nullptr, nullptr))) return rc;
    } else {  // x0 follows from the new first phase's contact: hsddp_update_problem(h, NULL, x0, NULL...)
        h->contacts.swap(contacts);
        h->contacts_current = true;
    }
    h->durations.swap(dur);
    h->t_cur = t_cur;
    stage(5);
    if (timing)
        std::fprintf(stderr, "hsddp_advance us: bookkeeping %.1f shift %.1f check %.1f contacts %.1f refs %.1f update %.1f\n",
                     tstage[0], tstage[1], tstage[2], tstage[3], tstage[4], tstage[5]);
    if (contact_change)  // per step: some element saw a contact change (the batch's flag when it agrees)
        for (int j = 0; j < n_steps; ++j) {
            int f = 0;
            for (int b = 0; b < B; ++b) f |= tr[rep[b]].flags[j];
            contact_change[j] = f;
        }
    return HSDDP_OK;
}

// hsddp_advance = advance_impl, then: the deferred shift's stream is drained before the host rows its
// copies read are released (whatever path left advance_impl), and its touchdown-overflow flag is
// read.  A touchdown overflow on a complete step (both shift paths) returns HSDDP_ERR_UNSUPPORTED
// with the handle ready to solve: new layout, references, contacts, x0, durations and clock, the
// phase keeping its first HSDDP_MAX_TD touchdown constraints.  When the step failed for another
// reason, that error is returned and an overflow is added to its message.
extern "C" int hsddp_advance(hsddp_handle h, int n_steps, float plan_duration, float dt_mpc, const double *x0,
                             int *contact_change)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    int overflow = 0;
    const int rc = advance_impl(h, n_steps, plan_duration, dt_mpc, x0, contact_change, overflow);
    if (h->shift_overflow_pending) {  // the deferred shift's flag (its copy is queued on the stream)
        const hipError_t e = hipStreamSynchronize(h->stream);
        if (e == hipSuccess && h->host_counter[6] != 0) overflow = 1;
        h->shift_overflow_pending = false;
        h->shift_keep.clear();
        h->scratch_reserved = 0;
        if (e != hipSuccess && rc == HSDDP_OK) return fail(HSDDP_ERR_DEVICE, std::string("advance: ") + hipGetErrorString(e));
    }
    static const char *msg = "a phase would carry more than HSDDP_MAX_TD touchdown constraints";
    if (rc == HSDDP_OK) return overflow ? fail(HSDDP_ERR_UNSUPPORTED, msg) : HSDDP_OK;
    if (overflow) fail(rc, std::string(hsddp_last_error()) + " (and " + msg + ")");
    return rc;
}

extern "C" int hsddp_get_phase_info(hsddp_handle h, int *contacts, double *durations)
{
    if (!h) return fail(HSDDP_ERR_ARG, "null handle");
    const Params &p = h->p;
    if (contacts) std::copy(h->contacts.begin(), h->contacts.end(), contacts);
    if (durations) {
        if (h->durations.size() != (size_t)p.B * p.P * 4)
            return fail(HSDDP_ERR_ARG, "no phase durations (references not built from a table)");
        std::copy(h->durations.begin(), h->durations.end(), durations);
    }
    return HSDDP_OK;
}
