// hsddp_reference.cpp — host side of the batched reference construction:
// the quad_reference.csv reader (QuadReference::load_top_level_data, Reference/QuadReference.cpp:
// 129-290) and the phase segmentation of HKDProblem::initialization (HKDMPC/HKD-TrajOpt/
// HKDProblem.cpp:15-68), both with the reference's float arithmetic.  The per-slot reference
// tensors themselves are built on the device (hsddp_mpc.hip, k_build_refs).
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "../../include/hsddp.h"

extern "C" int hsddp_ref_fail(int code, const char *msg);  // hsddp_api.cpp: sets hsddp_last_error

namespace {

// `count` numbers of the line into dst (the reference stops after its own bound; the vectors it
// reads into hold 12 or 4 entries)
template <typename T, typename F>
void read_words(const std::string &line, T *dst, int count, F conv)
{
    std::stringstream ls(line);
    std::string w;
    int i = 0;
    while (i < count && ls >> w) dst[i++] = conv(w);
}

double to_f(const std::string &w) { return (double)std::stof(w); }  // std::stof: float rounding
int to_i(const std::string &w) { return std::stoi(w); }

void swap_legs3(double *v)  // leg order (FR, FL, HR, HL) -> (FL, FR, HL, HR), 3 entries per leg
{
    double t[12];
    const int src[4] = {1, 0, 3, 2};
    for (int l = 0; l < 4; ++l)
        for (int a = 0; a < 3; ++a) t[3 * l + a] = v[3 * src[l] + a];
    std::memcpy(v, t, sizeof t);
}

// QuadReference::reorder_states (QuadReference.cpp:257-290): the MHPC convention
void reorder(hsddp_quad_state &q)
{
    double b[12];
    for (int a = 0; a < 3; ++a) {
        b[a] = q.body_state[3 + a];      // pos
        b[3 + a] = q.body_state[a];      // eul
        b[6 + a] = q.body_state[9 + a];  // vWorld
        b[9 + a] = q.body_state[6 + a];  // omega (eul rate slot)
    }
    b[2] = 0.25;
    std::memcpy(q.body_state, b, sizeof b);
    swap_legs3(q.qJ);
    std::memset(q.qJd, 0, sizeof q.qJd);
    swap_legs3(q.foot_placements);
    swap_legs3(q.grf);
    swap_legs3(q.torque);
    const int c[4] = {q.contact[1], q.contact[0], q.contact[3], q.contact[2]};
    const double d[4] = {q.status_dur[1], q.status_dur[0], q.status_dur[3], q.status_dur[2]};
    std::memcpy(q.contact, c, sizeof c);
    std::memcpy(q.status_dur, d, sizeof d);
    for (int l = 0; l < 4; ++l) {
        q.qJ[3 * l + 1] = -q.qJ[3 * l + 1];
        q.qJ[3 * l + 2] = -q.qJ[3 * l + 2];
        q.torque[3 * l + 1] = -q.torque[3 * l + 1];
        q.torque[3 * l + 2] = -q.torque[3 * l + 2];
    }
}

// approx_eq_scalar / approx_leq_scalar / approx_geq_scalar (HSDDP_Utils.h:46-78)
bool approx_eq(float a, float b) { return std::abs(a - b) <= 1e-6f; }
bool approx_leq(float a, float b) { return a < b || approx_eq(a, b); }
bool approx_geq(float a, float b) { return a > b || approx_eq(a, b); }

// sample index of relative time t (QuadReference.cpp:64-75, 81-91): left-clipped, moved right when
// past the half step, clamped to the window end
int sample_at(float t, float dt, int sz)
{
    int k = (int)std::floor(t / dt);
    if (t - k * dt > 0.5 * dt) k++;
    return k > sz ? sz : k;
}

}  // namespace

extern "C" int hsddp_load_quad_reference(const char *path, int reorder_legs, float *dt, hsddp_quad_state *out,
                                         int capacity)
{
    if (!path) return hsddp_ref_fail(HSDDP_ERR_ARG, "null path");
    std::ifstream f(path);
    if (!f) return hsddp_ref_fail(HSDDP_ERR_IO, (std::string("cannot open ") + path).c_str());
    hsddp_quad_state q;
    std::memset(&q, 0, sizeof q);
    float dtv = 0;
    int n = 0;
    std::string line;
    try {
        // keyword tests in the reference's order (a line is matched by substring, `dt` exactly)
        while (std::getline(f, line)) {
            if (line == "dt") {
                if (std::getline(f, line)) dtv = std::stof(line);
                continue;
            }
            if (line.find("body_state") != std::string::npos) {
                std::memset(&q, 0, sizeof q);  // quad_state.SetZero()
                if (std::getline(f, line)) read_words(line, q.body_state, 12, to_f);
                continue;
            }
            if (line.find("qJ") != std::string::npos) {
                if (std::getline(f, line)) read_words(line, q.qJ, 12, to_f);
                continue;
            }
            if (line.find("foot_placements") != std::string::npos) {
                if (std::getline(f, line)) read_words(line, q.foot_placements, 12, to_f);
                continue;
            }
            if (line.find("grf") != std::string::npos) {
                if (std::getline(f, line)) read_words(line, q.grf, 12, to_f);
                continue;
            }
            if (line.find("torque") != std::string::npos) {
                if (std::getline(f, line)) read_words(line, q.torque, 12, to_f);
                continue;
            }
            // the reference reads up to 12 words into these 4-vectors; 4 are kept here
            if (line.find("contact") != std::string::npos) {
                if (std::getline(f, line)) read_words(line, q.contact, 4, to_i);
                continue;
            }
            if (line.find("status_dur") != std::string::npos) {
                if (std::getline(f, line)) read_words(line, q.status_dur, 4, to_f);
                hsddp_quad_state r = q;
                if (reorder_legs) reorder(r);
                if (out && n < capacity) out[n] = r;
                ++n;
            }
        }
    } catch (const std::exception &e) {
        return hsddp_ref_fail(HSDDP_ERR_IO, (std::string("malformed reference file: ") + e.what()).c_str());
    }
    if (dt) *dt = dtv;
    return n;
}

extern "C" int hsddp_plan_phases(const hsddp_quad_state *w, int n_window, float dt_ref, float plan_duration,
                                 float dt_sim, float dt_mpc, hsddp_phase_plan *plan)
{
    if (!w || !plan || n_window < 1) return hsddp_ref_fail(HSDDP_ERR_ARG, "null argument / empty window");
    if (!(dt_ref > 0) || !(dt_sim > 0)) return hsddp_ref_fail(HSDDP_ERR_ARG, "dt_ref and dt_sim must be > 0");
    const int sz = n_window - 1;
    std::memset(plan, 0, sizeof *plan);
    int prev[4], cur[4];
    double dur[4];
    auto contact = [&](int *c, float t) { std::memcpy(c, w[sample_at(t, dt_ref, sz)].contact, 4 * sizeof(int)); };
    auto duration = [&](double *d, float t) { std::memcpy(d, w[sample_at(t, dt_ref, sz)].status_dur, 4 * sizeof(double)); };
    float t = 0.0f, start = 0.0f;
    contact(prev, t);
    duration(dur, t);
    int P = 0;
    while (approx_leq(t, plan_duration)) {
        contact(cur, t);
        const bool change = std::memcmp(cur, prev, sizeof cur) != 0;
        if (change || approx_geq(t, plan_duration)) {
            if (P >= HSDDP_MAX_PHASES) return hsddp_ref_fail(HSDDP_ERR_ARG, "more than HSDDP_MAX_PHASES phases");
            const float end = t;
            plan->start_times[P] = start;
            plan->end_times[P] = end;
            plan->horizons[P] = (int)std::round((end - start) / dt_sim);
            std::memcpy(plan->contacts[P], prev, sizeof prev);
            std::memcpy(plan->durations[P], dur, sizeof dur);
            ++P;
            std::memcpy(prev, cur, sizeof cur);
            duration(dur, t);
            start = end;
        }
        t += dt_sim;
    }
    plan->n_phases = P;
    // the last phase's next contact (add_tconstr_one_phase, HKDProblem.cpp:272-276)
    contact(plan->contacts[P], plan_duration + dt_mpc);
    for (int i = 0; i < P; ++i)
        if (plan->horizons[i] < 1) return hsddp_ref_fail(HSDDP_ERR_ARG, "a phase of zero knots (dt_sim too coarse)");
    return HSDDP_OK;
}
