// hsddp_facade.hpp — C++ facade over the C-ABI (include/hsddp.h) with the reference solver's
// class and member names, so that HKD-MPC callers keep their call sequence:
//
//   phases = deque<shared_ptr<SinglePhaseBase<double>>>   (HKDProblem.cpp:72-108)
//   solver.set_multiPhaseProblem(phases);                  (MultiPhaseDDP.h:27-35)
//   solver.set_initial_condition(x0);                      (MultiPhaseDDP.h:37)
//   solver.solve(option);                                  (MultiPhaseDDP.cpp:232-428)
//   solver.get_solver_info(...) / get_actual_cost()        (MultiPhaseDDP.cpp:532-541, .h:71)
//   results in each phase's Trajectory: Xbar, Ubar, K, X, U, Defect, dX, dU
//
// Header-only; link with libhsddp_amd.so.  Eigen is not available on this platform, so DVec /
// DMat / VecM / MatMN are small dense containers with Eigen's element access (operator(),
// size/rows/cols, setZero, data) and Eigen's column-major storage.
//
// The device evaluates the HKD model, costs and constraints itself, so a phase runs on the GPU
// only when its plugins are the hkd:: types below (the HKD registrations of
// HKDProblem::create_problem_one_phase / add_tconstr_one_phase, HKDProblem.cpp:225-310).  Any
// other std::function or cost/constraint object cannot run there: solve() throws
// std::runtime_error naming it — there is no CPU fallback.
#ifndef HSDDP_FACADE_HPP
#define HSDDP_FACADE_HPP

#include <algorithm>
#include <array>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/hsddp.h"

// ---- dense containers (Eigen-style access, column-major) -------------------------------------
template <typename T>
class DVec {
public:
    DVec() = default;
    explicit DVec(size_t n) : v_(n, T(0)) {}
    size_t size() const { return v_.size(); }
    T &operator()(size_t i) { return v_[i]; }
    const T &operator()(size_t i) const { return v_[i]; }
    T &operator[](size_t i) { return v_[i]; }
    const T &operator[](size_t i) const { return v_[i]; }
    void setZero() { std::fill(v_.begin(), v_.end(), T(0)); }
    void setZero(size_t n) { v_.assign(n, T(0)); }
    T *data() { return v_.data(); }
    const T *data() const { return v_.data(); }

private:
    std::vector<T> v_;
};

template <typename T>
class DMat {
public:
    DMat() = default;
    DMat(size_t r, size_t c) : r_(r), c_(c), v_(r * c, T(0)) {}
    size_t rows() const { return r_; }
    size_t cols() const { return c_; }
    T &operator()(size_t i, size_t j) { return v_[j * r_ + i]; }
    const T &operator()(size_t i, size_t j) const { return v_[j * r_ + i]; }
    void setZero() { std::fill(v_.begin(), v_.end(), T(0)); }
    void setZero(size_t r, size_t c) { r_ = r; c_ = c; v_.assign(r * c, T(0)); }
    T *data() { return v_.data(); }
    const T *data() const { return v_.data(); }

private:
    size_t r_ = 0, c_ = 0;
    std::vector<T> v_;
};

template <typename T, size_t n>
class VecM {
public:
    VecM() { a_.fill(T(0)); }
    static constexpr size_t size() { return n; }
    T &operator()(size_t i) { return a_[i]; }
    const T &operator()(size_t i) const { return a_[i]; }
    T &operator[](size_t i) { return a_[i]; }
    const T &operator[](size_t i) const { return a_[i]; }
    void setZero() { a_.fill(T(0)); }
    T *data() { return a_.data(); }
    const T *data() const { return a_.data(); }

private:
    std::array<T, n> a_;
};

template <typename T, size_t m, size_t n>
class MatMN {
public:
    MatMN() { a_.fill(T(0)); }
    static constexpr size_t rows() { return m; }
    static constexpr size_t cols() { return n; }
    T &operator()(size_t i, size_t j) { return a_[j * m + i]; }
    const T &operator()(size_t i, size_t j) const { return a_[j * m + i]; }
    void setZero() { a_.fill(T(0)); }
    T *data() { return a_.data(); }
    const T *data() const { return a_.data(); }

private:
    std::array<T, m * n> a_;
};

// ---- HSDDP_OPTION (HSDDP_CompoundTypes.h:18-60) and its INFO loader (:62-87) -------------------
struct HSDDP_OPTION {
    double alpha, gamma, update_penalty, update_relax, update_regularization, update_ReB;
    int max_DDP_iter, max_AL_iter, max_DDP_iter_runtime, max_AL_iter_runtime;
    double cost_thresh, tconstr_thresh, pconstr_thresh, dynamics_feas_thresh;
    double merit_rho, merit_scale, merit_offset;
    bool AL_active, ReB_active, smooth_active, MS;
    int nsteps_per_node;
    HSDDP_OPTION() { from_c(c_defaults()); }

    static hsddp_options c_defaults()
    {
        hsddp_options o;
        hsddp_default_options(&o);
        return o;
    }
    void from_c(const hsddp_options &o)
    {
        alpha = o.alpha; gamma = o.gamma; update_penalty = o.update_penalty; update_relax = o.update_relax;
        update_regularization = o.update_regularization; update_ReB = o.update_ReB;
        max_DDP_iter = o.max_DDP_iter; max_AL_iter = o.max_AL_iter;
        max_DDP_iter_runtime = o.max_DDP_iter_runtime; max_AL_iter_runtime = o.max_AL_iter_runtime;
        cost_thresh = o.cost_thresh; tconstr_thresh = o.tconstr_thresh; pconstr_thresh = o.pconstr_thresh;
        dynamics_feas_thresh = o.dynamics_feas_thresh;
        merit_rho = o.merit_rho; merit_scale = o.merit_scale; merit_offset = o.merit_offset;
        AL_active = o.AL_active; ReB_active = o.ReB_active; smooth_active = o.smooth_active; MS = o.MS;
        nsteps_per_node = o.nsteps_per_node;
    }
    hsddp_options to_c() const
    {
        hsddp_options o = c_defaults();
        o.alpha = alpha; o.gamma = gamma; o.update_penalty = update_penalty; o.update_relax = update_relax;
        o.update_regularization = update_regularization; o.update_ReB = update_ReB;
        o.max_DDP_iter = max_DDP_iter; o.max_AL_iter = max_AL_iter;
        o.max_DDP_iter_runtime = max_DDP_iter_runtime; o.max_AL_iter_runtime = max_AL_iter_runtime;
        o.cost_thresh = cost_thresh; o.tconstr_thresh = tconstr_thresh; o.pconstr_thresh = pconstr_thresh;
        o.dynamics_feas_thresh = dynamics_feas_thresh;
        o.merit_rho = merit_rho; o.merit_scale = merit_scale; o.merit_offset = merit_offset;
        o.AL_active = AL_active; o.ReB_active = ReB_active; o.smooth_active = smooth_active; o.MS = MS;
        o.nsteps_per_node = nsteps_per_node;
        return o;
    }
};

inline void loadHSDDPSetting(const std::string &filename, HSDDP_OPTION &option)
{
    hsddp_options o = option.to_c();
    if (hsddp_load_settings(filename.c_str(), &o) != HSDDP_OK) throw std::runtime_error(hsddp_last_error());
    option.from_c(o);
}

// ---- Trajectory (TrajectoryManagement.h:20-80), the fields the solver reads and writes --------
template <typename T, size_t xs, size_t us, size_t ys>
class Trajectory {
public:
    Trajectory() = default;
    Trajectory(T timeStep_, int horizon_) { create_data(timeStep_, horizon_); }
    void create_data(T timeStep_, int horizon_)
    {
        timeStep = timeStep_;
        horizon = horizon_;
        duration = timeStep * horizon;
        Xbar.assign(horizon + 1, VecM<T, xs>()); X = Xbar; Defect = Xbar; Defect_bar = Xbar; dX = Xbar;
        Ubar.assign(horizon, VecM<T, us>()); U = Ubar; dU = Ubar;
        K.assign(horizon, MatMN<T, us, xs>());
    }
    int size() { return (int)Xbar.size(); }

    T duration = 0, timeStep = 0;
    int horizon = 0;
    std::deque<VecM<T, xs>> Xbar, X, Defect, Defect_bar, dX;
    std::deque<VecM<T, us>> Ubar, U, dU;
    std::deque<MatMN<T, us, xs>> K;
};

// ---- plugin bases (SinglePhaseInterface.h:47-53, ConstraintsBase.h:267-268, 401-402) ----------
template <typename T, size_t xs, size_t us, size_t ys>
class CostBase {
public:
    virtual ~CostBase() = default;
    std::string cost_name;
};
template <typename T, size_t xs, size_t us, size_t ys>
class PathConstraintBase {
public:
    virtual ~PathConstraintBase() = default;
    std::string constraint_name;
};
template <typename T, size_t xs>
class TerminalConstraintBase {
public:
    virtual ~TerminalConstraintBase() = default;
    std::string constraint_name;
};

template <typename T>
class SinglePhaseBase {
public:
    virtual ~SinglePhaseBase() = default;
};

template <typename> class MultiPhaseDDP;

// ---- SinglePhase (SinglePhase.h:21-92): the setters the HKD problem builder calls -----------
template <typename T, size_t xs, size_t us, size_t ys>
class SinglePhase : public SinglePhaseBase<T> {
public:
    typedef VecM<T, xs> State;
    typedef VecM<T, us> Contrl;
    typedef VecM<T, ys == 0 ? 1 : ys> Output;
    typedef MatMN<T, xs, xs> StateMap;
    typedef MatMN<T, xs, us> ContrlMap;
    typedef MatMN<T, ys == 0 ? 1 : ys, xs> OutputMap;
    typedef MatMN<T, ys == 0 ? 1 : ys, us> DirectMap;
    friend class MultiPhaseDDP<T>;

    void set_trajectory(std::shared_ptr<Trajectory<T, xs, us, ys>> traj_) { traj = traj_; }
    void set_dynamics(std::function<void(State &, Output &, State &, Contrl &, T)> f) { dynamics = f; }
    void set_dynamics_partial(
        std::function<void(StateMap &, ContrlMap &, OutputMap &, DirectMap &, State &, Contrl &, T)> f)
    {
        dynamics_partial = f;
    }
    void set_resetmap(std::function<void(DVec<T> &, DVec<T> &)> f) { resetmap_func_handle = f; }
    void set_resetmap_partial(std::function<void(DMat<T> &, DVec<T> &)> f) { resetmap_partial_func_handle = f; }
    void set_time_offset(float t) { t_offset = t; }
    void add_cost(std::shared_ptr<CostBase<T, xs, us, ys>> c) { costs.push_back(c); }
    void add_pathConstraint(std::shared_ptr<PathConstraintBase<T, xs, us, ys>> c) { pconstraints.push_back(c); }
    void add_terminalConstraint(std::shared_ptr<TerminalConstraintBase<T, xs>> c) { tconstraints.push_back(c); }
    std::shared_ptr<Trajectory<T, xs, us, ys>> get_trajectory() { return traj; }

private:
    std::function<void(State &, Output &, State &, Contrl &, T)> dynamics;
    std::function<void(StateMap &, ContrlMap &, OutputMap &, DirectMap &, State &, Contrl &, T)> dynamics_partial;
    std::function<void(DVec<T> &, DVec<T> &)> resetmap_func_handle;
    std::function<void(DMat<T> &, DVec<T> &)> resetmap_partial_func_handle;
    std::vector<std::shared_ptr<CostBase<T, xs, us, ys>>> costs;
    std::vector<std::shared_ptr<PathConstraintBase<T, xs, us, ys>>> pconstraints;
    std::vector<std::shared_ptr<TerminalConstraintBase<T, xs>>> tconstraints;
    std::shared_ptr<Trajectory<T, xs, us, ys>> traj;
    float t_offset = 0;
};

// ---- the HKD registrations the device path evaluates ------------------------------------------
namespace hkd {
typedef SinglePhase<double, 24, 24, 0> Phase;

namespace detail {
// one batched model primitive on a single point, through device buffers (host convenience only:
// the solver never calls these — it evaluates the model inside its kernels)
template <typename F>
inline void on_device(const std::vector<std::pair<const void *, size_t>> &in, const std::vector<std::pair<void *, size_t>> &out,
                      F call)
{
    std::vector<void *> din, dout;
    for (auto &b : in) {
        void *p = hsddp_device_alloc(b.second, 0);
        if (!p || hsddp_memcpy_h2d(p, b.first, b.second) != HSDDP_OK) throw std::runtime_error(hsddp_last_error());
        din.push_back(p);
    }
    for (auto &b : out) {
        void *p = hsddp_device_alloc(b.second, 0);
        if (!p) throw std::runtime_error(hsddp_last_error());
        dout.push_back(p);
    }
    const int rc = call(din, dout);
    if (rc == HSDDP_OK) hsddp_device_synchronize(0);
    for (size_t i = 0; i < out.size() && rc == HSDDP_OK; ++i) hsddp_memcpy_d2h(out[i].first, dout[i], out[i].second);
    for (void *p : din) hsddp_device_free(p);
    for (void *p : dout) hsddp_device_free(p);
    if (rc != HSDDP_OK) throw std::runtime_error(hsddp_last_error());
}
}  // namespace detail

// HKD::Model::dynamics with this phase's contact (HKDModel.h:33-45; HKDProblem.cpp:231)
struct Dynamics {
    std::array<int, 4> contact{};
    double dt = 0.01;
    void operator()(Phase::State &xn, Phase::Output &, Phase::State &x, Phase::Contrl &u, double) const
    {
        const double c[4] = {(double)contact[0], (double)contact[1], (double)contact[2], (double)contact[3]};
        detail::on_device({{x.data(), 192}, {u.data(), 192}, {c, 32}}, {{xn.data(), 192}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_dynamics((double *)i[0], (double *)i[1], (double *)i[2], dt,
                                                        (double *)o[0], 1, nullptr);
                          });
    }
};
// HKD::Model::dynamics_partial (HKDModel.h:46-61): A, B in Eigen column-major layout
struct DynamicsPartial {
    std::array<int, 4> contact{};
    double dt = 0.01;
    void operator()(Phase::StateMap &A, Phase::ContrlMap &B, Phase::OutputMap &, Phase::DirectMap &, Phase::State &x,
                    Phase::Contrl &u, double) const
    {
        const double c[4] = {(double)contact[0], (double)contact[1], (double)contact[2], (double)contact[3]};
        detail::on_device({{x.data(), 192}, {u.data(), 192}, {c, 32}}, {{A.data(), 4608}, {B.data(), 4608}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_dynamics_partial((double *)i[0], (double *)i[1], (double *)i[2], dt,
                                                                (double *)o[0], (double *)o[1], 1, nullptr);
                          });
    }
};
// HKDReset::resetmap / resetmap_partial from this phase's contact to the next (HKDReset.h:41-136)
struct Resetmap {
    std::array<int, 4> contact{}, next_contact{};
    void operator()(DVec<double> &xn, DVec<double> &x) const
    {
        xn.setZero(24);
        detail::on_device({{x.data(), 192}, {contact.data(), 16}, {next_contact.data(), 16}}, {{xn.data(), 192}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_resetmap((double *)i[0], (int *)i[1], (int *)i[2], (double *)o[0], 1,
                                                        nullptr);
                          });
    }
};
struct ResetmapPartial {
    std::array<int, 4> contact{}, next_contact{};
    void operator()(DMat<double> &Px, DVec<double> &x) const
    {
        Px.setZero(24, 24);
        detail::on_device({{x.data(), 192}, {contact.data(), 16}, {next_contact.data(), 16}}, {{Px.data(), 4608}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_resetmap_partial((double *)i[0], (int *)i[1], (int *)i[2],
                                                                (double *)o[0], 1, nullptr);
                          });
    }
};

// HKDTrackingCost (HKDCost.h:8-38) with its per-knot reference (HKDReference.cpp:8-57) and
// HKDFootPlaceReg (HKDCost.cpp:5-63): weights shared by every phase of a problem
struct TrackingCost : CostBase<double, 24, 24, 0> {
    hsddp_hkd_weights weights;
    std::vector<std::array<double, 24>> x_ref;  // horizon + 1 states
    std::vector<std::array<double, 24>> u_ref;  // horizon + 1 (the last is unused, as the reference's lookup)
    TrackingCost() { hsddp_default_weights(&weights); cost_name = "HKD Tracking Cost"; }
};
struct FootPlaceReg : CostBase<double, 24, 24, 0> {
    std::vector<std::array<double, 12>> foot_ref;  // horizon + 1
    FootPlaceReg() { cost_name = "HKD Foot Placement Regularization"; }
};
// GRFConstraint + ReB (HKDConstraints.cpp:7-66; ConstraintsBase.h:204-263) and
// TouchDownConstraint + AL (HKDConstraints.cpp:69-171; ConstraintsBase.h:374-399)
struct GRFConstraint : PathConstraintBase<double, 24, 24, 0> {
    hsddp_constraint_params params;
    GRFConstraint() { hsddp_default_constraint_params(&params); constraint_name = "GRF constraint"; }
};
struct TouchDownConstraint : TerminalConstraintBase<double, 24> {
    std::array<int, 4> next_contact{};
    TouchDownConstraint() { constraint_name = "touch down constraint"; }
};
}  // namespace hkd

// ---- MultiPhaseDDP (MultiPhaseDDP.h:18-90) --------------------------------------------------
template <typename T>
class MultiPhaseDDP {
public:
    MultiPhaseDDP() = default;
    ~MultiPhaseDDP() { release(); }
    MultiPhaseDDP(const MultiPhaseDDP &) = delete;
    MultiPhaseDDP &operator=(const MultiPhaseDDP &) = delete;

    void set_multiPhaseProblem(std::deque<std::shared_ptr<SinglePhaseBase<T>>> phases_in)
    {
        phases = phases_in;
        n_phases = (int)phases.size();
        actual_cost = 0;
        max_pconstr = max_tconstr = 0;
    }
    void set_initial_condition(DVec<T> x0_in) { x0 = x0_in; }

    // MultiPhaseDDP::solve (MultiPhaseDDP.cpp:232-428) for this one trajectory on the GPU
    void solve(HSDDP_OPTION option);

    T get_actual_cost() { return actual_cost; }
    T measure_dynamics_feasibility(int = 2) { return feas; }
    // final values only: the device solve keeps no per-iteration history (the reference appends
    // one entry per accepted inner iteration, MultiPhaseDDP.cpp:277-280, 368-371)
    void get_solver_info(std::vector<float> &cost_out, std::vector<float> &dyn_feas_out,
                         std::vector<float> &eqn_feas_out, std::vector<float> &ineq_feas_out)
    {
        cost_out = {(float)actual_cost};
        dyn_feas_out = {(float)feas};
        eqn_feas_out = {(float)max_tconstr};
        ineq_feas_out = {(float)max_pconstr};
    }
    // per-element outcome of the last solve (hsddp_element_info)
    const hsddp_element_info &element_info() const { return info; }

private:
    typedef hkd::Phase Phase;
    void release()
    {
        if (handle) hsddp_destroy(handle);
        handle = nullptr;
    }
    static void check(int rc)
    {
        if (rc != HSDDP_OK) throw std::runtime_error(std::string("hsddp: ") + hsddp_last_error());
    }
    template <typename P, typename F>
    static const P *plugin(const F &f, const char *what, int i)
    {
        const P *p = f ? f.template target<P>() : nullptr;
        if (!p)
            throw std::runtime_error("phase " + std::to_string(i) + ": " + what +
                                     " is not the HKD registration (hkd::" + what +
                                     "); only HKD problems run on the device");
        return p;
    }

    std::deque<std::shared_ptr<SinglePhaseBase<T>>> phases;
    int n_phases = 0;
    DVec<T> x0;
    T actual_cost = 0, feas = 0, max_pconstr = 0, max_tconstr = 0;
    hsddp_element_info info{};
    hsddp_handle handle = nullptr;
};

template <typename T>
void MultiPhaseDDP<T>::solve(HSDDP_OPTION option)
{
    static_assert(std::is_same<T, double>::value, "the device path computes in fp64");
    if (n_phases < 1 || n_phases > HSDDP_MAX_PHASES) throw std::runtime_error("hsddp: 1..16 phases supported");
    if (x0.size() != 24) throw std::runtime_error("hsddp: set_initial_condition needs a 24-state x0");
    std::vector<Phase *> ph(n_phases);
    hsddp_problem_desc desc;
    std::memset(&desc, 0, sizeof desc);
    desc.device = 0;
    desc.batch = 1;
    desc.n_phases = n_phases;
    desc.ref_per_element = 0;
    hsddp_default_weights(&desc.weights);
    hsddp_default_constraint_params(&desc.cparams);
    std::vector<int> contacts(4 * (n_phases + 1));
    int S = 0, Kc = 0;
    for (int i = 0; i < n_phases; ++i) {
        ph[i] = dynamic_cast<Phase *>(phases[i].get());
        if (!ph[i]) throw std::runtime_error("phase " + std::to_string(i) + " is not SinglePhase<double,24,24,0>");
        if (!ph[i]->traj) throw std::runtime_error("phase " + std::to_string(i) + " has no trajectory");
        const auto *dyn = plugin<hkd::Dynamics>(ph[i]->dynamics, "Dynamics", i);
        plugin<hkd::DynamicsPartial>(ph[i]->dynamics_partial, "DynamicsPartial", i);
        desc.horizons[i] = ph[i]->traj->horizon;
        if (i == 0) desc.dt = ph[i]->traj->timeStep;
        for (int l = 0; l < 4; ++l) contacts[4 * i + l] = dyn->contact[l];
        S += desc.horizons[i] + 1;
        Kc += desc.horizons[i];
        bool tracking = false, foot = false;
        for (auto &c : ph[i]->costs) {
            if (auto *tc = dynamic_cast<hkd::TrackingCost *>(c.get())) { desc.weights = tc->weights; tracking = true; }
            else if (dynamic_cast<hkd::FootPlaceReg *>(c.get())) foot = true;
            else throw std::runtime_error("phase " + std::to_string(i) + ": cost '" + c->cost_name + "' cannot run on the device");
        }
        if (!tracking || !foot) throw std::runtime_error("phase " + std::to_string(i) + ": needs hkd::TrackingCost and hkd::FootPlaceReg");
        for (auto &c : ph[i]->pconstraints) {
            if (auto *g = dynamic_cast<hkd::GRFConstraint *>(c.get())) desc.cparams = g->params;
            else throw std::runtime_error("phase " + std::to_string(i) + ": path constraint '" + c->constraint_name + "' cannot run on the device");
        }
        for (auto &c : ph[i]->tconstraints) {
            auto *td = dynamic_cast<hkd::TouchDownConstraint *>(c.get());
            if (!td) throw std::runtime_error("phase " + std::to_string(i) + ": terminal constraint '" + c->constraint_name + "' cannot run on the device");
            if (i == n_phases - 1)
                for (int l = 0; l < 4; ++l) contacts[4 * n_phases + l] = td->next_contact[l];
        }
    }
    if (ph[n_phases - 1]->tconstraints.empty())  // no touchdown after the horizon: keep the contact
        for (int l = 0; l < 4; ++l) contacts[4 * n_phases + l] = contacts[4 * (n_phases - 1) + l];
    // references per state slot (phase-major, S = sum(N_i + 1))
    std::vector<double> rx(24 * S), ru(24 * S), rf(12 * S), Xb(24 * S), Ub(24 * Kc), K(576 * Kc);
    int s = 0, kc = 0;
    for (int i = 0; i < n_phases; ++i) {
        const hkd::TrackingCost *tc = nullptr;
        const hkd::FootPlaceReg *fr = nullptr;
        for (auto &c : ph[i]->costs) {
            if (!tc) tc = dynamic_cast<hkd::TrackingCost *>(c.get());
            if (!fr) fr = dynamic_cast<hkd::FootPlaceReg *>(c.get());
        }
        const int N = desc.horizons[i];
        if ((int)tc->x_ref.size() != N + 1 || (int)tc->u_ref.size() < N || (int)fr->foot_ref.size() != N + 1)
            throw std::runtime_error("phase " + std::to_string(i) + ": reference lengths must match the horizon");
        auto &tr = *ph[i]->traj;
        for (int k = 0; k <= N; ++k, ++s) {
            for (int j = 0; j < 24; ++j) {
                rx[24 * s + j] = tc->x_ref[k][j];
                ru[24 * s + j] = k < (int)tc->u_ref.size() ? tc->u_ref[k][j] : 0.0;
                Xb[24 * s + j] = tr.Xbar[k][j];
            }
            for (int j = 0; j < 12; ++j) rf[12 * s + j] = fr->foot_ref[k][j];
        }
        for (int k = 0; k < N; ++k, ++kc)
            for (int a = 0; a < 24; ++a) {
                Ub[24 * kc + a] = tr.Ubar[k][a];
                for (int b = 0; b < 24; ++b) K[576 * kc + 24 * a + b] = tr.K[k](a, b);  // row-major on the ABI
            }
    }
    release();
    check(hsddp_create(&desc, &handle));
    const hsddp_options o = option.to_c();
    check(hsddp_set_options(handle, &o));
    check(hsddp_upload_problem(handle, contacts.data(), x0.data(), rx.data(), ru.data(), rf.data()));
    check(hsddp_upload_warm_start(handle, Xb.data(), Ub.data(), K.data()));
    hsddp_stats st;
    check(hsddp_solve(handle, &st));
    std::vector<double> X(24 * S), U(24 * Kc), D(24 * S), dX(24 * S), dU(24 * Kc);
    check(hsddp_download_trajectory(handle, Xb.data(), Ub.data(), K.data()));
    check(hsddp_download_working(handle, X.data(), U.data(), D.data(), dX.data(), dU.data()));
    check(hsddp_download_element_info(handle, &info));
    s = kc = 0;
    for (int i = 0; i < n_phases; ++i) {
        auto &tr = *ph[i]->traj;
        const int N = desc.horizons[i];
        for (int k = 0; k <= N; ++k, ++s)
            for (int j = 0; j < 24; ++j) {
                tr.Xbar[k][j] = Xb[24 * s + j]; tr.X[k][j] = X[24 * s + j];
                tr.Defect[k][j] = D[24 * s + j]; tr.dX[k][j] = dX[24 * s + j];
            }
        for (int k = 0; k < N; ++k, ++kc)
            for (int a = 0; a < 24; ++a) {
                tr.Ubar[k][a] = Ub[24 * kc + a]; tr.U[k][a] = U[24 * kc + a]; tr.dU[k][a] = dU[24 * kc + a];
                for (int b = 0; b < 24; ++b) tr.K[k](a, b) = K[576 * kc + 24 * a + b];
            }
    }
    actual_cost = info.cost;
    feas = info.feas;
    max_tconstr = info.max_tconstr;
    max_pconstr = info.max_pconstr;
}

#endif  // HSDDP_FACADE_HPP
