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
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/hsddp.h"
#include "hsddp_pack.hpp"

// ---- dense containers (Eigen-style access, column-major) -------------------------------------
template <typename T, size_t n>
class VecM;
template <typename T>
class DVec {
public:
    DVec() = default;
    explicit DVec(size_t n) : v_(n, T(0)) {}
    template <size_t n>
    DVec(const VecM<T, n> &v) : v_(v.data(), v.data() + n) {}  // VecM -> DVec, as Eigen assigns
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

// element-wise comparison result (Eigen's cwiseEqual / cwiseNotEqual ... .any() / .all())
template <size_t n>
struct CwiseMask {
    std::array<bool, n> m{};
    bool any() const { for (bool b : m) if (b) return true; return false; }
    bool all() const { for (bool b : m) if (!b) return false; return true; }
};

template <typename T, size_t n>
class VecM {
public:
    typedef T Scalar;
    VecM() { a_.fill(T(0)); }
    VecM(const DVec<T> &v) { for (size_t i = 0; i < n; ++i) a_[i] = i < v.size() ? v[i] : T(0); }  // Eigen's DVec -> VecM
    static VecM Zero() { return VecM(); }
    static constexpr size_t size() { return n; }
    VecM &operator+=(const VecM &o) { for (size_t i = 0; i < n; ++i) a_[i] += o.a_[i]; return *this; }
    template <typename U>
    VecM<U, n> cast() const { VecM<U, n> r; for (size_t i = 0; i < n; ++i) r[i] = static_cast<U>(a_[i]); return r; }
    CwiseMask<n> cwiseEqual(const T &v) const { CwiseMask<n> r; for (size_t i = 0; i < n; ++i) r.m[i] = a_[i] == v; return r; }
    CwiseMask<n> cwiseEqual(const VecM &o) const { CwiseMask<n> r; for (size_t i = 0; i < n; ++i) r.m[i] = a_[i] == o.a_[i]; return r; }
    CwiseMask<n> cwiseNotEqual(const VecM &o) const { CwiseMask<n> r; for (size_t i = 0; i < n; ++i) r.m[i] = a_[i] != o.a_[i]; return r; }
    bool operator==(const VecM &o) const { return a_ == o.a_; }
    bool operator!=(const VecM &o) const { return a_ != o.a_; }
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
    static MatMN Zero() { return MatMN(); }
    static constexpr size_t rows() { return m; }
    MatMN &operator+=(const MatMN &o) { for (size_t i = 0; i < m * n; ++i) a_[i] += o.a_[i]; return *this; }
    void setIdentity() { a_.fill(T(0)); for (size_t i = 0; i < (m < n ? m : n); ++i) (*this)(i, i) = T(1); }
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

template <typename> class MultiPhaseDDP;

// ---- cost / constraint data (HSDDP_CompoundTypes.h:89-150, ConstraintsBase.h:12-86) -----------
template <typename T, size_t xs_, size_t us_, size_t ys_>
struct RCostData {
    T l;
    VecM<T, xs_> lx;
    VecM<T, us_> lu;
    VecM<T, ys_> ly;
    MatMN<T, xs_, xs_> lxx;
    MatMN<T, us_, xs_> lux;
    MatMN<T, us_, us_> luu;
    MatMN<T, ys_, ys_> lyy;
    RCostData() { Zeros(); }
    void Zeros()
    {
        l = 0;
        lx.setZero(); lu.setZero(); ly.setZero(); lxx.setZero(); luu.setZero(); lux.setZero(); lyy.setZero();
    }
    void add(const RCostData &c)
    {
        l += c.l;
        lx += c.lx; lu += c.lu; ly += c.ly; lxx += c.lxx; luu += c.luu; lux += c.lux; lyy += c.lyy;
    }
};

template <typename T, size_t xs_>
struct TCostData {
    T Phi;
    VecM<T, xs_> Phix;
    MatMN<T, xs_, xs_> Phixx;
    TCostData() { Zeros(); }
    void Zeros() { Phi = 0; Phix.setZero(); Phixx.setZero(); }
    void add(const TCostData &c) { Phi += c.Phi; Phix += c.Phix; Phixx += c.Phixx; }
};

template <typename T, size_t xs, size_t us, size_t ys>
struct IneqConstrData {
    T g = 0;
    VecM<T, xs> gx;
    VecM<T, us> gu;
    VecM<T, ys> gy;
    MatMN<T, xs, xs> gxx;
    MatMN<T, us, us> guu;
    MatMN<T, ys, ys> gyy;
    static IneqConstrData Zero() { return IneqConstrData(); }
};

template <typename T, size_t xs>
struct TConstrData {
    T h = 0;
    VecM<T, xs> hx;
    MatMN<T, xs, xs> hxx;
};

template <typename T>
struct AL_Param_Struct {
    T lambda = 0, sigma = 0, sigma_max = 0;
    void update_penalty(T beta) { sigma *= beta; }
    void update_Lagrange(T h) { lambda += h * sigma; }
};

template <typename T>
struct REB_Param_Struct {
    T delta = 0.1, delta_min = 0.01, eps = 1;
    void update_relax(T beta) { delta *= beta; delta = std::fmax(delta, delta_min); }
    void update_weight(T beta) { eps *= beta; }
};

// ---- Trajectory (TrajectoryManagement.h:20-82 / .cpp) ----------------------------------------
// After MultiPhaseDDP::solve: Xbar, Ubar, K, X, U, Defect, Defect_bar, dX, dU, Xsim (= X + Defect),
// A, B and rcostData (the LQ model of the last LQ_approximation), tcostData, G[0] and H[0] (the
// value function at the phase start, get_value_approx).  V, dV and G/H past the first knot are not
// kept by the device solve and stay zero.
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
        const size_t n1 = horizon + 1, n = horizon;
        Xbar.assign(n1, VecM<T, xs>()); X = Xbar; Xsim = Xbar; Defect_bar = Xbar; Defect = Xbar; dX = Xbar; G = Xbar;
        Ubar.assign(n, VecM<T, us>()); U = Ubar; dU = Ubar;
        Y.assign(n, VecM<T, ys>());
        A.assign(n1, MatMN<T, xs, xs>()); H = A;
        B.assign(n, MatMN<T, xs, us>());
        C.assign(n, MatMN<T, ys, xs>());
        D.assign(n, MatMN<T, ys, us>());
        V.assign(n1, T(0)); dV = V;
        K.assign(n1, MatMN<T, us, xs>());
        rcostData.assign(n, RCostData<T, xs, us, ys>());
    }
    void zero_all() { create_data(timeStep, horizon); }
    void clear()
    {
        Xbar.clear(); X.clear(); Ubar.clear(); U.clear(); Y.clear(); Xsim.clear(); Defect_bar.clear(); Defect.clear();
        A.clear(); B.clear(); C.clear(); D.clear(); V.clear(); dV.clear(); dU.clear(); G.clear(); H.clear();
        K.clear(); dX.clear(); rcostData.clear();
    }
    void update_nominal_vals()  // TrajectoryManagement.cpp:110-115
    {
        std::copy(X.begin(), X.end(), Xbar.begin());
        std::copy(U.begin(), U.end(), Ubar.begin());
        std::copy(Defect.begin(), Defect.end(), Defect_bar.begin());
    }
    void pop_front()  // :118-141
    {
        Xbar.pop_front(); X.pop_front(); Ubar.pop_front(); U.pop_front(); Y.pop_front(); Xsim.pop_front();
        Defect.pop_front(); Defect_bar.pop_front(); A.pop_front(); B.pop_front(); C.pop_front(); D.pop_front();
        V.pop_front(); dV.pop_front(); dU.pop_front(); G.pop_front(); H.pop_front(); K.pop_front(); dX.pop_front();
        rcostData.pop_front();
        horizon--;
    }
    void push_back_zero() { push_back_state(DVec<T>(VecM<T, xs>())); }  // :143-166
    void push_back_state(const DVec<T> &state_to_add)                  // :168-191
    {
        Xbar.push_back(VecM<T, xs>(state_to_add)); X.push_back(VecM<T, xs>(state_to_add));
        Ubar.push_back(VecM<T, us>()); U.push_back(VecM<T, us>()); Y.push_back(VecM<T, ys>());
        Xsim.push_back(VecM<T, xs>()); Defect.push_back(VecM<T, xs>()); Defect_bar.push_back(VecM<T, xs>());
        A.push_back(MatMN<T, xs, xs>()); B.push_back(MatMN<T, xs, us>()); C.push_back(MatMN<T, ys, xs>());
        D.push_back(MatMN<T, ys, us>()); V.push_back(T(0)); dV.push_back(T(0)); dU.push_back(VecM<T, us>());
        G.push_back(VecM<T, xs>()); H.push_back(MatMN<T, xs, xs>()); K.push_back(MatMN<T, us, xs>());
        dX.push_back(VecM<T, xs>()); rcostData.push_back(RCostData<T, xs, us, ys>());
        horizon++;
    }
    int size() { return (int)Xbar.size(); }
    void compute_defect()  // :193-199
    {
        for (int k = 0; k <= horizon; ++k)
            for (size_t j = 0; j < xs; ++j) Defect[k][j] = Xsim[k][j] - X[k][j];
    }
    T measure_dynamics_feasibility(int norm_id = 2)  // :201-208 (2-norm of the stacked defects)
    {
        T s = 0, mx = 0;
        for (auto &d : Defect)
            for (size_t j = 0; j < xs; ++j) { s += d[j] * d[j]; mx = std::max(mx, std::fabs(d[j])); }
        return norm_id == 2 ? std::sqrt(s) : mx;
    }

    T duration = 0, timeStep = 0;
    int horizon = 0;
    std::deque<VecM<T, xs>> Xbar, X;
    std::deque<VecM<T, us>> Ubar, U;
    std::deque<VecM<T, ys>> Y;
    std::deque<VecM<T, xs>> Xsim, Defect_bar, Defect;
    std::deque<MatMN<T, xs, xs>> A;
    std::deque<MatMN<T, xs, us>> B;
    std::deque<MatMN<T, ys, xs>> C;
    std::deque<MatMN<T, ys, us>> D;
    std::deque<T> V, dV;
    std::deque<VecM<T, us>> dU;
    std::deque<VecM<T, xs>> G;
    std::deque<MatMN<T, xs, xs>> H;
    std::deque<MatMN<T, us, xs>> K;
    std::deque<VecM<T, xs>> dX;
    std::deque<RCostData<T, xs, us, ys>> rcostData;
    TCostData<T, xs> tcostData;
};

// ---- what a phase's plugins tell the device solve ----------------------------------------------
// The device evaluates the HKD model, costs and constraints in its own kernels, so
// MultiPhaseDDP::solve never calls a plugin per knot.  Instead every plugin that can run there
// describes itself once per solve through the interfaces below (the cost weights it applies, the
// references it reads, its constraint parameters); solve() checks that the phases agree with each
// other and with what one device handle can hold, and refuses anything else.
namespace hsddp_facade {

// Dynamics / reset callbacks are opaque std::functions (a std::bind of HKD::Model<T>::dynamics in
// the reference, HKDProblem.cpp:229-239).  solve() reads the contact and dt they bind by calling
// them once in probe mode: HKD::Model / HKDReset (hkd_trajopt.hpp) record their bound arguments
// instead of evaluating.  A callback that never reaches them is not the HKD model.
enum ProbeKind { PROBE_OFF = 0, PROBE_DYNAMICS, PROBE_DYNAMICS_PARTIAL, PROBE_RESET, PROBE_RESET_PARTIAL };
struct Probe {
    int kind = PROBE_OFF, hits = 0;
    int c[4] = {0, 0, 0, 0}, cn[4] = {0, 0, 0, 0};
    double dt = 0;
    // the objects the model call received (outputs, inputs): a callback that is exactly the HKD
    // registration forwards the solver's own arguments (std::bind forwards references)
    const void *out[2] = {nullptr, nullptr}, *in[2] = {nullptr, nullptr};
};
inline Probe &probe()
{
    thread_local Probe p;
    return p;
}
// record the bound arguments and the forwarded objects when probing for `kind`; true = do not
// evaluate (the outputs stay untouched)
template <typename CV, typename DT>
inline bool probe_record(int kind, const CV &c, const CV *cn, DT dt, const void *out0, const void *out1,
                         const void *in0, const void *in1)
{
    Probe &p = probe();
    if (p.kind != kind) return false;
    ++p.hits;
    for (int l = 0; l < 4; ++l) {
        p.c[l] = (int)c[l];
        p.cn[l] = cn ? (int)(*cn)[l] : 0;
    }
    p.dt = (double)dt;
    p.out[0] = out0; p.out[1] = out1;
    p.in[0] = in0; p.in[1] = in1;
    return true;
}

// One cost term of one phase, as the device evaluates it: the effective weight diagonals under the
// phase's contact (HKDTrackingCost Q, R, Qf: HKDCost.h:14-36; HKDFootPlaceReg Qfoot: HKDCost.h:56-69)
// and the references at knot k / time t of the phase (t = t_offset + k dt, SinglePhase.cpp:243-287).
struct CostSpec {
    int terms = 0;  // HSDDP_TERM_TRACKING and / or HSDDP_TERM_FOOT
    // tracking: Q, R, Qf diagonals (off-diagonal entries must be zero)
    double q[24] = {}, r[24] = {}, qf[24] = {};
    // foot regularisation: Qfoot diagonal, terminal cost / gradient factors (HKDCost.cpp:49,63)
    double qfoot[12] = {}, foot_term_cost = 10, foot_term_grad = 20;
    // the weights themselves when the plugin holds them as hsddp_hkd_weights (hkd:: types)
    const hsddp_hkd_weights *exact = nullptr;
    std::function<void(int k, float t, double *xr, double *ur)> track_ref;
    // foot placements and the body position they are taken relative to (pcom NULL: x_ref's)
    std::function<void(int k, float t, double *pf, double *pcom)> foot_ref;
    bool foot_pcom = false;  // foot_ref writes pcom
    // per-knot reference tables the term holds (-1: looked up by time, any horizon): the solve
    // refuses tables that do not cover the phase (x / foot: N + 1 rows, u: at least N)
    int x_rows = -1, u_rows = -1, foot_rows = -1;
};
struct DeviceCost {
    virtual ~DeviceCost() = default;
    virtual void device_spec(CostSpec &spec, const int *contact) const = 0;
};
// GRFConstraint + its ReB parameters (HKDConstraints.cpp:7-66, ConstraintsBase.h:204-263)
struct GrfSpec {
    int contact[4] = {0, 0, 0, 0};
    double mu = 0.7, delta = 0.1, delta_min = 0.01, eps = 1;
};
struct DevicePathConstraint {
    virtual ~DevicePathConstraint() = default;
    virtual void device_spec(GrfSpec &spec) const = 0;
};
// TouchDownConstraint + its AL parameters (HKDConstraints.cpp:69-171, ConstraintsBase.h:374-399)
struct TdSpec {
    int impact[4] = {0, 0, 0, 0};
    double sigma = 5, lambda = 0, sigma_max = 0, ground = 0;
};
struct DeviceTerminalConstraint {
    virtual ~DeviceTerminalConstraint() = default;
    virtual void device_spec(TdSpec &spec) const = 0;
};

// The weight diagonals the device applies under contact c (q_diag, r_diag, foot_weight and the
// terminal Qf of csrc/hsddp_device.h), in the device's operation order
inline void device_diagonals(const hsddp_hkd_weights &w, const int *c, double *q, double *r, double *qf, double *qfoot)
{
    for (int j = 0; j < 24; ++j) {
        const double qb = j < 3 ? w.q_eul[j] : j < 6 ? w.q_pos[j - 3] : j < 9 ? w.q_omega[j - 6] : j < 12 ? w.q_v[j - 9] : 0.0;
        q[j] = j < 12 ? qb : w.q_qJ * (1 - c[(j - 12) / 3]);
        r[j] = j < 12 ? w.r_grf : w.r_qJd;
        qf[j] = w.qf_gain * w.qf_scale[j] * q[j];
        if (j < 12) qfoot[j] = w.foot_gain * w.foot_w[j % 3] * c[j / 3];
    }
}

// device of the facade's point evaluations (the hkd:: plugin virtuals) on this thread
inline int &device()
{
    thread_local int d = 0;
    return d;
}
inline void set_device(int d) { device() = d; }

}  // namespace hsddp_facade

// ---- plugin bases with the reference's signatures ---------------------------------------------
// CostBase (SinglePhaseInterface.h:35-57).  The solver evaluates costs on the device; a cost runs
// there only when it describes itself to the solve (hsddp_facade::DeviceCost: the hkd:: types
// below, HKDTrackingCost / HKDFootPlaceReg in hkd_trajopt.hpp).
template <typename T, size_t xs_, size_t us_, size_t ys_>
class CostBase {
public:
    typedef VecM<T, xs_> State;
    typedef VecM<T, us_> Contrl;
    typedef VecM<T, ys_> Output;
    typedef RCostData<T, xs_, us_, ys_> RCost;
    typedef TCostData<T, xs_> TCost;

    CostBase(const std::string &cost_name_in) : cost_name(cost_name_in) {}
    virtual ~CostBase() = default;
    virtual void running_cost(RCost &, const State &x, const Contrl &u, const Output &y, T dt, float t) = 0;
    virtual void running_cost_par(RCost &, const State &x, const Contrl &u, const Output &y, T dt, float t) = 0;
    virtual void terminal_cost(TCost &, const State &x, float tend) = 0;
    virtual void terminal_cost_par(TCost &, const State &x, float tend) = 0;

    std::string cost_name;
};

// SinglePhaseReferenceAbstract (SinglePhaseInterface.h:12-34): the reference a tracking cost reads
template <size_t xs, size_t us, size_t ys>
class SinglePhaseReferenceAbstract {
public:
    virtual ~SinglePhaseReferenceAbstract() = default;
    virtual void get_reference_at_t(VecM<double, xs> &xr, VecM<double, us> &ur, VecM<double, ys> &yr, float t)
    {
        (void)xr; (void)ur; (void)yr; (void)t;
        std::printf("Need to wrap around the function get_reference_at_t for your problem \n");
    }
    virtual void get_reference_at_t(VecM<double, xs> &xr, float t)
    {
        (void)xr; (void)t;
        std::printf("Need to wrap around the function get_reference_at_t for your problem \n");
    }
};

// QuadraticCost / QuadraticTrackingCost (SinglePhaseInterface.h:59-134, .cpp:5-118): diagonal-free
// generic weights Q, R, S, Qf.  Their point evaluations are plain host arithmetic (these are the
// solver library's generic plugin bases, not the device path: a phase runs on the device only with
// a cost that describes itself, e.g. HKDTrackingCost, whose Q / R / Qf the solve reads).
template <typename T, size_t xs_, size_t us_, size_t ys_>
class QuadraticCost : public CostBase<T, xs_, us_, ys_> {
public:
    typedef CostBase<T, xs_, us_, ys_> Base;
    using typename Base::State;
    using typename Base::Contrl;
    using typename Base::Output;
    using typename Base::RCost;
    using typename Base::TCost;

    explicit QuadraticCost(const std::string &name = "Quadratic Cost") : Base(name)
    {
        Q.setIdentity(); R.setIdentity(); S.setZero(); Qf.setIdentity();
    }
    void running_cost(RCost &rc, const State &x, const Contrl &u, const Output &y, T dt, float t = 0) override
    {
        (void)t;
        rc.l = dt * (0.5 * quad(Q, x) + 0.5 * quad(R, u) + 0.5 * quad(S, y));
    }
    void running_cost_par(RCost &rc, const State &x, const Contrl &u, const Output &y, T dt, float t = 0) override
    {
        (void)t; (void)y;
        mul(Q, x, dt, rc.lx); mul(R, u, dt, rc.lu);
        scale(Q, dt, rc.lxx); scale(R, dt, rc.luu); rc.lux.setZero();
    }
    void terminal_cost(TCost &tc, const State &x, float tend = 0) override { (void)tend; tc.Phi = 0.5 * quad(Qf, x); }
    void terminal_cost_par(TCost &tc, const State &x, float tend = 0) override
    {
        (void)tend;
        mul(Qf, x, T(1), tc.Phix);
        tc.Phixx = Qf;
    }

protected:
    template <size_t n>
    static T quad(const MatMN<T, n, n> &M, const VecM<T, n> &v)
    {
        T s = 0;
        for (size_t a = 0; a < n; ++a)
            for (size_t b = 0; b < n; ++b) s += v[a] * M(a, b) * v[b];
        return s;
    }
    template <size_t n>
    static void mul(const MatMN<T, n, n> &M, const VecM<T, n> &v, T f, VecM<T, n> &out)
    {
        for (size_t a = 0; a < n; ++a) {
            T s = 0;
            for (size_t b = 0; b < n; ++b) s += M(a, b) * v[b];
            out[a] = f * s;
        }
    }
    template <size_t n>
    static void scale(const MatMN<T, n, n> &M, T f, MatMN<T, n, n> &out)
    {
        for (size_t a = 0; a < n; ++a)
            for (size_t b = 0; b < n; ++b) out(a, b) = f * M(a, b);
    }
    MatMN<T, xs_, xs_> Q;
    MatMN<T, us_, us_> R;
    MatMN<T, ys_, ys_> S;
    MatMN<T, xs_, xs_> Qf;
};

template <typename T, size_t xs_, size_t us_, size_t ys_>
class QuadraticTrackingCost : public QuadraticCost<T, xs_, us_, ys_> {
public:
    typedef QuadraticCost<T, xs_, us_, ys_> Base;
    using typename Base::State;
    using typename Base::Contrl;
    using typename Base::Output;
    using typename Base::RCost;
    using typename Base::TCost;

    explicit QuadraticTrackingCost(const std::string &name = "Quadratic Cost") : Base(name) {}
    void set_reference(SinglePhaseReferenceAbstract<xs_, us_, ys_> *reference_in) { reference = reference_in; }
    SinglePhaseReferenceAbstract<xs_, us_, ys_> *get_reference() const { return reference; }

    void running_cost(RCost &rc, const State &x, const Contrl &u, const Output &y, T dt, float t = 0) override
    {
        State dx;
        Contrl du;
        diff(x, u, t, dx, du);
        Base::running_cost(rc, dx, du, y, dt, t);
    }
    void running_cost_par(RCost &rc, const State &x, const Contrl &u, const Output &y, T dt, float t = 0) override
    {
        State dx;
        Contrl du;
        diff(x, u, t, dx, du);
        Base::running_cost_par(rc, dx, du, y, dt, t);
    }
    void terminal_cost(TCost &tc, const State &x, float tend = 0) override
    {
        State dx;
        Contrl du;
        diff(x, Contrl(), tend, dx, du);
        Base::terminal_cost(tc, dx, tend);
    }
    void terminal_cost_par(TCost &tc, const State &x, float tend = 0) override
    {
        State dx;
        Contrl du;
        diff(x, Contrl(), tend, dx, du);
        Base::terminal_cost_par(tc, dx, tend);
    }

private:
    void diff(const State &x, const Contrl &u, float t, State &dx, Contrl &du) const
    {
        if (!reference) throw std::runtime_error(this->cost_name + ": set_reference was not called");
        VecM<double, xs_> xr;
        VecM<double, us_> ur;
        VecM<double, ys_> yr;
        reference->get_reference_at_t(xr, ur, yr, t);
        for (size_t j = 0; j < xs_; ++j) dx[j] = x[j] - (T)xr[j];
        for (size_t j = 0; j < us_; ++j) du[j] = u[j] - (T)ur[j];
    }
    SinglePhaseReferenceAbstract<xs_, us_, ys_> *reference = nullptr;
};

// PathConstraintBase (ConstraintsBase.h:88-327): per-knot constraint data and ReB parameters, the
// ReB cost / partials, the parameter schedule; compute_violation / compute_partial per knot.
template <typename T, size_t xs_, size_t us_, size_t ys_>
class PathConstraintBase {
public:
    typedef VecM<T, xs_> State;
    typedef VecM<T, us_> Contrl;
    typedef VecM<T, ys_> Output;
    typedef std::vector<IneqConstrData<T, xs_, us_, ys_>> ConstrDataType;
    typedef std::vector<REB_Param_Struct<T>> ReBDataType;

    size_t size = 0, len = 0;
    std::string name;
    std::deque<ConstrDataType> data;
    std::deque<ReBDataType> params;
    REB_Param_Struct<T> param_init;
    T max_violation = 0, ReB_cost = 0;
    VecM<T, us_> ReB_grad_u;
    VecM<T, xs_> ReB_grad_x;
    VecM<T, ys_> ReB_grad_y;
    MatMN<T, us_, us_> ReB_hess_u;
    MatMN<T, xs_, xs_> ReB_hess_x;
    MatMN<T, ys_, ys_> ReB_hess_y;

    PathConstraintBase() = default;
    PathConstraintBase(const std::string &name_) : name(name_) {}
    PathConstraintBase(int size_, int len_, const std::string &name_) : size(size_), len(len_), name(name_) {}
    virtual ~PathConstraintBase() = default;

    void create_data()
    {
        clear_data();
        for (size_t i = 0; i < len; ++i) data.push_back(ConstrDataType(size));
    }
    void clear_data() { data.clear(); }
    void initialize_params(const REB_Param_Struct<T> &p)
    {
        param_init = p;
        params.clear();
        for (size_t k = 0; k < len; ++k) params.push_back(ReBDataType(size, p));
    }
    void initialize_params()
    {
        REB_Param_Struct<T> p;
        p.delta = 0.01; p.delta_min = 0.001; p.eps = 1;
        initialize_params(p);
    }
    void reset_params() {}
    void update_params(T thresh, T beta_relax, T beta_weight)  // :160-176
    {
        for (size_t k = 0; k < len; ++k)
            for (size_t i = 0; i < size; ++i) {
                if (data[k][i].g > -thresh) continue;
                params[k][i].update_weight(beta_weight);
                params[k][i].update_relax(beta_relax);
            }
    }
    void update_horizon_len(int len_) { len = len_; }
    void update_constraint_size(int size_in) { size = size_in; }
    void update_max_violation(int k)  // :187-200
    {
        if (k == 0) max_violation = 0;
        T m = 0;
        for (auto &c : data[k]) m = std::min(m, c.g);
        max_violation = std::min(max_violation, m);
    }
    void compute_ReB_cost(size_t k)  // :201-221
    {
        ReB_cost = 0;
        for (size_t i = 0; i < size; ++i) {
            const T g = data[k][i].g, delta = params[k][i].delta, eps = params[k][i].eps;
            T barr;
            if (g > delta) barr = -std::log(g);
            else barr = .5 * (((g - 2 * delta) / delta) * ((g - 2 * delta) / delta) - 1) - std::log(delta);
            ReB_cost += eps * barr;
        }
    }
    void compute_ReB_partials(size_t k)  // :222-263
    {
        ReB_grad_u.setZero(); ReB_grad_x.setZero(); ReB_grad_y.setZero();
        ReB_hess_u.setZero(); ReB_hess_x.setZero(); ReB_hess_y.setZero();
        for (size_t i = 0; i < size; ++i) {
            const auto &c = data[k][i];
            const T g = c.g, delta = params[k][i].delta, eps = params[k][i].eps;
            const T bd = g > delta ? -1.0 / g : (g - 2 * delta) / delta / delta;
            const T bdd = g > delta ? std::pow(g, -2) : std::pow(delta, -2);
            auto acc = [&](auto &grad, auto &hess, const auto &gv, const auto &gvv, size_t n) {
                for (size_t a = 0; a < n; ++a) {
                    grad[a] += eps * bd * gv[a];
                    for (size_t b = 0; b < n; ++b) hess(a, b) += eps * (bdd * gv[a] * gv[b] + bd * gvv(a, b));
                }
            };
            acc(ReB_grad_u, ReB_hess_u, c.gu, c.guu, us_);
            acc(ReB_grad_x, ReB_hess_x, c.gx, c.gxx, xs_);
            acc(ReB_grad_y, ReB_hess_y, c.gy, c.gyy, ys_);
        }
    }
    // call update_max_violation in compute_violation in the derived class
    virtual void compute_partial(const State &, const Contrl &, const Output &, int k) = 0;
    virtual void compute_violation(const State &, const Contrl &, const Output &, int k) = 0;

    void pop_front() { data.pop_front(); params.pop_front(); len--; }
    void push_back() { data.push_back(ConstrDataType(size)); params.push_back(params.back()); len++; }
    void pop_front_n(int n) { for (int i = 0; i < n; ++i) pop_front(); }
    void push_back_n(int n) { for (int i = 0; i < n; ++i) push_back(); }
};

// TerminalConstraintBase (ConstraintsBase.h:329-405): AL parameters and terms of the phase end.
template <typename T, size_t xs_>
class TerminalConstraintBase {
public:
    typedef VecM<T, xs_> State;
    size_t size = 0;
    std::string name;
    std::vector<TConstrData<T, xs_>> data;
    std::vector<AL_Param_Struct<T>> params;
    AL_Param_Struct<T> param_init;
    T max_violation = 0, AL_cost = 0;
    VecM<T, xs_> AL_gradient;
    MatMN<T, xs_, xs_> AL_hessian;

    TerminalConstraintBase() = default;
    TerminalConstraintBase(const std::string &name_) : name(name_) {}
    TerminalConstraintBase(int size_, const std::string &name_) : size(size_), name(name_) {}
    virtual ~TerminalConstraintBase() = default;

    void create_data() { data = std::vector<TConstrData<T, xs_>>(size); }
    void clear_data() { data.clear(); }
    void resize_data() { data.resize(size); }
    void update_constraint_size(size_t size_) { size = size_; }
    void initialize_params()
    {
        AL_Param_Struct<T> p;
        p.lambda = 0; p.sigma = 5;
        initialize_params(p);
    }
    void initialize_params(const AL_Param_Struct<T> &p) { param_init = p; params.assign(size, p); }
    void reset_params() {}
    void update_params(T thresh, T beta)  // :354-372
    {
        for (size_t i = 0; i < size; ++i) {
            if (std::fabs(data[i].h) < thresh) continue;
            if (std::fabs(data[i].h) > 0.005) {
                params[i].update_penalty(beta);
                params[i].sigma = std::min(params[i].sigma, params[i].sigma_max);
            } else {
                params[i].update_Lagrange(data[i].h);
            }
        }
    }
    void update_max_violation()
    {
        max_violation = 0.0;
        for (auto &c : data) max_violation = std::max(max_violation, (T)std::fabs(c.h));
    }
    void compute_AL_cost()
    {
        AL_cost = 0;
        for (size_t i = 0; i < size; ++i) {
            const T s = params[i].sigma, l = params[i].lambda, h = data[i].h;
            AL_cost += 0.5 * s * h * h;
            AL_cost += l * h;
        }
    }
    void compute_AL_partials()  // quirk A4: (sigma (1 + h) + lambda) hx hx^T
    {
        AL_gradient.setZero();
        AL_hessian.setZero();
        for (size_t i = 0; i < size; ++i) {
            const T s = params[i].sigma, l = params[i].lambda, h = data[i].h;
            const auto &hx = data[i].hx;
            for (size_t a = 0; a < xs_; ++a) {
                AL_gradient[a] += (s * h + l) * hx[a];
                for (size_t b = 0; b < xs_; ++b) AL_hessian(a, b) += (s * (1 + h) + l) * (hx[a] * hx[b]);
            }
        }
    }
    virtual void compute_violation(const State &) = 0;
    virtual void compute_partial(const State &) = 0;
};

// SinglePhaseBase (SinglePhaseBase.h:10-88): the interface MultiPhaseDDP drives per phase.
struct HSDDP_OPTION;
template <typename T>
class SinglePhaseBase {
    friend class MultiPhaseDDP<T>;

public:
    SinglePhaseBase() = default;
    virtual ~SinglePhaseBase() = default;
    virtual void warmstart() = 0;
    virtual void initialization() = 0;
    virtual void set_initial_condition(DVec<T> &x0_) = 0;
    virtual void set_initial_condition(DVec<T> &x0_, DVec<T> &xsim_0_) { (void)x0_; (void)xsim_0_; }
    virtual void set_initial_condition_dx(DVec<T> &dx0_) = 0;
    virtual void set_nominal_initial_condition(DVec<T> &x0_) { (void)x0_; }
    virtual void linear_rollout(T eps, HSDDP_OPTION &) = 0;
    virtual bool hybrid_rollout(T eps, HSDDP_OPTION &, bool is_last_phase = false) = 0;
    virtual void LQ_approximation(HSDDP_OPTION &) = 0;
    virtual bool backward_sweep(T regularization, DVec<T> Gprime, DMat<T> Hprime) = 0;
    virtual DVec<T> resetmap(DVec<T> &) = 0;
    virtual void resetmap_partial(DMat<T> &Px, DVec<T> &x) = 0;
    virtual void get_value_approx(DVec<T> &G, DMat<T> &H) = 0;
    virtual void get_exp_cost_change(T &dV_1, T &dV_2) = 0;
    virtual void get_terminal_state(DVec<T> &xend) = 0;
    virtual void get_terminal_state(DVec<T> &xend, DVec<T> &xsim_end) = 0;
    virtual void get_terminal_state_dx(DVec<T> &dx_end) = 0;
    virtual T get_actual_cost() = 0;
    virtual T get_max_tconstrs() { return (T)(0); }
    virtual T get_max_pconstrs() { return (T)(0); }
    virtual size_t get_state_dim() { return 0; }
    virtual size_t get_control_dim() { return 0; }
    virtual void update_AL_params(HSDDP_OPTION &) {}
    virtual void update_REB_params(HSDDP_OPTION &) {}
    virtual void update_nominal_trajectory() = 0;
    virtual void empty_control() {}
    virtual void push_back_default() {}
    virtual void pop_front() {}
    virtual void reset_params() {}
    virtual T measure_dynamics_feasibility(int norm_id) { (void)norm_id; return 0; }
    virtual void update_SS_config(int ss_sz) { (void)ss_sz; }
    virtual void compute_cost(const HSDDP_OPTION &option) = 0;
    virtual void get_trajectory(std::vector<std::vector<float>> &x_tau, std::vector<std::vector<float>> &u_tau)
    {
        (void)x_tau; (void)u_tau;
    }
    virtual void print() {}
};

template <typename> class MultiPhaseDDP;

// ---- SinglePhase (SinglePhase.h:21-170) -------------------------------------------------------
// The setters HKDProblem calls, and SinglePhaseBase's interface.  The per-phase numerical steps
// (linear / hybrid rollout, LQ approximation, backward sweep, compute_cost) run for all phases at
// once inside the device solve (MultiPhaseDDP::solve); called one phase at a time from the host
// they throw std::logic_error — there is no CPU implementation of them.  The accessors read the
// state the last device solve left in the phase's Trajectory.
template <typename T, size_t xs, size_t us, size_t ys>
class SinglePhase : public SinglePhaseBase<T> {
public:
    typedef VecM<T, xs> State;
    typedef VecM<T, us> Contrl;
    typedef VecM<T, ys> Output;  // zero-size for HKD (ys = 0), as HKD::Model's OutputType
    typedef MatMN<T, xs, xs> StateMap;
    typedef MatMN<T, xs, us> ContrlMap;
    typedef MatMN<T, ys, xs> OutputMap;
    typedef MatMN<T, ys, us> DirectMap;
    friend class MultiPhaseDDP<T>;

    void set_trajectory(std::shared_ptr<Trajectory<T, xs, us, ys>> traj_) { traj = traj_; phase_horizon = traj_->horizon; }
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

    // SinglePhaseBase
    void warmstart() override {}  // the device solve starts from Trajectory::Xbar / Ubar / K
    void initialization() override { SS_set.clear(); }
    void set_initial_condition(DVec<T> &x0_) override { x_init = x0_; }
    void set_initial_condition(DVec<T> &x0_, DVec<T> &xsim_0_) override { x_init = x0_; xsim_init = xsim_0_; }
    void set_initial_condition_dx(DVec<T> &dx0_) override { dx_init = dx0_; }
    void linear_rollout(T, HSDDP_OPTION &) override { device_only("linear_rollout"); }
    bool hybrid_rollout(T, HSDDP_OPTION &, bool = false) override { device_only("hybrid_rollout"); return false; }
    void LQ_approximation(HSDDP_OPTION &) override { device_only("LQ_approximation"); }
    bool backward_sweep(T, DVec<T>, DMat<T>) override { device_only("backward_sweep"); return false; }
    void compute_cost(const HSDDP_OPTION &) override { device_only("compute_cost"); }
    DVec<T> resetmap(DVec<T> &x) override  // SinglePhase.cpp:62-71
    {
        DVec<T> xn(xs);
        if (resetmap_func_handle) resetmap_func_handle(xn, x);
        else xn = x;
        return xn;
    }
    void resetmap_partial(DMat<T> &Px, DVec<T> &x) override  // :73-80
    {
        if (resetmap_partial_func_handle) resetmap_partial_func_handle(Px, x);
        else { Px.setZero(xs, xs); for (size_t i = 0; i < xs; ++i) Px(i, i) = 1; }
    }
    void get_value_approx(DVec<T> &G_out, DMat<T> &H_out) override  // :82-87 (G[0], H[0] of the last sweep)
    {
        G_out = DVec<T>(traj->G[0]);
        H_out.setZero(xs, xs);
        for (size_t a = 0; a < xs; ++a)
            for (size_t b = 0; b < xs; ++b) H_out(a, b) = traj->H[0](a, b);
    }
    void get_exp_cost_change(T &dV_1_out, T &dV_2_out) override { dV_1_out = dV_1; dV_2_out = dV_2; }
    void get_terminal_state(DVec<T> &xend) override { xend = DVec<T>(traj->X.back()); }
    void get_terminal_state(DVec<T> &xend, DVec<T> &xsim_end) override
    {
        xend = DVec<T>(traj->X.back());
        xsim_end = DVec<T>(traj->Xsim.back());
    }
    void get_terminal_state_dx(DVec<T> &dx_end) override { dx_end = DVec<T>(traj->dX.back()); }
    T get_actual_cost() override { return actual_cost; }  // running + terminal cost of the last compute_cost
    size_t get_state_dim() override { return xs; }
    size_t get_control_dim() override { return us; }
    void update_nominal_trajectory() override { traj->update_nominal_vals(); }
    void empty_control() override { for (auto &u : traj->Ubar) u.setZero(); }
    void push_back_default() override  // SinglePhase.cpp:485-491
    {
        traj->push_back_state(DVec<T>(traj->X.back()));
        for (auto &c : pconstraints) c->push_back_n(1);
        phase_horizon = traj->horizon;
    }
    void pop_front() override  // :496-501
    {
        traj->pop_front();
        for (auto &c : pconstraints) c->pop_front_n(1);
        phase_horizon = traj->horizon;
    }
    T measure_dynamics_feasibility(int norm_id) override { return traj->measure_dynamics_feasibility(norm_id); }
    void update_SS_config(int ss_sz) override  // SinglePhase.h:161-164
    {
        SS_set.clear();
        for (int i = 0; i < ss_sz; ++i) SS_set.push_back(i);
    }
    void get_trajectory(std::vector<std::vector<float>> &x_tau, std::vector<std::vector<float>> &u_tau) override
    {
        for (int k = 0; k < phase_horizon; ++k) {
            std::vector<float> xk, uk;
            for (size_t i = 0; i < xs; ++i) xk.push_back((float)traj->X[k][i]);
            for (size_t i = 0; i < us; ++i) uk.push_back((float)traj->U[k][i]);
            x_tau.push_back(xk);
            u_tau.push_back(uk);
        }
    }

    std::vector<int> SS_set;
    int phase_horizon = 0;

private:
    [[noreturn]] static void device_only(const char *what)
    {
        throw std::logic_error(std::string("SinglePhase::") + what +
                               " runs for all phases inside the device solve (MultiPhaseDDP::solve)");
    }
    std::function<void(State &, Output &, State &, Contrl &, T)> dynamics;
    std::function<void(StateMap &, ContrlMap &, OutputMap &, DirectMap &, State &, Contrl &, T)> dynamics_partial;
    std::function<void(DVec<T> &, DVec<T> &)> resetmap_func_handle;
    std::function<void(DMat<T> &, DVec<T> &)> resetmap_partial_func_handle;
    std::vector<std::shared_ptr<CostBase<T, xs, us, ys>>> costs;
    std::vector<std::shared_ptr<PathConstraintBase<T, xs, us, ys>>> pconstraints;
    std::vector<std::shared_ptr<TerminalConstraintBase<T, xs>>> tconstraints;
    std::shared_ptr<Trajectory<T, xs, us, ys>> traj;
    float t_offset = 0;
    DVec<T> x_init, xsim_init, dx_init;
    T actual_cost = 0, dV_1 = 0, dV_2 = 0;
};

// ---- the HKD registrations the device path evaluates ------------------------------------------
namespace hkd {
typedef SinglePhase<double, 24, 24, 0> Phase;
typedef Phase::State State;
typedef Phase::Contrl Contrl;
typedef VecM<double, 0> Output;  // ys = 0: CostBase<double, 24, 24, 0>::Output

namespace detail {
// Point evaluations of the model / plugin primitives from the host (convenience for callers that
// use them one point at a time; the solver never does — it evaluates the model in its kernels).
// Device buffers come from a per-thread arena that only grows, so a call costs its copies and the
// kernel, not allocations.
struct Arena {
    std::vector<std::pair<void *, size_t>> bufs;
    void *get(size_t i, size_t bytes)
    {
        if (bufs.size() <= i) bufs.resize(i + 1, {nullptr, 0});
        if (bufs[i].second < bytes) {
            if (bufs[i].first) hsddp_device_free(bufs[i].first);
            bufs[i].first = hsddp_device_alloc(bytes, hsddp_facade::device());
            bufs[i].second = bufs[i].first ? bytes : 0;
            if (!bufs[i].first) throw std::runtime_error(hsddp_last_error());
        }
        return bufs[i].first;
    }
    ~Arena()
    {
        for (auto &b : bufs)
            if (b.first) hsddp_device_free(b.first);
    }
};
inline Arena &arena()
{
    thread_local Arena a;
    return a;
}
template <typename F>
inline void on_device(const std::vector<std::pair<const void *, size_t>> &in, const std::vector<std::pair<void *, size_t>> &out,
                      F call)
{
    std::vector<void *> din, dout;
    size_t slot = 0;
    for (auto &b : in) {
        void *p = arena().get(slot++, b.second);
        if (hsddp_memcpy_h2d(p, b.first, b.second) != HSDDP_OK) throw std::runtime_error(hsddp_last_error());
        din.push_back(p);
    }
    for (auto &b : out) dout.push_back(arena().get(slot++, b.second));
    const int rc = call(din, dout);
    if (rc == HSDDP_OK) hsddp_device_synchronize(hsddp_facade::device());
    for (size_t i = 0; i < out.size() && rc == HSDDP_OK; ++i) hsddp_memcpy_d2h(out[i].first, dout[i], out[i].second);
    if (rc != HSDDP_OK) throw std::runtime_error(hsddp_last_error());
}
// knot index of time t on a grid starting at t0 with step dt (the references are held per knot)
inline size_t knot_at(float t, float t0, double dt, size_t n)
{
    const long k = std::lround(((double)t - (double)t0) / dt);
    return (size_t)std::min<long>(std::max<long>(k, 0), (long)n - 1);
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

// The HKD costs as CostBase plugins (HKDCost.h:8-99).  The references are held per knot of the
// phase (x_ref, u_ref, foot_ref: horizon + 1 rows), looked up at t = t_start + k knot_dt (the
// reference's costs look them up by time through HKDSinglePhaseReference / QuadReference).
// Weights are shared by every phase of a problem.  Their virtuals evaluate on the device
// (hsddp_hkd_running_cost / hsddp_hkd_terminal_cost) with the solver's own term formulas.
struct HKDCostRefs {
    std::array<int, 4> contact{};
    std::vector<std::array<double, 24>> x_ref;   // horizon + 1 states
    std::vector<std::array<double, 24>> u_ref;   // horizon + 1 (the last is unused, as the reference's lookup)
    std::vector<std::array<double, 12>> foot_ref;  // horizon + 1 (HKDFootPlaceReg)
    float t_start = 0;
    double knot_dt = 0.01;
};
template <int TERMS>
struct HKDCostTerm : CostBase<double, 24, 24, 0>, HKDCostRefs, hsddp_facade::DeviceCost {
    hsddp_hkd_weights weights;  // TrackingCost: its tracking fields apply; FootPlaceReg: its foot fields
    explicit HKDCostTerm(const std::string &name) : CostBase<double, 24, 24, 0>(name) { hsddp_default_weights(&weights); }

    // the device solve reads this term's weights and its per-knot references (knot k of the phase)
    void device_spec(hsddp_facade::CostSpec &spec, const int *c) const override
    {
        spec.terms = TERMS;
        spec.exact = &weights;
        double qfoot[12];
        hsddp_facade::device_diagonals(weights, c, spec.q, spec.r, spec.qf, qfoot);
        if (TERMS & HSDDP_TERM_FOOT) {
            std::copy(qfoot, qfoot + 12, spec.qfoot);
            spec.foot_term_cost = weights.foot_term_cost;
            spec.foot_term_grad = weights.foot_term_grad;
        }
        // row counts checked against the phase horizon by the solve (describe) before any lookup
        if (TERMS & HSDDP_TERM_TRACKING) {
            spec.x_rows = (int)x_ref.size();
            spec.u_rows = (int)u_ref.size();
            spec.track_ref = [this](int k, float, double *xr, double *ur) {
                for (int j = 0; j < 24; ++j) { xr[j] = x_ref[k][j]; ur[j] = k < (int)u_ref.size() ? u_ref[k][j] : 0.0; }
            };
        }
        if (TERMS & HSDDP_TERM_FOOT) {
            spec.foot_rows = (int)foot_ref.size();
            spec.foot_ref = [this](int k, float, double *pf, double *) {
                for (int j = 0; j < 12; ++j) pf[j] = foot_ref[k][j];
            };
        }
    }

    void running_cost(RCost &rc, const State &x, const Contrl &u, const Output &, double dt, float t) override
    {
        eval_running(rc, x, u, dt, t, false);
    }
    void running_cost_par(RCost &rc, const State &x, const Contrl &u, const Output &, double dt, float t) override
    {
        eval_running(rc, x, u, dt, t, true);
    }
    void terminal_cost(TCost &tc, const State &x, float tend) override { eval_terminal(tc, x, tend, false); }
    void terminal_cost_par(TCost &tc, const State &x, float tend) override { eval_terminal(tc, x, tend, true); }

private:
    void refs_at(float t, std::array<double, 24> &xr, std::array<double, 24> &ur, std::array<double, 12> &pf) const
    {
        const size_t n = x_ref.size();
        if (!n) throw std::runtime_error(cost_name + ": no references set");
        const size_t k = detail::knot_at(t, t_start, knot_dt, n);
        xr = x_ref[k];
        ur = k < u_ref.size() ? u_ref[k] : std::array<double, 24>{};
        pf = k < foot_ref.size() ? foot_ref[k] : std::array<double, 12>{};
    }
    // running_cost fills l, running_cost_par the derivatives (HKDCost.cpp:5-33, 40-48 pattern)
    void eval_running(RCost &rc, const State &x, const Contrl &u, double dt, float t, bool par) const
    {
        std::array<double, 24> xr, ur;
        std::array<double, 12> pf;
        refs_at(t, xr, ur, pf);
        double l = 0, lxx[576], luu[576];
        detail::on_device({{x.data(), 192}, {u.data(), 192}, {contact.data(), 16}, {xr.data(), 192}, {ur.data(), 192},
                           {pf.data(), 96}},
                          {{&l, 8}, {rc.lx.data(), 192}, {rc.lu.data(), 192}, {lxx, 4608}, {luu, 4608}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_running_cost((double *)i[0], (double *)i[1], (int *)i[2], (double *)i[3],
                                                            (double *)i[4], (double *)i[5], &weights, dt, TERMS,
                                                            (double *)o[0], (double *)o[1], (double *)o[2],
                                                            (double *)o[3], (double *)o[4], 1, nullptr);
                          });
        if (!par) { rc.l = l; return; }
        std::memcpy(rc.lxx.data(), lxx, sizeof lxx);
        std::memcpy(rc.luu.data(), luu, sizeof luu);
        rc.lux.setZero();
    }
    void eval_terminal(TCost &tc, const State &x, float tend, bool par) const
    {
        std::array<double, 24> xr, ur;
        std::array<double, 12> pf;
        refs_at(tend, xr, ur, pf);
        double Phi = 0, Phixx[576];
        std::array<double, 24> Phix{};
        detail::on_device({{x.data(), 192}, {contact.data(), 16}, {xr.data(), 192}, {pf.data(), 96}},
                          {{&Phi, 8}, {Phix.data(), 192}, {Phixx, 4608}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_terminal_cost((double *)i[0], (int *)i[1], (double *)i[2], (double *)i[3],
                                                             &weights, TERMS, (double *)o[0], (double *)o[1],
                                                             (double *)o[2], 1, nullptr);
                          });
        if (!par) { tc.Phi = Phi; return; }
        for (int j = 0; j < 24; ++j) tc.Phix[j] = Phix[j];
        std::memcpy(tc.Phixx.data(), Phixx, sizeof Phixx);
    }
};
// HKDTrackingCost (HKDCost.h:8-38) and HKDFootPlaceReg (HKDCost.h:40-99, HKDCost.cpp:5-63)
struct TrackingCost : HKDCostTerm<HSDDP_TERM_TRACKING> {
    TrackingCost() : HKDCostTerm("HKD Tracking Cost") {}
};
struct FootPlaceReg : HKDCostTerm<HSDDP_TERM_FOOT> {
    FootPlaceReg() : HKDCostTerm("HKD Foot Placement Regularization") {}
};

// GRFConstraint + ReB (HKDConstraints.h:8-27, HKDConstraints.cpp:7-66; ConstraintsBase.h:204-263):
// 5 friction-pyramid rows per stance leg
struct GRFConstraint : PathConstraintBase<double, 24, 24, 0>, hsddp_facade::DevicePathConstraint {
    hsddp_constraint_params cparams;  // mu_fric and the GRF_ReB parameters apply
    std::array<int, 4> ctact_status{{1, 1, 1, 1}};
    GRFConstraint() : PathConstraintBase("GRF") { hsddp_default_constraint_params(&cparams); set_contact(ctact_status); }
    explicit GRFConstraint(const std::array<int, 4> &ctact) : GRFConstraint() { set_contact(ctact); }
    void set_contact(const std::array<int, 4> &ctact)
    {
        ctact_status = ctact;
        int n = 0;
        for (int l = 0; l < 4; ++l) n += ctact[l] > 0;
        update_constraint_size(5 * n);
    }
    void set_friction_coefficient(double mu) { cparams.mu_fric = mu; }
    void device_spec(hsddp_facade::GrfSpec &spec) const override
    {
        for (int l = 0; l < 4; ++l) spec.contact[l] = ctact_status[l];
        spec.mu = cparams.mu_fric;
        spec.delta = cparams.grf_delta; spec.delta_min = cparams.grf_delta_min; spec.eps = cparams.grf_eps;
    }
    void compute_violation(const State &, const Contrl &u, const Output &, int k) override
    {
        if (data.empty()) create_data();
        double g[20], gu[480];
        eval(u, g, gu);
        for (size_t i = 0; i < data[k].size(); ++i) data[k][i].g = g[i];
        update_max_violation(k);
    }
    void compute_partial(const State &, const Contrl &u, const Output &, int k) override
    {
        double g[20], gu[480];
        eval(u, g, gu);
        for (size_t i = 0; i < data[k].size(); ++i)
            for (int j = 0; j < 24; ++j) data[k][i].gu[j] = gu[24 * i + j];
    }

private:
    void eval(const Contrl &u, double *g, double *gu) const
    {
        detail::on_device({{u.data(), 192}, {ctact_status.data(), 16}}, {{g, 160}, {gu, 3840}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_grf_constraint((double *)i[0], (int *)i[1], cparams.mu_fric,
                                                              (double *)o[0], (double *)o[1], 1, nullptr);
                          });
    }
};
// TouchDownConstraint + AL (HKDConstraints.h:29-51, HKDConstraints.cpp:69-171;
// ConstraintsBase.h:374-399).  next_contact: the contact after the phase (the legs touching down
// are those with contact 0 now and 1 next); ctor(impact_status) as the reference's.
struct TouchDownConstraint : TerminalConstraintBase<double, 24>, hsddp_facade::DeviceTerminalConstraint {
    std::array<int, 4> contact{}, next_contact{};
    double ground_height = 0;
    TouchDownConstraint() : TerminalConstraintBase("TouchDwon") {}
    // AL parameters: initialize_params' (ConstraintsBase.h:349-353), else the constraint_params.info defaults
    void device_spec(hsddp_facade::TdSpec &spec) const override
    {
        for (int l = 0; l < 4; ++l) spec.impact[l] = contact[l] == 0 && next_contact[l] == 1;
        hsddp_constraint_params cp;
        hsddp_default_constraint_params(&cp);
        const bool set = !params.empty();
        spec.sigma = set ? param_init.sigma : cp.td_sigma;
        spec.lambda = set ? param_init.lambda : cp.td_lambda;
        spec.sigma_max = set ? param_init.sigma_max : cp.td_sigma_max;
        spec.ground = ground_height;
    }
    explicit TouchDownConstraint(const std::array<int, 4> &impact_status) : TouchDownConstraint()
    {
        for (int l = 0; l < 4; ++l) { contact[l] = impact_status[l] ? 0 : 1; next_contact[l] = 1; }
        size_t n = 0;
        for (int l = 0; l < 4; ++l) n += impact_status[l] != 0;
        update_constraint_size(n);
    }
    void update_ground_height(double g) { ground_height = g; }
    void compute_violation(const State &x) override
    {
        double h[4], hx[96];
        eval(x, h, hx);
        if (data.size() != size) create_data();
        for (size_t i = 0; i < size; ++i) data[i].h = h[i];
        update_max_violation();
    }
    void compute_partial(const State &x) override
    {
        double h[4], hx[96];
        eval(x, h, hx);
        if (data.size() != size) create_data();
        for (size_t i = 0; i < size; ++i)
            for (int j = 0; j < 24; ++j) data[i].hx[j] = hx[24 * i + j];
    }

private:
    void eval(const State &x, double *h, double *hx) const
    {
        detail::on_device({{x.data(), 192}, {contact.data(), 16}, {next_contact.data(), 16}}, {{h, 32}, {hx, 768}},
                          [&](std::vector<void *> &i, std::vector<void *> &o) {
                              return hsddp_hkd_touchdown_constraint((double *)i[0], (int *)i[1], (int *)i[2], ground_height,
                                                                    (double *)o[0], (double *)o[1], 1, nullptr);
                          });
    }
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
    // extension: the HIP device this solver runs on (default 0)
    void set_device(int d) { device = d; }

    // MultiPhaseDDP::solve (MultiPhaseDDP.cpp:232-428) for this one trajectory on the GPU; afterwards
    // every phase's Trajectory holds the solution, the working trajectory, the LQ model and terminal
    // data of the last LQ_approximation and the value function at the phase start
    void solve(HSDDP_OPTION option);

    // The device problem the phases describe (no device work): descriptor (layout, dt, weights,
    // ReB / AL parameters), contacts [P+1][4], per-slot references and the warm start.  solve()
    // uploads exactly this; it throws std::runtime_error for anything one device handle cannot
    // hold or that is not the HKD problem.
    struct Problem {
        hsddp_problem_desc desc;
        int S = 0, Kc = 0;
        std::vector<int> shooting;  // [P]: SS_set = {0 .. shooting[i] - 1}
        // constraint parameters (hsddp_upload_constraint_params): touchdown legs [P][HSDDP_MAX_TD],
        // AL sigma / lambda [P][HSDDP_MAX_TD][4], ReB delta / eps [Kc][20]
        std::vector<int> td_legs;
        std::vector<double> al_sigma, al_lambda, reb_delta, reb_eps;
        std::vector<int> contacts;
        std::vector<double> ref_x, ref_u, ref_foot, Xbar, Ubar, K;
    };
    Problem describe();

    T get_actual_cost() { return actual_cost; }
    T measure_dynamics_feasibility(int = 2) { return feas; }
    // the per-iteration buffers (MultiPhaseDDP.cpp:532-541): the initial entry and one per inner
    // iteration that passed the later-termination test (:277-280, 368-371)
    void get_solver_info(std::vector<float> &cost_out, std::vector<float> &dyn_feas_out,
                         std::vector<float> &eqn_feas_out, std::vector<float> &ineq_feas_out)
    {
        cost_out = cost_buffer;
        dyn_feas_out = dyn_feas_buffer;
        eqn_feas_out = eqn_feas_buffer;
        ineq_feas_out = ineq_feas_buffer;
    }
    // per-element outcome of the last solve (hsddp_element_info)
    const hsddp_element_info &element_info() const { return info; }

private:
    typedef hkd::Phase Phase;
    struct Bound {  // the arguments a dynamics / reset registration binds
        int c[4] = {0, 0, 0, 0}, cn[4] = {0, 0, 0, 0};
        double dt = 0;
    };
    // Device handles outlive the solver object: HKDMPCSolver::update builds a new MultiPhaseDDP for
    // every MPC tick (HKDMPC.cpp:127-131), so a released handle is parked in a small process-wide
    // pool and the next solver with the same descriptor (weights, parameters, Kc, device; any
    // layout) takes it over instead of allocating and capturing again.  The pool is never torn
    // down (no HIP calls during static destruction); it holds at most kPoolSize handles.
    struct PoolEntry {
        hsddp_problem_desc key;
        int Kc;
        hsddp_handle h;
    };
    static constexpr size_t kPoolSize = 2;
    static std::mutex &pool_mutex()
    {
        static std::mutex *m = new std::mutex;
        return *m;
    }
    static std::vector<PoolEntry> &pool()
    {
        static std::vector<PoolEntry> *p = new std::vector<PoolEntry>;
        return *p;
    }
    static std::atomic<int> &creations()
    {
        static std::atomic<int> *n = new std::atomic<int>(0);
        return *n;
    }
    void release()
    {
        if (!handle) return;
        std::lock_guard<std::mutex> lk(pool_mutex());
        auto &pl = pool();
        if (pl.size() < kPoolSize) pl.push_back({handle_desc, handle_Kc, handle});
        else hsddp_destroy(handle);
        handle = nullptr;
    }
    // a pooled handle for (key, Kc), or a new one
    void acquire(const hsddp_problem_desc &full, const hsddp_problem_desc &key, int Kc)
    {
        {
            std::lock_guard<std::mutex> lk(pool_mutex());
            auto &pl = pool();
            for (size_t j = 0; j < pl.size(); ++j)
                if (pl[j].Kc == Kc && !std::memcmp(&pl[j].key, &key, sizeof key)) {
                    handle = pl[j].h;
                    pl.erase(pl.begin() + j);
                    break;
                }
        }
        if (!handle) {
            check(hsddp_create(&full, &handle));
            ++creations();
            check(hsddp_set_value_export(handle, 1));  // G[0], H[0] per phase for get_value_approx
        }
        handle_desc = key;
        handle_Kc = Kc;
    }
    static void check(int rc)
    {
        if (rc != HSDDP_OK) throw std::runtime_error(std::string("hsddp: ") + hsddp_last_error());
    }
    [[noreturn]] static void refuse(int i, const std::string &what)
    {
        throw std::runtime_error("phase " + std::to_string(i) + ": " + what);
    }
    // call a registered callback once in probe mode: true when it is exactly the HKD model / reset
    // registration — it reaches the model once, forwards the solver's own output and input objects
    // (outs, ins: what the model call must receive) and leaves the outputs as they were (the model
    // does not evaluate in probe mode, so any write is the callback's own logic).  A callback that
    // transforms x / u or post-processes the model's result would be dropped by the device solve,
    // so it is refused.
    template <typename F, typename... A>
    static bool probe_call(int kind, const F &f, Bound &out, std::array<const void *, 2> outs,
                           std::array<const void *, 2> ins, const std::function<bool()> &outputs_untouched,
                           A &...args)
    {
        if (!f) return false;
        struct Guard {
            ~Guard() { hsddp_facade::probe().kind = hsddp_facade::PROBE_OFF; }
        } guard;
        hsddp_facade::Probe &p = hsddp_facade::probe();
        p.kind = kind;
        p.hits = 0;
        try {
            f(args...);
        } catch (...) {
            return false;
        }
        if (p.hits != 1) return false;
        for (int j = 0; j < 2; ++j)
            if (p.out[j] != outs[j] || p.in[j] != ins[j]) return false;
        if (!outputs_untouched()) return false;
        for (int l = 0; l < 4; ++l) { out.c[l] = p.c[l]; out.cn[l] = p.cn[l]; }
        out.dt = p.dt;
        return true;
    }
    // a recognisable fill for the probe's output objects (alternating signs, so that clamps in
    // either direction show up)
    static double probe_fill(size_t j) { return (j & 1 ? -1234.5678125 : 1234.5678125) * (1.0 + j / 64.0); }
    template <typename M>
    static void fill(M &m, size_t n)
    {
        for (size_t j = 0; j < n; ++j) m.data()[j] = probe_fill(j);
    }
    template <typename M>
    static bool filled(const M &m, size_t n)
    {
        for (size_t j = 0; j < n; ++j)
            if (m.data()[j] != probe_fill(j)) return false;
        return true;
    }
    static bool read_dynamics(const Phase &ph, Bound &b);
    static bool read_dynamics_partial(const Phase &ph, Bound &b);
    static int read_reset(const Phase &ph, Bound &b);  // 0: none registered, 1: read, -1: not HKDReset
    void write_back_constraints(const Problem &pr);
    static hsddp_hkd_weights derive_weights(const std::vector<hsddp_facade::CostSpec> &track,
                                            const std::vector<hsddp_facade::CostSpec> &foot,
                                            const std::vector<int> &contacts);

    std::deque<std::shared_ptr<SinglePhaseBase<T>>> phases;
    int n_phases = 0, device = 0;
    DVec<T> x0;
    T actual_cost = 0, feas = 0, max_pconstr = 0, max_tconstr = 0;
    std::vector<float> cost_buffer, dyn_feas_buffer, eqn_feas_buffer, ineq_feas_buffer;
    hsddp_element_info info{};
    hsddp_handle handle = nullptr;
    hsddp_problem_desc handle_desc{};  // the live handle's descriptor without its layout
    int handle_Kc = 0;

public:
    // extension: device handles the process's solvers have created so far
    static int handle_creations() { return creations().load(); }
};

template <typename T>
bool MultiPhaseDDP<T>::read_dynamics(const Phase &ph, Bound &b)
{
    if (const auto *d = ph.dynamics.template target<hkd::Dynamics>()) {
        for (int l = 0; l < 4; ++l) b.c[l] = d->contact[l];
        b.dt = d->dt;
        return true;
    }
    typename Phase::State xn, x;
    typename Phase::Output y;
    typename Phase::Contrl u;
    double t = 0;
    fill(xn, 24);
    return probe_call(hsddp_facade::PROBE_DYNAMICS, ph.dynamics, b, {&xn, nullptr}, {&x, &u},
                      [&] { return filled(xn, 24); }, xn, y, x, u, t);
}

template <typename T>
bool MultiPhaseDDP<T>::read_dynamics_partial(const Phase &ph, Bound &b)
{
    if (const auto *d = ph.dynamics_partial.template target<hkd::DynamicsPartial>()) {
        for (int l = 0; l < 4; ++l) b.c[l] = d->contact[l];
        b.dt = d->dt;
        return true;
    }
    typename Phase::StateMap A;
    typename Phase::ContrlMap B;
    typename Phase::OutputMap C;
    typename Phase::DirectMap D;
    typename Phase::State x;
    typename Phase::Contrl u;
    double t = 0;
    fill(A, 576);
    fill(B, 576);
    return probe_call(hsddp_facade::PROBE_DYNAMICS_PARTIAL, ph.dynamics_partial, b, {&A, &B}, {&x, &u},
                      [&] { return filled(A, 576) && filled(B, 576); }, A, B, C, D, x, u, t);
}

template <typename T>
int MultiPhaseDDP<T>::read_reset(const Phase &ph, Bound &b)
{
    const auto &f = ph.resetmap_func_handle;
    const auto &fp = ph.resetmap_partial_func_handle;
    if (!f && !fp) return 0;
    Bound bp;
    if (const auto *r = f.template target<hkd::Resetmap>()) {
        for (int l = 0; l < 4; ++l) { b.c[l] = r->contact[l]; b.cn[l] = r->next_contact[l]; }
    } else {
        DVec<double> xn(24), x(24);
        fill(xn, 24);
        if (!probe_call(hsddp_facade::PROBE_RESET, f, b, {&xn, nullptr}, {&x, nullptr},
                        [&] { return xn.size() == 24 && filled(xn, 24); }, xn, x))
            return -1;
    }
    if (const auto *r = fp.template target<hkd::ResetmapPartial>()) {
        for (int l = 0; l < 4; ++l) { bp.c[l] = r->contact[l]; bp.cn[l] = r->next_contact[l]; }
    } else {
        DMat<double> Px(24, 24);
        DVec<double> x(24);
        fill(Px, 576);
        if (!probe_call(hsddp_facade::PROBE_RESET_PARTIAL, fp, bp, {&Px, nullptr}, {&x, nullptr},
                        [&] { return Px.rows() == 24 && Px.cols() == 24 && filled(Px, 576); }, Px, x))
            return -1;
    }
    for (int l = 0; l < 4; ++l)
        if (b.c[l] != bp.c[l] || b.cn[l] != bp.cn[l]) return -1;
    return 1;
}

// One hsddp_hkd_weights that reproduces every phase's effective diagonals bit for bit (the device
// holds one weight set per handle and masks it by each phase's contact).  Terms holding their weights
// as hsddp_hkd_weights (hkd::) give them directly; for the reference's classes (Q, R, Qf, Qfoot
// matrices) the gains keep their default and each scale is the quotient that reproduces the product
// the device forms.
template <typename T>
hsddp_hkd_weights MultiPhaseDDP<T>::derive_weights(const std::vector<hsddp_facade::CostSpec> &track,
                                                   const std::vector<hsddp_facade::CostSpec> &foot,
                                                   const std::vector<int> &contacts)
{
    hsddp_hkd_weights w;
    hsddp_default_weights(&w);
    const int P = (int)track.size();
    // the factor f with g * f == target (g * f rounded): the default when it does, else near target / g
    auto factor = [](double g, double target, double dflt) {
        if (target == 0 || g * dflt == target) return dflt;
        const double f0 = target / g;
        for (double f : {f0, std::nextafter(f0, 1e300), std::nextafter(f0, -1e300)})
            if (g * f == target) return f;
        return f0;
    };
    if (track[0].exact) {
        const hsddp_hkd_weights &e = *track[0].exact;
        std::memcpy(w.q_eul, e.q_eul, sizeof w.q_eul); std::memcpy(w.q_pos, e.q_pos, sizeof w.q_pos);
        std::memcpy(w.q_omega, e.q_omega, sizeof w.q_omega); std::memcpy(w.q_v, e.q_v, sizeof w.q_v);
        w.q_qJ = e.q_qJ; std::memcpy(w.qf_scale, e.qf_scale, sizeof w.qf_scale); w.qf_gain = e.qf_gain;
        w.r_grf = e.r_grf; w.r_qJd = e.r_qJd;
    } else {
        const double *q = track[0].q;
        for (int a = 0; a < 3; ++a) { w.q_eul[a] = q[a]; w.q_pos[a] = q[3 + a]; w.q_omega[a] = q[6 + a]; w.q_v[a] = q[9 + a]; }
        w.r_grf = track[0].r[0];
        w.r_qJd = track[0].r[12];
        bool qj = false;
        for (int i = 0; i < P && !qj; ++i)
            for (int l = 0; l < 4 && !qj; ++l)
                if (!contacts[4 * i + l]) { w.q_qJ = track[i].q[12 + 3 * l]; qj = true; }
        // the device forms (qf_gain * qf_scale) * q: the scale whose product rounds to Qf
        for (int j = 0; j < 24; ++j)
            for (int i = 0; i < P; ++i)
                if (track[i].q[j] != 0) {
                    const double tq = track[i].qf[j], qq = track[i].q[j], s0 = tq / qq / w.qf_gain;
                    for (double s : {w.qf_scale[j], s0, std::nextafter(s0, 1e300), std::nextafter(s0, -1e300)})
                        if (w.qf_gain * s * qq == tq) { w.qf_scale[j] = s; break; }
                    break;
                }
    }
    if (foot[0].exact) {
        const hsddp_hkd_weights &e = *foot[0].exact;
        std::memcpy(w.foot_w, e.foot_w, sizeof w.foot_w);
        w.foot_gain = e.foot_gain;
    } else {
        for (int a = 0; a < 3; ++a)
            for (int i = 0; i < P; ++i) {
                int l = 0;
                while (l < 4 && !contacts[4 * i + l]) ++l;
                if (l < 4) { w.foot_w[a] = factor(w.foot_gain, foot[i].qfoot[3 * l + a], w.foot_w[a]); break; }
            }
    }
    w.foot_term_cost = foot[0].foot_term_cost;
    w.foot_term_grad = foot[0].foot_term_grad;
    // every phase's diagonals as the device forms them from w
    for (int i = 0; i < P; ++i) {
        double q[24], r[24], qf[24], qfoot[12];
        hsddp_facade::device_diagonals(w, &contacts[4 * i], q, r, qf, qfoot);
        for (int j = 0; j < 24; ++j)
            if (q[j] != track[i].q[j] || r[j] != track[i].r[j] || qf[j] != track[i].qf[j])
                refuse(i, "tracking weights (Q, R, Qf) differ from the other phases' or are not the HKD pattern "
                          "(diagonal, qJ weighted on swing legs only): one device handle holds one weight set");
        for (int j = 0; j < 12; ++j)
            if (qfoot[j] != foot[i].qfoot[j])
                refuse(i, "foot-placement weights (Qfoot) differ from the other phases' or are not the HKD pattern");
        if (foot[i].foot_term_cost != w.foot_term_cost || foot[i].foot_term_grad != w.foot_term_grad)
            refuse(i, "foot-placement terminal factors differ from the other phases'");
    }
    return w;
}

template <typename T>
typename MultiPhaseDDP<T>::Problem MultiPhaseDDP<T>::describe()
{
    static_assert(std::is_same<T, double>::value, "the device path computes in fp64");
    if (n_phases < 1 || n_phases > HSDDP_MAX_PHASES) throw std::runtime_error("hsddp: 1..16 phases supported");
    if (x0.size() != 24) throw std::runtime_error("hsddp: set_initial_condition needs a 24-state x0");
    const int P = n_phases;
    Problem pr;
    std::memset(&pr.desc, 0, sizeof pr.desc);
    hsddp_problem_desc &desc = pr.desc;
    desc.device = device;
    desc.batch = 1;
    desc.n_phases = P;
    desc.ref_per_element = 0;
    hsddp_default_constraint_params(&desc.cparams);
    std::vector<Phase *> ph(P);
    std::vector<std::shared_ptr<Trajectory<double, 24, 24, 0>>> trajs(P);
    std::vector<Bound> dyn(P), rst(P);
    std::vector<int> has_reset(P);
    pr.contacts.assign(4 * (P + 1), 0);
    for (int i = 0; i < P; ++i) {
        ph[i] = dynamic_cast<Phase *>(phases[i].get());
        if (!ph[i]) refuse(i, "is not SinglePhase<double,24,24,0>");
        trajs[i] = ph[i]->traj;
        if (!trajs[i]) refuse(i, "has no trajectory (set_trajectory)");
        Bound dp;
        if (!read_dynamics(*ph[i], dyn[i]))
            refuse(i, "Dynamics is not the HKD registration (hkd::Dynamics, or HKD::Model<T>::dynamics bound to the "
                      "phase contact and dt); only HKD problems run on the device");
        if (!read_dynamics_partial(*ph[i], dp))
            refuse(i, "DynamicsPartial is not the HKD registration (hkd::DynamicsPartial, or "
                      "HKD::Model<T>::dynamics_partial); only HKD problems run on the device");
        for (int l = 0; l < 4; ++l)
            if (dp.c[l] != dyn[i].c[l] || (dyn[i].c[l] != 0 && dyn[i].c[l] != 1))
                refuse(i, "dynamics and dynamics_partial bind different contacts (or a contact other than 0 / 1)");
        if (dp.dt != dyn[i].dt || dyn[i].dt != (double)trajs[i]->timeStep || dyn[i].dt != dyn[0].dt)
            refuse(i, "the dynamics' dt must equal the trajectory time step of every phase");
        for (int l = 0; l < 4; ++l) pr.contacts[4 * i + l] = dyn[i].c[l];
        has_reset[i] = read_reset(*ph[i], rst[i]);
        if (has_reset[i] < 0) refuse(i, "resetmap / resetmap_partial is not the HKD registration (hkd::Resetmap, or "
                                        "HKDReset<T>::resetmap(_partial) bound to the phase's contacts)");
        if (has_reset[i])
            for (int l = 0; l < 4; ++l)
                if (rst[i].c[l] != dyn[i].c[l]) refuse(i, "the resetmap's current contact differs from the dynamics'");
    }
    // terminal constraints: every phase's TouchDownConstraint objects in registration order, each
    // with its legs and its current AL parameters (TerminalConstraintBase::params, one row per leg in
    // leg order).  HKDProblem::update registers one more on the last phase at every step after it
    // has reached its end (HKDProblem.cpp:199-202), and the parameters evolve across MPC ticks
    // (reset_params is a no-op), so the solve uploads them and writes the updated ones back.
    hsddp_constraint_params cp0;
    hsddp_default_constraint_params(&cp0);
    pr.td_legs.assign((size_t)P * HSDDP_MAX_TD, 0);
    pr.al_sigma.assign((size_t)P * HSDDP_MAX_TD * 4, cp0.td_sigma);
    pr.al_lambda.assign((size_t)P * HSDDP_MAX_TD * 4, cp0.td_lambda);
    hsddp_facade::TdSpec td0;
    bool td_seen = false;
    for (int i = 0; i < P; ++i) {
        int slot = 0;
        for (auto &c : ph[i]->tconstraints) {
            const auto *dc = dynamic_cast<const hsddp_facade::DeviceTerminalConstraint *>(c.get());
            if (!dc) refuse(i, "terminal constraint '" + c->name + "' cannot run on the device");
            hsddp_facade::TdSpec s;
            dc->device_spec(s);
            int mask = 0, rows = 0;
            for (int l = 0; l < 4; ++l)
                if (s.impact[l]) { mask |= 1 << l; ++rows; }
            if (!mask) continue;  // no rows: no AL terms
            if (slot == HSDDP_MAX_TD)
                refuse(i, "more than " + std::to_string(HSDDP_MAX_TD) + " touchdown constraints on one phase");
            if (td_seen && (s.sigma_max != td0.sigma_max || s.ground != td0.ground))
                refuse(i, "touchdown sigma_max / ground height differ from another constraint's (one set per handle)");
            if (!td_seen) td0 = s;
            td_seen = true;
            const bool own = c->params.size() == (size_t)rows;  // initialize_params ran (else the defaults)
            if (!own && !c->params.empty()) refuse(i, "touchdown constraint parameters do not match its rows");
            pr.td_legs[(size_t)i * HSDDP_MAX_TD + slot] = mask;
            for (int l = 0, r = 0; l < 4; ++l) {
                if (!((mask >> l) & 1)) continue;
                const size_t q = ((size_t)i * HSDDP_MAX_TD + slot) * 4 + l;
                pr.al_sigma[q] = own ? (double)c->params[r].sigma : s.sigma;
                pr.al_lambda[q] = own ? (double)c->params[r].lambda : s.lambda;
                ++r;
            }
            ++slot;
        }
    }
    if (td_seen) {
        desc.cparams.td_sigma = td0.sigma; desc.cparams.td_lambda = td0.lambda;
        desc.cparams.td_sigma_max = td0.sigma_max; desc.cparams.ground_height = td0.ground;
    }
    // the contact after the horizon: the last phase's reset target, else the touchdown legs' stance
    for (int l = 0; l < 4; ++l) {
        int td = 0;
        for (int j = 0; j < HSDDP_MAX_TD; ++j) td |= (pr.td_legs[(size_t)(P - 1) * HSDDP_MAX_TD + j] >> l) & 1;
        pr.contacts[4 * P + l] = has_reset[P - 1] ? rst[P - 1].cn[l] : (td ? 1 : pr.contacts[4 * (P - 1) + l]);
    }
    for (int i = 0; i < P; ++i)
        for (int l = 0; l < 4; ++l) {
            const int c = pr.contacts[4 * i + l], cn = pr.contacts[4 * (i + 1) + l];
            if (has_reset[i] && rst[i].cn[l] != cn) refuse(i, "the resetmap's next contact differs from the next phase's");
            if (!has_reset[i] && c != cn && i < P - 1)
                refuse(i, "the contact changes at the phase end but no resetmap (HKDReset) is registered");
        }
    // path constraints: GRF friction pyramids with their per-knot ReB parameters
    // (PathConstraintBase::params [knot][row], 5 rows per stance leg in leg order)
    hsddp_facade::GrfSpec g0;
    bool grf_seen = false;
    for (int i = 0; i < P; ++i) {
        int stance = 0, n_grf = 0;
        for (int l = 0; l < 4; ++l) stance += pr.contacts[4 * i + l];
        for (auto &c : ph[i]->pconstraints) {
            const auto *dc = dynamic_cast<const hsddp_facade::DevicePathConstraint *>(c.get());
            if (!dc) refuse(i, "path constraint '" + c->name + "' cannot run on the device");
            hsddp_facade::GrfSpec s;
            dc->device_spec(s);
            for (int l = 0; l < 4; ++l)
                if (s.contact[l] != pr.contacts[4 * i + l]) refuse(i, "GRF constraint contact differs from the phase's");
            ++n_grf;
            if (grf_seen && (s.mu != g0.mu || s.delta_min != g0.delta_min))
                refuse(i, "GRF friction coefficient / ReB delta_min differ from another phase's (one set per handle)");
            if (!grf_seen) g0 = s;
            grf_seen = true;
        }
        if (stance > 0 && n_grf != 1) refuse(i, "a phase with stance legs needs exactly one GRF constraint");
    }
    if (grf_seen) {
        desc.cparams.mu_fric = g0.mu;
        desc.cparams.grf_delta = g0.delta; desc.cparams.grf_delta_min = g0.delta_min; desc.cparams.grf_eps = g0.eps;
    }
    // costs: one tracking and one foot-placement term per phase
    std::vector<hsddp_facade::CostSpec> track(P), foot(P);
    for (int i = 0; i < P; ++i) {
        int nt = 0, nf = 0;
        for (auto &c : ph[i]->costs) {
            const auto *dc = dynamic_cast<const hsddp_facade::DeviceCost *>(c.get());
            if (!dc) refuse(i, "cost '" + c->cost_name + "' cannot run on the device");
            hsddp_facade::CostSpec s;
            dc->device_spec(s, &pr.contacts[4 * i]);
            if (s.terms & HSDDP_TERM_TRACKING) { track[i] = s; ++nt; }
            if (s.terms & HSDDP_TERM_FOOT) { foot[i] = s; ++nf; }
        }
        if (nt != 1 || nf != 1)
            refuse(i, "needs one HKD tracking cost and one foot-placement regularisation (HKDTrackingCost / "
                      "HKDFootPlaceReg, or hkd::TrackingCost / hkd::FootPlaceReg)");
        const int N = trajs[i]->horizon;
        if ((track[i].x_rows >= 0 && track[i].x_rows != N + 1) || (track[i].u_rows >= 0 && track[i].u_rows < N) ||
            (foot[i].foot_rows >= 0 && foot[i].foot_rows != N + 1))
            refuse(i, "reference tables must match the horizon (x_ref and foot_ref: N + 1 rows, u_ref: at least N)");
    }
    desc.weights = derive_weights(track, foot, pr.contacts);
    hsddp_pack::layout(trajs, desc.horizons, desc.dt, pr.S, pr.Kc);
    // per-knot ReB parameters of the GRF constraints (initialize_params ran: its own, else the spec's)
    pr.reb_delta.assign((size_t)pr.Kc * 20, desc.cparams.grf_delta);
    pr.reb_eps.assign((size_t)pr.Kc * 20, desc.cparams.grf_eps);
    for (int i = 0, k0 = 0; i < P; k0 += desc.horizons[i], ++i)
        for (auto &c : ph[i]->pconstraints) {
            hsddp_facade::GrfSpec s;
            dynamic_cast<const hsddp_facade::DevicePathConstraint *>(c.get())->device_spec(s);
            const int N = desc.horizons[i];
            if (c->params.empty()) {
                for (int k = 0; k < N; ++k)
                    for (int r = 0; r < 20; ++r) {
                        pr.reb_delta[(size_t)(k0 + k) * 20 + r] = s.delta;
                        pr.reb_eps[(size_t)(k0 + k) * 20 + r] = s.eps;
                    }
                continue;
            }
            if ((int)c->params.size() != N) refuse(i, "GRF constraint parameters do not cover the phase horizon");
            for (int k = 0; k < N; ++k) {
                const auto &row = c->params[k];
                if (row.size() != c->size) refuse(i, "GRF constraint parameters do not match its rows");
                for (int l = 0, q = 0; l < 4; ++l) {
                    if (!s.contact[l]) continue;
                    for (int r = 0; r < 5; ++r, ++q) {
                        pr.reb_delta[(size_t)(k0 + k) * 20 + 5 * l + r] = row[q].delta;
                        pr.reb_eps[(size_t)(k0 + k) * 20 + 5 * l + r] = row[q].eps;
                    }
                }
            }
        }
    // shooting states: SinglePhase::SS_set (update_SS_config, SinglePhase.h:161-164), read as the
    // rollout reads it (find(k) for k = 0 .. N, SinglePhase.cpp:187-220): entries past N are never
    // queried.  The device holds SS_set = {0 .. m - 1}; the knot-parallel rollout simulates the
    // states after the last shooting one in the last phase only — HKDProblem::update leaves a new
    // last phase of horizon <= 2 with an empty set (HKDProblem.cpp:203-217), every other phase full.
    pr.shooting.assign(P, 0);
    for (int i = 0; i < P; ++i) {
        const int N = desc.horizons[i];
        std::vector<int> in;
        for (int s : ph[i]->SS_set)
            if (s >= 0 && s <= N) in.push_back(s);
        std::sort(in.begin(), in.end());
        in.erase(std::unique(in.begin(), in.end()), in.end());
        for (size_t j = 0; j < in.size(); ++j)
            if (in[j] != (int)j)
                refuse(i, "shooting states (SS_set) other than {0 .. m-1} cannot run on the device");
        pr.shooting[i] = (int)in.size();
        if (i < P - 1 && pr.shooting[i] != N + 1)
            refuse(i, "has non-shooting states (SS_set covers " + std::to_string(pr.shooting[i]) + " of " +
                          std::to_string(N + 1) + " states; call update_SS_config(N + 1) as HKDProblem.cpp:104 does): "
                          "the device rollout simulates non-shooting states in the last phase only");
    }
    // references at every knot's time t = t_offset + k dt (SinglePhase.cpp:243-287)
    hsddp_pack::pack_references(P, desc.horizons, [&](int i, int k, double *xr, double *ur, double *pf) {
        const float t = (float)(ph[i]->t_offset + k * trajs[i]->timeStep);
        double pcom[3] = {0, 0, 0};
        track[i].track_ref(k, t, xr, ur);
        foot[i].foot_ref(k, t, pf, pcom);
        if (foot[i].foot_pcom && (pcom[0] != xr[3] || pcom[1] != xr[4] || pcom[2] != xr[5]))
            refuse(i, "the foot-placement reference's body position differs from the tracking reference's at knot " +
                          std::to_string(k) + " (the device takes both from one reference)");
    }, pr.ref_x, pr.ref_u, pr.ref_foot);
    hsddp_pack::pack_trajectories(trajs, pr.Xbar, pr.Ubar, pr.K);
    return pr;
}

// the solve's AL / ReB parameters back into the phases' constraint objects (their params rows,
// in the order describe() read them); objects whose params were never initialised stay as they are
template <typename T>
void MultiPhaseDDP<T>::write_back_constraints(const Problem &pr)
{
    for (int i = 0, k0 = 0; i < n_phases; k0 += pr.desc.horizons[i], ++i) {
        Phase *ph = dynamic_cast<Phase *>(phases[i].get());
        int slot = 0;
        for (auto &c : ph->tconstraints) {
            hsddp_facade::TdSpec s;
            dynamic_cast<const hsddp_facade::DeviceTerminalConstraint *>(c.get())->device_spec(s);
            int mask = 0;
            for (int l = 0; l < 4; ++l) mask |= s.impact[l] ? 1 << l : 0;
            if (!mask) continue;
            if (!c->params.empty())
                for (int l = 0, r = 0; l < 4; ++l) {
                    if (!((mask >> l) & 1)) continue;
                    const size_t q = ((size_t)i * HSDDP_MAX_TD + slot) * 4 + l;
                    c->params[r].sigma = (T)pr.al_sigma[q];
                    c->params[r].lambda = (T)pr.al_lambda[q];
                    ++r;
                }
            ++slot;
        }
        for (auto &c : ph->pconstraints) {
            if (c->params.empty()) continue;
            hsddp_facade::GrfSpec s;
            dynamic_cast<const hsddp_facade::DevicePathConstraint *>(c.get())->device_spec(s);
            for (int k = 0; k < pr.desc.horizons[i]; ++k)
                for (int l = 0, q = 0; l < 4; ++l) {
                    if (!s.contact[l]) continue;
                    for (int r = 0; r < 5; ++r, ++q) {
                        c->params[k][q].delta = (T)pr.reb_delta[(size_t)(k0 + k) * 20 + 5 * l + r];
                        c->params[k][q].eps = (T)pr.reb_eps[(size_t)(k0 + k) * 20 + 5 * l + r];
                    }
                }
        }
    }
}

template <typename T>
void MultiPhaseDDP<T>::solve(HSDDP_OPTION option)
{
    Problem pr = describe();
    const int P = n_phases, S = pr.S, Kc = pr.Kc;
    std::vector<std::shared_ptr<Trajectory<double, 24, 24, 0>>> trajs(P);
    for (int i = 0; i < P; ++i) trajs[i] = dynamic_cast<Phase *>(phases[i].get())->traj;
    // One handle while the weights, parameters and the total knot count stay the same: the MPC
    // loop's receding-horizon updates (HKDProblem::update) move knots between phases and add or
    // drop phases, which the live handle takes as a new layout (hsddp_set_layout, no device
    // allocation and no re-capture of anything but the iteration graphs of the new layout).
    hsddp_problem_desc key = pr.desc;
    key.n_phases = 0;
    std::memset(key.horizons, 0, sizeof key.horizons);
    if (!handle || std::memcmp(&key, &handle_desc, sizeof handle_desc) != 0 || Kc != handle_Kc) {
        release();
        acquire(pr.desc, key, Kc);
    }
    check(hsddp_set_layout(handle, P, pr.desc.horizons, pr.shooting.data(), nullptr));
    const hsddp_options o = option.to_c();
    check(hsddp_set_options(handle, &o));
    check(hsddp_upload_problem(handle, pr.contacts.data(), x0.data(), pr.ref_x.data(), pr.ref_u.data(), pr.ref_foot.data()));
    check(hsddp_upload_warm_start(handle, pr.Xbar.data(), pr.Ubar.data(), pr.K.data()));
    check(hsddp_upload_constraint_params(handle, pr.reb_delta.data(), pr.reb_eps.data(), pr.td_legs.data(),
                                         pr.al_sigma.data(), pr.al_lambda.data()));
    hsddp_stats st;
    check(hsddp_solve(handle, &st));
    // the constraint objects keep the parameters the solve's AL / ReB updates left (the next MPC
    // tick starts from them, as the reference's objects do)
    check(hsddp_download_constraint_params(handle, pr.reb_delta.data(), pr.reb_eps.data(), nullptr,
                                           pr.al_sigma.data(), pr.al_lambda.data()));
    write_back_constraints(pr);
    // solution, working trajectory, LQ model, terminal data, value function, solver info
    std::vector<double> &Xb = pr.Xbar, &Ub = pr.Ubar, &K = pr.K;
    check(hsddp_download_trajectory(handle, Xb.data(), Ub.data(), K.data()));
    hsddp_pack::unpack_trajectories(trajs, Xb.data(), Ub.data(), K.data());
    std::vector<double> X(24 * S), U(24 * Kc), D(24 * S), dX(24 * S), dU(24 * Kc);
    check(hsddp_download_working(handle, X.data(), U.data(), D.data(), dX.data(), dU.data()));
    hsddp_pack::unpack_working(trajs, X.data(), U.data(), D.data(), dX.data(), dU.data());
    std::vector<double> A(576 * Kc), Bm(576 * Kc), l(Kc), lx(24 * Kc), lu(24 * Kc), lxx(576 * Kc), luu(576 * Kc);
    check(hsddp_download_lq(handle, A.data(), Bm.data(), l.data(), lx.data(), lu.data(), lxx.data(), luu.data()));
    hsddp_pack::unpack_lq(trajs, A.data(), Bm.data(), l.data(), lx.data(), lu.data(), lxx.data(), luu.data());
    std::vector<double> Phi(P), Phix(24 * P), Phixx(576 * P), G(24 * P), H(576 * P);
    check(hsddp_download_terminal(handle, Phi.data(), Phix.data(), Phixx.data(), nullptr));
    check(hsddp_download_value(handle, G.data(), H.data()));
    hsddp_pack::unpack_terminal_value(trajs, Phi.data(), Phix.data(), Phixx.data(), G.data(), H.data());
    check(hsddp_download_element_info(handle, &info));
    const int cap = 1 + std::max(0, option.max_AL_iter) * std::max(0, option.max_DDP_iter);
    std::vector<float> c(cap), f(cap), e(cap), q(cap);
    int count = 0;
    check(hsddp_download_solver_info(handle, cap, c.data(), f.data(), e.data(), q.data(), &count));
    cost_buffer.assign(c.begin(), c.begin() + count);
    dyn_feas_buffer.assign(f.begin(), f.begin() + count);
    eqn_feas_buffer.assign(e.begin(), e.begin() + count);
    ineq_feas_buffer.assign(q.begin(), q.begin() + count);
    size_t kc = 0;
    for (int i = 0; i < P; ++i) {  // SinglePhase::get_actual_cost: running + terminal cost
        double pc = 0;
        for (int k = 0; k < pr.desc.horizons[i]; ++k, ++kc) pc += l[kc];
        dynamic_cast<Phase *>(phases[i].get())->actual_cost = pc + Phi[i];
    }
    actual_cost = info.cost;
    feas = info.feas;
    max_tconstr = info.max_tconstr;
    max_pconstr = info.max_pconstr;
}

#endif  // HSDDP_FACADE_HPP
