// hkd_trajopt.hpp — the HKD-TrajOpt and Reference classes with the reference's names and
// signatures, so that HKDProblem's own registrations (HKDProblem.cpp:15-111, 225-310) compile
// against the facade and solve on the GPU:
//
//   bind(&HKD::Model<T>::dynamics, &hkdModel, _1.._5, phase_contact, (T)dt_sim)    HKDModel.h:33-45
//   bind(&HKD::Model<T>::dynamics_partial, &hkdModel, _1.._7, phase_contact, dt)  HKDModel.h:46-61
//   make_shared<HKDTrackingCost<T>>(phase_contact)->set_reference(&hkd_reference)  HKDCost.h:8-38
//   make_shared<HKDFootPlaceReg<T>>(phase_contact)->set_quad_reference(quad_ref)   HKDCost.h:40-99
//   make_shared<GRFConstraint<T>>(phase_contact), initialize_params(grf_reb_param) HKDConstraints.h:8-27
//   bind(&HKDReset<T>::resetmap(_partial), &hkdReset, _1, _2, contact, next)      HKDReset.h:41-136
//   make_shared<TouchDownConstraint<T>>(touchdown_status), initialize_params(td)  HKDConstraints.h:29-51
//   QuadReference / HKDSinglePhaseReference                                       QuadReference.h, HKDReference.h
//
// MultiPhaseDDP::solve (hsddp_facade.hpp) reads what each registration binds — the dynamics' and
// reset's contacts and dt by calling them once in probe mode (HKD::Model / HKDReset record their
// bound arguments instead of evaluating), the costs' weights and references, the constraints'
// parameters — and runs the whole solve on the device.  Called directly (point by point), the
// model, reset, foot cost and constraints evaluate through the device primitives of the C-ABI;
// QuadReference and HKDSinglePhaseReference are the reference's host-side bookkeeping (time
// indexing of a sample table).  T = double (the device path computes in fp64).
#ifndef HKD_TRAJOPT_HPP
#define HKD_TRAJOPT_HPP

#include <cmath>
#include <cstdio>
#include <deque>
#include <string>
#include <vector>

#include "hsddp_facade.hpp"

// ---- HSDDP_Utils.h helpers HKDProblem.cpp uses ------------------------------------------------
// indices i with v[i] == val (HSDDP_Utils.h:21-34)
template <typename V, typename S>
std::vector<int> find_eigen(const V &v, const S &val)
{
    std::vector<int> idx;
    for (int i = 0; i < (int)v.size(); ++i)
        if (v[i] == static_cast<typename V::Scalar>(val)) idx.push_back(i);
    return idx;
}
// |n1 - n2| <= 1e-6 in float (HSDDP_Utils.h:44-55), and the <= / >= built on it (:57-79)
template <typename T1, typename T2>
bool approx_eq_scalar(T1 n1, T2 n2)
{
    const float tol = 1e-6;
    const float err = std::abs(n1 - n2);
    return err <= tol;
}
template <typename T1, typename T2>
bool approx_leq_scalar(T1 n1, T2 n2) { return n1 < n2 || approx_eq_scalar(n1, n2); }
template <typename T1, typename T2>
bool approx_geq_scalar(T1 n1, T2 n2) { return n1 > n2 || approx_eq_scalar(n1, n2); }

template <typename T>
using Vec3 = VecM<T, 3>;

// ---- HKD::Model (HKDModel.h:11-62) -----------------------------------------------------------
namespace HKD {
const size_t xs = 24;
const size_t us = 24;
const size_t ys = 0;

template <typename T>
class Model {
public:
    typedef VecM<T, xs> StateType;
    typedef VecM<T, us> ContrlType;
    typedef VecM<T, ys> OutputType;
    typedef VecM<T, 12> JointType;
    typedef MatMN<T, xs, xs> StateMap;
    typedef MatMN<T, xs, us> ContrlMap;
    typedef MatMN<T, ys, xs> OutputMap;
    typedef MatMN<T, ys, us> DirectMap;
    typedef VecM<int, 4> CtactStatusType;

    // x_next = hkinodyn(x, u, dt, contact) (explicit Euler, HKDModel.h:33-45)
    void dynamics(StateType &xnext, OutputType &y, StateType &x, ContrlType &u, T t, CtactStatusType &ctact_status, T &dt)
    {
        (void)y; (void)t;
        if (hsddp_facade::probe_record(hsddp_facade::PROBE_DYNAMICS, ctact_status, (const CtactStatusType *)nullptr, dt,
                                       &xnext, nullptr, &x, &u))
            return;
        static_assert(std::is_same<T, double>::value, "the device model computes in fp64");
        const double c[4] = {(double)ctact_status[0], (double)ctact_status[1], (double)ctact_status[2], (double)ctact_status[3]};
        const double h = dt;
        hkd::detail::on_device({{x.data(), 192}, {u.data(), 192}, {c, 32}}, {{xnext.data(), 192}},
                               [&](std::vector<void *> &i, std::vector<void *> &o) {
                                   return hsddp_hkd_dynamics((double *)i[0], (double *)i[1], (double *)i[2], h,
                                                             (double *)o[0], 1, nullptr);
                               });
    }
    // A, B = hkinodyn_par(x, u, dt, contact) in Eigen column-major storage (HKDModel.h:46-61)
    void dynamics_partial(StateMap &A, ContrlMap &B, OutputMap &C, DirectMap &D, StateType &x, ContrlType &u, T t,
                          CtactStatusType &ctact_status, T &dt)
    {
        (void)C; (void)D; (void)t;
        if (hsddp_facade::probe_record(hsddp_facade::PROBE_DYNAMICS_PARTIAL, ctact_status, (const CtactStatusType *)nullptr,
                                       dt, &A, &B, &x, &u))
            return;
        static_assert(std::is_same<T, double>::value, "the device model computes in fp64");
        const double c[4] = {(double)ctact_status[0], (double)ctact_status[1], (double)ctact_status[2], (double)ctact_status[3]};
        const double h = dt;
        hkd::detail::on_device({{x.data(), 192}, {u.data(), 192}, {c, 32}}, {{A.data(), 4608}, {B.data(), 4608}},
                               [&](std::vector<void *> &i, std::vector<void *> &o) {
                                   return hsddp_hkd_dynamics_partial((double *)i[0], (double *)i[1], (double *)i[2], h,
                                                                     (double *)o[0], (double *)o[1], 1, nullptr);
                               });
    }
};
}  // namespace HKD

// compute_hkd_state (HKDModel.h:65-96): qdummy of a swing leg = its joint angles, of a stance leg
// = its foot position (device forward kinematics)
template <typename T>
void compute_hkd_state(Vec3<T> &eul, Vec3<T> &pos, VecM<T, 12> &qJ, VecM<T, 12> &qdummy, const VecM<int, 4> &c)
{
    std::vector<double> x(4 * 24, 0.0), pf(12);
    std::vector<int> legs = {0, 1, 2, 3};
    for (int l = 0; l < 4; ++l) {
        double *xl = &x[24 * l];
        for (int a = 0; a < 3; ++a) { xl[a] = eul[a]; xl[3 + a] = pos[a]; }
        for (int j = 0; j < 12; ++j) xl[12 + j] = qJ[j];
    }
    hkd::detail::on_device({{x.data(), x.size() * 8}, {legs.data(), 16}}, {{pf.data(), 96}},
                           [&](std::vector<void *> &i, std::vector<void *> &o) {
                               return hsddp_hkd_foot_position((double *)i[0], (int *)i[1], (double *)o[0], 4, nullptr);
                           });
    for (int l = 0; l < 4; ++l)
        for (int a = 0; a < 3; ++a) qdummy[3 * l + a] = c[l] == 0 ? qJ[3 * l + a] : (T)pf[3 * l + a];
}

// ---- HKDReset (HKDReset.h:9-136) -------------------------------------------------------------
template <typename T>
class HKDReset {
public:
    static const size_t xs = 24, us = 24, ys = 0;

    // x at a contact switch c -> cn: a leg lifting off takes the default joint angles, a leg
    // touching down its foot position projected onto the ground plane
    void resetmap(DVec<T> &xnext, DVec<T> &x, VecM<int, 4> &c, VecM<int, 4> &cn)
    {
        if (hsddp_facade::probe_record(hsddp_facade::PROBE_RESET, c, &cn, 0.0, &xnext, nullptr, &x, nullptr)) return;
        static_assert(std::is_same<T, double>::value, "the device model computes in fp64");
        int ci[4], cni[4];
        for (int l = 0; l < 4; ++l) { ci[l] = c[l]; cni[l] = cn[l]; }
        xnext.setZero(24);
        hkd::detail::on_device({{x.data(), 192}, {ci, 16}, {cni, 16}}, {{xnext.data(), 192}},
                               [&](std::vector<void *> &i, std::vector<void *> &o) {
                                   return hsddp_hkd_resetmap((double *)i[0], (int *)i[1], (int *)i[2], (double *)o[0], 1,
                                                             nullptr);
                               });
    }
    // its Jacobian Px (24 x 24, column-major)
    void resetmap_partial(DMat<T> &Px, DVec<T> &x, VecM<int, 4> &c, VecM<int, 4> &cn)
    {
        if (hsddp_facade::probe_record(hsddp_facade::PROBE_RESET_PARTIAL, c, &cn, 0.0, &Px, nullptr, &x, nullptr)) return;
        static_assert(std::is_same<T, double>::value, "the device model computes in fp64");
        int ci[4], cni[4];
        for (int l = 0; l < 4; ++l) { ci[l] = c[l]; cni[l] = cn[l]; }
        Px.setZero(24, 24);
        hkd::detail::on_device({{x.data(), 192}, {ci, 16}, {cni, 16}}, {{Px.data(), 4608}},
                               [&](std::vector<void *> &i, std::vector<void *> &o) {
                                   return hsddp_hkd_resetmap_partial((double *)i[0], (int *)i[1], (int *)i[2],
                                                                     (double *)o[0], 1, nullptr);
                               });
    }
};

// ---- QuadReference (Reference/QuadReference.h:14-190, QuadReference.cpp) ------------------------
struct QuadAugmentedState {
    VecM<double, 12> body_state;       // eul, pos, omega, vWorld
    VecM<double, 12> qJ, qJd, foot_placements, grf, torque;
    VecM<int, 4> contact;
    VecM<double, 4> status_dur;
    void SetZero() { *this = QuadAugmentedState(); }
};

class QuadReferenceData {
public:
    QuadReferenceData() = default;
    explicit QuadReferenceData(size_t sz) : astates(sz) {}
    float get_duration() { return end_time - start_time; }
    size_t size() const { return astates.size(); }
    void clear() { astates.clear(); }
    void pop_front() { astates.pop_front(); }
    void push_back(QuadAugmentedState &s) { astates.push_back(s); }
    QuadAugmentedState &operator[](size_t k) { return astates.at(k); }
    QuadAugmentedState &at(size_t k) { return astates.at(k); }
    QuadAugmentedState *get_ptr(size_t k) { return &astates.at(k); }
    std::deque<QuadAugmentedState>::iterator begin() { return astates.begin(); }
    std::deque<QuadAugmentedState>::iterator end() { return astates.end(); }
    std::deque<QuadAugmentedState> &get_container() { return astates; }

    float dt = 0, start_time = 0, end_time = 0;

private:
    std::deque<QuadAugmentedState> astates;
};

// A planning window into a long sample table: the window starts at sample k_cur (time t_cur) and
// holds sz + 1 samples (sz = round(horizon / dt) + 1); queries take a time relative to the window
// start and snap to the nearest sample (float arithmetic as QuadReference.cpp:60-120, quirk A18).
class QuadReference {
public:
    // parse a quad_reference.csv (QuadReference.cpp:129-290; the C-ABI's parser, values through float)
    void load_top_level_data(const std::string &fname, bool reorder = false)
    {
        float dtf = 0;
        const int n = hsddp_load_quad_reference(fname.c_str(), reorder ? 1 : 0, &dtf, nullptr, 0);
        if (n <= 0) throw std::runtime_error(std::string("QuadReference: ") + hsddp_last_error());
        std::vector<hsddp_quad_state> rows(n);
        hsddp_load_quad_reference(fname.c_str(), reorder ? 1 : 0, &dtf, rows.data(), n);
        tp_data.clear();
        for (const hsddp_quad_state &r : rows) {
            QuadAugmentedState s;
            for (int j = 0; j < 12; ++j) {
                s.body_state[j] = r.body_state[j]; s.qJ[j] = r.qJ[j]; s.qJd[j] = r.qJd[j];
                s.foot_placements[j] = r.foot_placements[j]; s.grf[j] = r.grf[j]; s.torque[j] = r.torque[j];
            }
            for (int l = 0; l < 4; ++l) { s.contact[l] = r.contact[l]; s.status_dur[l] = r.status_dur[l]; }
            tp_data.push_back(s);
        }
        tp_data.dt = dtf;
    }
    // the window at the table's start (QuadReference.cpp:6-27)
    void initialize(float plan_horizon)
    {
        t_cur = 0;
        k_cur = 0;
        dt = tp_data.dt;
        dur = plan_horizon;
        sz = (int)std::round(plan_horizon / dt) + 1;
        if ((int)tp_data.size() < sz + 1) throw std::runtime_error("QuadReference: table shorter than the plan window");
        data.clear();
        for (int k = 0; k <= sz; ++k) data.push_back(tp_data[k]);
        data.start_time = t_cur;
        data.end_time = t_cur + dur;
    }
    // advance the window by dt_sim (whole reference steps, QuadReference.cpp:34-50)
    void step(float dt_sim)
    {
        for (int i = 1; approx_leq_scalar(i * dt, dt_sim); ++i) {
            ++k_cur;
            t_cur += dt;
            if (k_cur + sz >= (int)tp_data.size()) throw std::runtime_error("QuadReference: stepped past the table end");
            data.pop_front();
            data.push_back(tp_data[k_cur + sz]);
            data.start_time = t_cur;
            data.end_time = t_cur + dur;
        }
    }
    void update_foot_placements(const VecM<double, 12> &) {}  // not implemented in the reference either
    QuadAugmentedState *get_a_reference_ptr_at_t(float t) { return data.get_ptr(index_at(t)); }
    void get_contact_at_t(VecM<int, 4> &contact, float t) { contact = data[index_at(t)].contact; }
    void get_contact_duration_at_t(VecM<double, 4> &d, float t) { d = data[index_at(t)].status_dur; }
    QuadReferenceData *get_data_ptr() { return &data; }
    QuadReferenceData *get_tp_data_ptr() { return &tp_data; }
    int get_data_size() { return sz; }
    float get_dt() { return dt; }
    float get_start_time() { return data.start_time; }
    float get_end_time() { return data.end_time; }

private:
    // the sample nearest to t: floor, then one up past the half step; clamped to the window end
    int index_at(float t) const
    {
        int k = (int)std::floor(t / dt);
        if (t - k * dt > 0.5 * dt) ++k;
        if (k > sz) {
            std::fprintf(stderr, "warning: queried reference out of scope (t = %f)\n", t + t_cur);
            k = sz;
        }
        return k;
    }
    QuadReferenceData data, tp_data;
    float t_cur = 0, dur = 0, dt = 0;
    int k_cur = 0, sz = 0;
};

// HKDSinglePhaseReference (HKDReference.h:14-35, HKDReference.cpp:8-57): the HKD state reference
// [body_state, per leg: foot position (stance) or joint angles (swing)], control [grf, qJd]
class HKDSinglePhaseReference : public SinglePhaseReferenceAbstract<24, 24, 0> {
public:
    void set_quadruped_reference(QuadReference *quad_ref) { quad_ref_ = quad_ref; }
    void get_reference_at_t(VecM<double, 24> &xt, VecM<double, 24> &ut, VecM<double, 0> &yt, float t) override
    {
        (void)yt;
        get_reference_at_t(xt, t);
        if (!state_) return;
        for (int j = 0; j < 12; ++j) { ut[j] = state_->grf[j]; ut[12 + j] = state_->qJd[j]; }
    }
    void get_reference_at_t(VecM<double, 24> &xt, float t) override
    {
        state_ = quad_ref_ ? quad_ref_->get_a_reference_ptr_at_t(t) : nullptr;
        if (!state_) {
            std::fprintf(stderr, "error: quad_ref is nullptr\n");
            return;
        }
        for (int j = 0; j < 12; ++j) xt[j] = state_->body_state[j];
        for (int l = 0; l < 4; ++l)
            for (int a = 0; a < 3; ++a)
                xt[12 + 3 * l + a] = state_->contact[l] > 0 ? state_->foot_placements[3 * l + a] : state_->qJ[3 * l + a];
    }

private:
    QuadReference *quad_ref_ = nullptr;
    QuadAugmentedState *state_ = nullptr;
};

// ---- HKD costs (HKDCost.h, HKDCost.cpp) -------------------------------------------------------
// HKDTrackingCost: QuadraticTrackingCost with the HKD weights for one contact (HKDCost.h:8-38):
// Q = diag(eul 1 4 5, pos 1 1 30, omega .2, v 4 1 .5, qJ .2 (1 - c_leg)), Qf = 20 diag(scale) Q,
// R = diag(GRF .2, qJd .1).  The device solve reads Q, R, Qf and the reference it is set to.
template <typename T>
class HKDTrackingCost : public QuadraticTrackingCost<T, HKD::xs, HKD::us, HKD::ys>, public hsddp_facade::DeviceCost {
public:
    explicit HKDTrackingCost(VecM<int, 4> contact) : QuadraticTrackingCost<T, HKD::xs, HKD::us, HKD::ys>()
    {
        const T qb[12] = {1, 4, 5, 1, 1, 30, .2, .2, .2, 4, 1, .5};
        const T scale[24] = {1, 1, 2, 1, 1, 20, .3, .3, .3, 1, 3, 1, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01, .01};
        this->Q.setZero();
        this->Qf.setZero();
        this->R.setZero();
        for (int j = 0; j < 24; ++j) {
            this->Q(j, j) = j < 12 ? qb[j] : T(.2 * (1 - contact[(j - 12) / 3]));
            this->Qf(j, j) = (20 * scale[j]) * this->Q(j, j);
            this->R(j, j) = j < 12 ? T(.2) : T(.1);
        }
    }
    void device_spec(hsddp_facade::CostSpec &spec, const int *) const override
    {
        spec.terms = HSDDP_TERM_TRACKING;
        for (int a = 0; a < 24; ++a)
            for (int b = 0; b < 24; ++b)
                if (a != b && (this->Q(a, b) != 0 || this->R(a, b) != 0 || this->Qf(a, b) != 0))
                    throw std::runtime_error(this->cost_name + ": the device applies diagonal Q, R, Qf only");
        for (int j = 0; j < 24; ++j) { spec.q[j] = this->Q(j, j); spec.r[j] = this->R(j, j); spec.qf[j] = this->Qf(j, j); }
        auto *ref = this->get_reference();
        if (!ref) throw std::runtime_error(this->cost_name + ": set_reference was not called");
        spec.track_ref = [ref](int, float t, double *xr, double *ur) {
            VecM<double, 24> x, u;
            VecM<double, 0> y;
            ref->get_reference_at_t(x, u, y, t);
            for (int j = 0; j < 24; ++j) { xr[j] = x[j]; ur[j] = u[j]; }
        };
    }
};

// HKDFootPlaceReg (HKDCost.h:40-99, HKDCost.cpp:5-63): foot positions relative to the body, against
// the reference's footholds relative to the reference body, weighted by Qfoot = 20 diag(3c, c, 0)
// per leg; running cost dt/2 d^T Qfoot d, terminal 10 d^T Qfoot d.
template <typename T>
class HKDFootPlaceReg : public CostBase<T, HKD::xs, HKD::us, HKD::ys>, public hsddp_facade::DeviceCost {
public:
    typedef CostBase<T, HKD::xs, HKD::us, HKD::ys> Base;
    using typename Base::State;
    using typename Base::Contrl;
    using typename Base::Output;
    using typename Base::RCost;
    using typename Base::TCost;

    explicit HKDFootPlaceReg(const VecM<int, 4> &contact) : Base("Foot regularization"), contact_(contact)
    {
        for (int l = 0; l < 4; ++l) {
            Qfoot(3 * l, 3 * l) = 3 * contact[l];
            Qfoot(3 * l + 1, 3 * l + 1) = contact[l];
        }
        for (int j = 0; j < 12; ++j) Qfoot(j, j) *= 20;
    }
    void set_quad_reference(QuadReference *quad_reference_in) { quad_reference = quad_reference_in; }

    void running_cost(RCost &rc, const State &x, const Contrl &u, const Output &, T dt, float t = 0) override
    {
        eval(x, u, dt, t, &rc, nullptr, false);
    }
    void running_cost_par(RCost &rc, const State &x, const Contrl &u, const Output &, T dt, float t = 0) override
    {
        eval(x, u, dt, t, &rc, nullptr, true);
    }
    void terminal_cost(TCost &tc, const State &x, float tend = 0) override { eval(x, Contrl(), 0, tend, nullptr, &tc, false); }
    void terminal_cost_par(TCost &tc, const State &x, float tend = 0) override { eval(x, Contrl(), 0, tend, nullptr, &tc, true); }

    void device_spec(hsddp_facade::CostSpec &spec, const int *) const override
    {
        spec.terms = HSDDP_TERM_FOOT;
        for (int a = 0; a < 12; ++a)
            for (int b = 0; b < 12; ++b)
                if (a != b && Qfoot(a, b) != 0) throw std::runtime_error(this->cost_name + ": the device applies a diagonal Qfoot only");
        for (int j = 0; j < 12; ++j) spec.qfoot[j] = Qfoot(j, j);
        QuadReference *qr = quad_reference;
        if (!qr) throw std::runtime_error(this->cost_name + ": set_quad_reference was not called");
        spec.foot_pcom = true;
        spec.foot_ref = [qr](int, float t, double *pf, double *pcom) {
            const QuadAugmentedState *s = qr->get_a_reference_ptr_at_t(t);
            for (int j = 0; j < 12; ++j) pf[j] = s->foot_placements[j];
            for (int a = 0; a < 3; ++a) pcom[a] = s->body_state[3 + a];
        };
    }

private:
    // point evaluation on the device (hsddp_hkd_running_cost / _terminal_cost, foot terms), the
    // weights expressed as the device's (gain 20, leg weights from Qfoot)
    void eval(const State &x, const Contrl &u, T dt, float t, RCost *rc, TCost *tc, bool par) const
    {
        if (!quad_reference) throw std::runtime_error(this->cost_name + ": set_quad_reference was not called");
        const QuadAugmentedState *s = quad_reference->get_a_reference_ptr_at_t(t);
        hsddp_hkd_weights w;
        hsddp_default_weights(&w);
        for (int l = 0; l < 4; ++l)
            if (contact_[l])
                for (int a = 0; a < 3; ++a) w.foot_w[a] = Qfoot(3 * l + a, 3 * l + a) / w.foot_gain;
        int c[4];
        for (int l = 0; l < 4; ++l) c[l] = contact_[l];
        double xr[24] = {}, ur[24] = {}, pf[12];
        for (int a = 0; a < 3; ++a) xr[3 + a] = s->body_state[3 + a];
        for (int j = 0; j < 12; ++j) pf[j] = s->foot_placements[j];
        double v = 0, g[24] = {}, gu[24], H[576], Huu[576];
        if (rc) {
            hkd::detail::on_device({{x.data(), 192}, {u.data(), 192}, {c, 16}, {xr, 192}, {ur, 192}, {pf, 96}},
                                   {{&v, 8}, {g, 192}, {gu, 192}, {H, 4608}, {Huu, 4608}},
                                   [&](std::vector<void *> &i, std::vector<void *> &o) {
                                       return hsddp_hkd_running_cost((double *)i[0], (double *)i[1], (int *)i[2],
                                                                     (double *)i[3], (double *)i[4], (double *)i[5], &w, dt,
                                                                     HSDDP_TERM_FOOT, (double *)o[0], (double *)o[1],
                                                                     (double *)o[2], (double *)o[3], (double *)o[4], 1,
                                                                     nullptr);
                                   });
            if (!par) { rc->l = v; return; }
            for (int a = 0; a < 24; ++a) {
                rc->lx[a] = g[a];
                for (int b = 0; b < 24; ++b) rc->lxx(a, b) = H[24 * a + b];
            }
        } else {
            hkd::detail::on_device({{x.data(), 192}, {c, 16}, {xr, 192}, {pf, 96}}, {{&v, 8}, {g, 192}, {H, 4608}},
                                   [&](std::vector<void *> &i, std::vector<void *> &o) {
                                       return hsddp_hkd_terminal_cost((double *)i[0], (int *)i[1], (double *)i[2],
                                                                      (double *)i[3], &w, HSDDP_TERM_FOOT, (double *)o[0],
                                                                      (double *)o[1], (double *)o[2], 1, nullptr);
                                   });
            if (!par) { tc->Phi = v; return; }
            for (int a = 0; a < 24; ++a) {
                tc->Phix[a] = g[a];
                for (int b = 0; b < 24; ++b) tc->Phixx(a, b) = H[24 * a + b];
            }
        }
    }
    VecM<int, 4> contact_;
    MatMN<T, 12, 12> Qfoot;
    QuadReference *quad_reference = nullptr;
};

// ---- HKD constraints (HKDConstraints.h, HKDConstraints.cpp) ------------------------------------
// GRFConstraint: 5 friction-pyramid rows per stance leg (HKDConstraints.cpp:7-66), ReB-handled
template <typename T>
class GRFConstraint : public PathConstraintBase<T, 24, 24, 0>, public hsddp_facade::DevicePathConstraint {
    typedef PathConstraintBase<T, 24, 24, 0> Base;
    T mu_fric = .7;

public:
    using typename Base::State;
    using typename Base::Contrl;
    using typename Base::Output;

    explicit GRFConstraint(const VecM<int, 4> &ctact_) : Base("GRF"), ctact_status(ctact_)
    {
        ctact_foot_ids = find_eigen(ctact_status, 1);
        this->update_constraint_size(5 * (int)ctact_foot_ids.size());
    }
    void set_friction_coefficient(T mu_fric_in) { mu_fric = mu_fric_in; }
    void compute_violation(const State &, const Contrl &u, const Output &, int k) override
    {
        double g[20], gu[480];
        eval(u, g, gu);
        for (size_t i = 0; i < this->data[k].size(); ++i) this->data[k][i].g = g[i];
        this->update_max_violation(k);
    }
    void compute_partial(const State &, const Contrl &u, const Output &, int k) override
    {
        double g[20], gu[480];
        eval(u, g, gu);
        for (size_t i = 0; i < this->data[k].size(); ++i)
            for (int j = 0; j < 24; ++j) this->data[k][i].gu[j] = gu[24 * i + j];
    }
    void device_spec(hsddp_facade::GrfSpec &spec) const override
    {
        for (int l = 0; l < 4; ++l) spec.contact[l] = ctact_status[l];
        spec.mu = mu_fric;
        spec.delta = this->param_init.delta; spec.delta_min = this->param_init.delta_min; spec.eps = this->param_init.eps;
    }

    VecM<int, 4> ctact_status;
    std::vector<int> ctact_foot_ids;

private:
    void eval(const Contrl &u, double *g, double *gu) const
    {
        int c[4];
        for (int l = 0; l < 4; ++l) c[l] = ctact_status[l];
        const double mu = mu_fric;
        hkd::detail::on_device({{u.data(), 192}, {c, 16}}, {{g, 160}, {gu, 3840}},
                               [&](std::vector<void *> &i, std::vector<void *> &o) {
                                   return hsddp_hkd_grf_constraint((double *)i[0], (int *)i[1], mu, (double *)o[0],
                                                                   (double *)o[1], 1, nullptr);
                               });
    }
};

// TouchDownConstraint: the touching-down feet's height at the phase end (HKDConstraints.cpp:69-171),
// AL-handled
template <typename T>
class TouchDownConstraint : public TerminalConstraintBase<T, 24>, public hsddp_facade::DeviceTerminalConstraint {
    typedef TerminalConstraintBase<T, 24> Base;

public:
    using typename Base::State;

    explicit TouchDownConstraint(const VecM<int, 4> &impact) : Base("TouchDown"), impact_status(impact)
    {
        impact_foot_ids = find_eigen(impact_status, 1);
        this->update_constraint_size(impact_foot_ids.size());
    }
    void update_ground_height(T gheight_in) { ground_height = gheight_in; }
    void compute_violation(const State &x) override
    {
        double h[4], hx[96];
        eval(x, h, hx);
        if (this->data.size() != this->size) this->create_data();
        for (size_t i = 0; i < this->size; ++i) this->data[i].h = h[i];
        this->update_max_violation();
    }
    void compute_partial(const State &x) override
    {
        double h[4], hx[96];
        eval(x, h, hx);
        if (this->data.size() != this->size) this->create_data();
        for (size_t i = 0; i < this->size; ++i)
            for (int j = 0; j < 24; ++j) this->data[i].hx[j] = hx[24 * i + j];
    }
    void device_spec(hsddp_facade::TdSpec &spec) const override
    {
        for (int l = 0; l < 4; ++l) spec.impact[l] = impact_status[l] != 0;
        spec.sigma = this->param_init.sigma;
        spec.lambda = this->param_init.lambda;
        spec.sigma_max = this->param_init.sigma_max;
        spec.ground = ground_height;
    }

private:
    void eval(const State &x, double *h, double *hx) const
    {
        int c[4], cn[4];  // legs touching down: contact 0 now, 1 next
        for (int l = 0; l < 4; ++l) { c[l] = impact_status[l] ? 0 : 1; cn[l] = 1; }
        const double gh = ground_height;
        hkd::detail::on_device({{x.data(), 192}, {c, 16}, {cn, 16}}, {{h, 32}, {hx, 768}},
                               [&](std::vector<void *> &i, std::vector<void *> &o) {
                                   return hsddp_hkd_touchdown_constraint((double *)i[0], (int *)i[1], (int *)i[2], gh,
                                                                         (double *)o[0], (double *)o[1], 1, nullptr);
                               });
    }
    VecM<int, 4> impact_status;
    T ground_height = 0;
    std::vector<int> impact_foot_ids;
};

// ---- HKDProblem's data and parameters (HKDProblem.h:20-90) --------------------------------------
struct HKDPlanConfig {
    float plan_duration;       // planning horizon (s)
    float timeStep;            // simulation time step
    int nsteps_between_mpc;    // simulation steps between MPC updates
};

template <typename T>
struct HKDProblemData {
    QuadReference *quad_ref_ptr = nullptr;
    std::deque<std::shared_ptr<Trajectory<T, 24, 24, 0>>> trajectory_ptrs;
    std::deque<std::shared_ptr<SinglePhase<T, 24, 24, 0>>> phase_ptrs;
    std::deque<int> phase_horizons;
    std::deque<bool> is_phase_reach_end;
    std::deque<float> phase_start_times, phase_end_times;
    std::deque<VecM<double, 4>> contact_durations;
    std::deque<VecM<int, 4>> phase_contacts;
    int n_phases = 0;

    void clear() { *this = HKDProblemData(); }
    void pop_front_phase()
    {
        trajectory_ptrs.pop_front(); phase_ptrs.pop_front(); phase_start_times.pop_front(); phase_end_times.pop_front();
        phase_horizons.pop_front(); is_phase_reach_end.pop_front(); phase_contacts.pop_front(); contact_durations.pop_front();
        n_phases--;
    }
};

// loadConstrintParameters (HKDProblem.h:70-90): GRF_ReB, Swing_ReB, TD_AL of constraint_params.info
template <typename T>
inline void loadConstrintParameters(const std::string &fileName, REB_Param_Struct<T> &GRF_reb_param,
                                    REB_Param_Struct<T> &Swing_reb_param, AL_Param_Struct<T> &TD_al_param)
{
    hsddp_constraint_params cp;
    hsddp_default_constraint_params(&cp);
    if (hsddp_load_constraint_params(fileName.c_str(), &cp) != HSDDP_OK) throw std::runtime_error(hsddp_last_error());
    GRF_reb_param.delta = cp.grf_delta; GRF_reb_param.delta_min = cp.grf_delta_min; GRF_reb_param.eps = cp.grf_eps;
    Swing_reb_param.delta = cp.swing_delta; Swing_reb_param.delta_min = cp.swing_delta_min; Swing_reb_param.eps = cp.swing_eps;
    TD_al_param.sigma = cp.td_sigma; TD_al_param.lambda = cp.td_lambda; TD_al_param.sigma_max = cp.td_sigma_max;
}

#endif  // HKD_TRAJOPT_HPP
