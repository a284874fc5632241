// plugin_check — the reference's plugin API compiles against the facade unchanged, and the
// facade's own HKD plugins are real implementations of it.
//
// Host part (no device): a cost, a path constraint and a terminal constraint written with the exact
// declarations of the reference's HKD plugins (HKDCost.h:75-81 `override`s of CostBase's four pure
// virtuals, HKDConstraints.h:21-22 / 36-37) and a user SinglePhaseBase compile and work; hkd::
// TrackingCost / FootPlaceReg / GRFConstraint / TouchDownConstraint derive from the bases;
// MultiPhaseDDP::solve refuses a phase carrying a user cost (no CPU fallback); the bases' ReB / AL
// helpers give their closed forms; per-phase numerical steps throw (they run in the device solve).
// Device part (argument "gpu"): the hkd:: plugins' virtuals equal the batched C-ABI primitives.
#include <cstdio>

#include "hkd_trajopt.hpp"  // hsddp_facade.hpp + the HKD-TrajOpt classes (HKD::Model, HKDReset)

#define CHECK(c)                                                                    \
    do {                                                                            \
        if (!(c)) {                                                                 \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__);     \
            return 1;                                                               \
        }                                                                           \
    } while (0)

// ---- a user cost with HKDCost.h's declarations (HKDFootPlaceReg, :75-81) ----------------------
template <typename T>
class UserFootCost : public CostBase<T, 24, 24, 0> {
public:
    using typename CostBase<T, 24, 24, 0>::State;
    using typename CostBase<T, 24, 24, 0>::Contrl;
    using typename CostBase<T, 24, 24, 0>::Output;
    using typename CostBase<T, 24, 24, 0>::RCost;
    using typename CostBase<T, 24, 24, 0>::TCost;

    UserFootCost() : CostBase<T, 24, 24, 0>("User Foot Cost") {}

    void running_cost(RCost &, const State &x, const Contrl &u, const Output &y, T dt, float t = 0) override;
    void running_cost_par(RCost &, const State &x, const Contrl &u, const Output &y, T dt, float t = 0) override;
    void terminal_cost(TCost &, const State &x, float tend = 0) override;
    void terminal_cost_par(TCost &, const State &x, float tend = 0) override;
};
template <typename T>
void UserFootCost<T>::running_cost(RCost &rc, const State &x, const Contrl &u, const Output &, T dt, float)
{
    rc.l = 0;
    for (int j = 0; j < 24; ++j) rc.l += .5 * dt * (x[j] * x[j] + u[j] * u[j]);
}
template <typename T>
void UserFootCost<T>::running_cost_par(RCost &rc, const State &x, const Contrl &u, const Output &, T dt, float)
{
    for (int j = 0; j < 24; ++j) { rc.lx[j] = dt * x[j]; rc.lu[j] = dt * u[j]; rc.lxx(j, j) = dt; rc.luu(j, j) = dt; }
}
template <typename T>
void UserFootCost<T>::terminal_cost(TCost &tc, const State &x, float)
{
    tc.Phi = 0;
    for (int j = 0; j < 24; ++j) tc.Phi += .5 * x[j] * x[j];
}
template <typename T>
void UserFootCost<T>::terminal_cost_par(TCost &tc, const State &x, float)
{
    for (int j = 0; j < 24; ++j) { tc.Phix[j] = x[j]; tc.Phixx(j, j) = 1; }
}

// ---- constraints with HKDConstraints.h's declarations -----------------------------------------
template <typename T>
class UserGRF : public PathConstraintBase<T, 24, 24, 0> {
    using typename PathConstraintBase<T, 24, 24, 0>::State;
    using typename PathConstraintBase<T, 24, 24, 0>::Contrl;
    using typename PathConstraintBase<T, 24, 24, 0>::Output;

public:
    UserGRF() : PathConstraintBase<T, 24, 24, 0>("GRF") { this->update_constraint_size(1); }
    void compute_violation(const State &, const Contrl &u, const Output &, int k) override
    {
        this->data[k][0].g = u[2];
        this->update_max_violation(k);
    }
    void compute_partial(const State &, const Contrl &, const Output &, int k) override { this->data[k][0].gu[2] = 1; }
};
template <typename T>
class UserTD : public TerminalConstraintBase<T, 24> {
    using typename TerminalConstraintBase<T, 24>::State;

public:
    UserTD() : TerminalConstraintBase<T, 24>("TouchDwon") { this->update_constraint_size(1); this->create_data(); }
    void compute_violation(const State &x) { this->data[0].h = x[5] - 0.1; this->update_max_violation(); }
    void compute_partial(const State &) { this->data[0].hx[5] = 1; }
};

// ---- a user phase implementing SinglePhaseBase's pure virtuals (SinglePhaseBase.h:21-88) ------
struct UserPhase : SinglePhaseBase<double> {
    void warmstart() override {}
    void initialization() override {}
    void set_initial_condition(DVec<double> &) override {}
    void set_initial_condition_dx(DVec<double> &) override {}
    void linear_rollout(double, HSDDP_OPTION &) override {}
    bool hybrid_rollout(double, HSDDP_OPTION &, bool) override { return true; }
    void LQ_approximation(HSDDP_OPTION &) override {}
    bool backward_sweep(double, DVec<double>, DMat<double>) override { return true; }
    DVec<double> resetmap(DVec<double> &x) override { return x; }
    void resetmap_partial(DMat<double> &Px, DVec<double> &) override { Px.setZero(24, 24); }
    void get_value_approx(DVec<double> &, DMat<double> &) override {}
    void get_exp_cost_change(double &a, double &b) override { a = b = 0; }
    void get_terminal_state(DVec<double> &) override {}
    void get_terminal_state(DVec<double> &, DVec<double> &) override {}
    void get_terminal_state_dx(DVec<double> &) override {}
    double get_actual_cost() override { return 0; }
    void update_nominal_trajectory() override {}
    void compute_cost(const HSDDP_OPTION &) override {}
};

static bool close(double a, double b, double tol = 1e-13) { return std::fabs(a - b) <= tol * std::max(1.0, std::fabs(b)); }

static int host_checks()
{
    typedef SinglePhase<double, 24, 24, 0> Phase;
    // the facade's HKD plugins are the bases' implementations
    static_assert(std::is_base_of<CostBase<double, 24, 24, 0>, hkd::TrackingCost>::value, "TrackingCost");
    static_assert(std::is_base_of<CostBase<double, 24, 24, 0>, hkd::FootPlaceReg>::value, "FootPlaceReg");
    static_assert(std::is_base_of<PathConstraintBase<double, 24, 24, 0>, hkd::GRFConstraint>::value, "GRF");
    static_assert(std::is_base_of<TerminalConstraintBase<double, 24>, hkd::TouchDownConstraint>::value, "TD");
    static_assert(std::is_abstract<CostBase<double, 24, 24, 0>>::value, "CostBase is abstract");
    static_assert(std::is_abstract<SinglePhaseBase<double>>::value, "SinglePhaseBase is abstract");

    // the user cost through the base interface (RCostData / TCostData, HSDDP_CompoundTypes.h:91-150)
    std::shared_ptr<CostBase<double, 24, 24, 0>> cost = std::make_shared<UserFootCost<double>>();
    RCostData<double, 24, 24, 0> rc, sum;
    TCostData<double, 24> tc;
    VecM<double, 24> x, u;
    VecM<double, 0> y;
    for (int j = 0; j < 24; ++j) { x[j] = 0.1 * j; u[j] = -0.05 * j; }
    cost->running_cost(rc, x, u, y, 0.01, 0.0f);
    cost->running_cost_par(rc, x, u, y, 0.01, 0.0f);
    cost->terminal_cost(tc, x, 0.0f);
    cost->terminal_cost_par(tc, x, 0.0f);
    sum.add(rc);
    sum.add(rc);
    CHECK(close(sum.l, 2 * rc.l) && close(sum.lx[7], 2 * 0.01 * 0.7) && close(tc.Phix[3], 0.3));

    // GRF-like path constraint: ReB cost / partials in closed form (ConstraintsBase.h:201-263)
    UserGRF<double> grf;
    grf.update_horizon_len(2);
    grf.create_data();
    REB_Param_Struct<double> rp;
    rp.delta = 0.1; rp.delta_min = 0.01; rp.eps = 2;
    grf.initialize_params(rp);
    for (double fz : {0.5, 0.05}) {  // both branches g > delta, g <= delta
        u[2] = fz;
        grf.compute_violation(x, u, y, 1);
        grf.compute_partial(x, u, y, 1);
        grf.compute_ReB_cost(1);
        grf.compute_ReB_partials(1);
        const double d = 0.1, t = (fz - 2 * d) / d;
        const double b = fz > d ? -std::log(fz) : .5 * (t * t - 1) - std::log(d);
        const double d1 = fz > d ? -1 / fz : (fz - 2 * d) / d / d, d2 = fz > d ? 1 / (fz * fz) : 1 / (d * d);
        CHECK(close(grf.ReB_cost, 2 * b) && close(grf.ReB_grad_u[2], 2 * d1) && close(grf.ReB_hess_u(2, 2), 2 * d2));
    }
    CHECK(grf.max_violation == 0);
    grf.push_back_n(1);
    CHECK(grf.len == 3 && grf.data.size() == 3 && grf.params.size() == 3);
    grf.pop_front_n(2);
    CHECK(grf.len == 1 && grf.data.size() == 1);

    // TD-like terminal constraint: AL cost / partials incl. quirk A4 (ConstraintsBase.h:374-399)
    UserTD<double> td;
    AL_Param_Struct<double> ap;
    ap.sigma = 50; ap.lambda = 1.5; ap.sigma_max = 1e4;
    td.initialize_params(ap);
    x[5] = 0.3;
    td.compute_violation(x);
    td.compute_partial(x);
    td.compute_AL_cost();
    td.compute_AL_partials();
    const double h = 0.3 - 0.1;
    CHECK(close(td.AL_cost, .5 * 50 * h * h + 1.5 * h) && close(td.AL_gradient[5], 50 * h + 1.5));
    CHECK(close(td.AL_hessian(5, 5), 50 * (1 + h) + 1.5) && close(td.max_violation, h));

    // a phase holding the user cost: solve() refuses it (no CPU fallback)
    auto phase = std::make_shared<Phase>();
    auto traj = std::make_shared<Trajectory<double, 24, 24, 0>>(0.01, 5);
    phase->set_trajectory(traj);
    hkd::Dynamics dyn;
    hkd::DynamicsPartial dpar;
    phase->set_dynamics(dyn);
    phase->set_dynamics_partial(dpar);
    phase->add_cost(cost);
    MultiPhaseDDP<double> solver;
    solver.set_multiPhaseProblem({phase});
    solver.set_initial_condition(DVec<double>(24));
    bool refused = false;
    try {
        solver.solve(HSDDP_OPTION());
    } catch (const std::runtime_error &e) {
        refused = std::string(e.what()).find("cost 'User Foot Cost' cannot run on the device") != std::string::npos;
    }
    CHECK(refused);

    // SinglePhaseBase through the facade phase: numerical steps belong to the device solve
    SinglePhaseBase<double> *base = phase.get();
    HSDDP_OPTION opt;
    bool threw = false;
    try {
        base->LQ_approximation(opt);
    } catch (const std::logic_error &) {
        threw = true;
    }
    CHECK(threw);
    CHECK(base->get_state_dim() == 24 && base->get_control_dim() == 24);
    // receding-horizon bookkeeping (SinglePhase.cpp:485-501, TrajectoryManagement.cpp:118-191)
    traj->X.back()[4] = 2.5;
    base->push_back_default();
    CHECK(traj->horizon == 6 && traj->Xbar.size() == 7 && traj->Xbar.back()[4] == 2.5 && traj->K.size() == 7);
    base->pop_front();
    CHECK(traj->horizon == 5 && traj->Ubar.size() == 5 && traj->rcostData.size() == 5);
    UserPhase up;  // a user phase type is a SinglePhaseBase
    CHECK(up.get_state_dim() == 0);

    // the weights the device solve applies come from the registered costs: FootPlaceReg's own foot
    // weights, TrackingCost's tracking weights; phases that disagree are refused (one set per handle)
    auto hkd_phase = [](int N, const std::array<int, 4> &c, const std::array<int, 4> &cn,
                        std::shared_ptr<hkd::TrackingCost> &tc, std::shared_ptr<hkd::FootPlaceReg> &fr) {
        auto ph = std::make_shared<Phase>();
        ph->set_trajectory(std::make_shared<Trajectory<double, 24, 24, 0>>(0.01, N));
        hkd::Dynamics d;
        hkd::DynamicsPartial dp;
        hkd::Resetmap rm;
        hkd::ResetmapPartial rmp;
        d.contact = dp.contact = rm.contact = rmp.contact = c;
        rm.next_contact = rmp.next_contact = cn;
        ph->set_dynamics(d);
        ph->set_dynamics_partial(dp);
        ph->set_resetmap(rm);
        ph->set_resetmap_partial(rmp);
        tc = std::make_shared<hkd::TrackingCost>();
        fr = std::make_shared<hkd::FootPlaceReg>();
        tc->x_ref.assign(N + 1, {});
        tc->u_ref.assign(N + 1, {});
        fr->foot_ref.assign(N + 1, {});
        ph->add_cost(tc);
        ph->add_cost(fr);
        ph->add_pathConstraint(std::make_shared<hkd::GRFConstraint>(c));
        ph->update_SS_config(N + 1);  // every state a shooting state (HKDProblem.cpp:104)
        return ph;
    };
    std::shared_ptr<hkd::TrackingCost> tc0, tc1;
    std::shared_ptr<hkd::FootPlaceReg> fr0, fr1;
    const std::array<int, 4> trot_a{{1, 0, 0, 1}}, trot_b{{0, 1, 1, 0}};
    auto p0 = hkd_phase(4, trot_a, trot_a, tc0, fr0), p1 = hkd_phase(4, trot_a, trot_a, tc1, fr1);
    for (auto &f : {fr0, fr1}) {  // non-default foot weights on the foot term only
        f->weights.foot_w[0] = 2; f->weights.foot_w[1] = 0.5; f->weights.foot_gain = 10; f->weights.foot_term_cost = 7;
    }
    tc0->weights.q_pos[2] = tc1->weights.q_pos[2] = 42;
    MultiPhaseDDP<double> ws;
    ws.set_multiPhaseProblem({p0, p1});
    ws.set_initial_condition(DVec<double>(24));
    const hsddp_problem_desc d0 = ws.describe().desc;
    CHECK(d0.weights.foot_w[0] == 2 && d0.weights.foot_w[1] == 0.5 && d0.weights.foot_gain == 10 &&
          d0.weights.foot_term_cost == 7 && d0.weights.q_pos[2] == 42);
    tc1->weights.q_pos[2] = 41;  // the phases disagree: refused
    bool mixed = false;
    try {
        ws.describe();
    } catch (const std::runtime_error &e) {
        mixed = std::string(e.what()).find("phase 1: tracking weights") != std::string::npos;
    }
    CHECK(mixed);
    tc1->weights.q_pos[2] = 42;
    fr1->weights.foot_w[0] = 3;
    mixed = false;
    try {
        ws.describe();
    } catch (const std::runtime_error &e) {
        mixed = std::string(e.what()).find("phase 1: foot-placement weights") != std::string::npos;
    }
    CHECK(mixed);
    // a contact change at the phase end needs the reset registered; a GRF constraint's contact must be the phase's
    auto q0 = hkd_phase(4, trot_a, trot_b, tc0, fr0), q1 = hkd_phase(4, trot_b, trot_b, tc1, fr1);
    q0->set_resetmap(nullptr);
    q0->set_resetmap_partial(nullptr);
    ws.set_multiPhaseProblem({q0, q1});
    mixed = false;
    try {
        ws.describe();
    } catch (const std::runtime_error &e) {
        mixed = std::string(e.what()).find("no resetmap") != std::string::npos;
    }
    CHECK(mixed);

    // shooting states (SinglePhase::SS_set): the last phase may keep an empty set (HKDProblem::update
    // leaves a new last phase of <= 2 knots without one), any other phase must be all shooting
    auto refused_with = [&](const std::string &needle) {
        try {
            ws.describe();
        } catch (const std::runtime_error &e) {
            return std::string(e.what()).find(needle) != std::string::npos;
        }
        return false;
    };
    auto s0 = hkd_phase(4, trot_a, trot_a, tc0, fr0), s1 = hkd_phase(2, trot_a, trot_a, tc1, fr1);
    fr0->weights = fr1->weights;
    s1->SS_set.clear();
    ws.set_multiPhaseProblem({s0, s1});
    const auto pr = ws.describe();
    CHECK(pr.shooting.size() == 2 && pr.shooting[0] == 5 && pr.shooting[1] == 0);
    s1->update_SS_config(7);  // entries past N are never queried (SinglePhase.cpp:187-220)
    CHECK(ws.describe().shooting[1] == 3);
    s0->SS_set.clear();
    CHECK(refused_with("phase 0: has non-shooting states"));
    s0->SS_set = {0, 2, 3, 4, 5};
    CHECK(refused_with("phase 0: shooting states (SS_set) other than"));
    s0->update_SS_config(5);
    // per-knot reference tables must cover the phase
    tc0->x_ref.pop_back();
    CHECK(refused_with("phase 0: reference tables must match the horizon"));
    tc0->x_ref.push_back({});
    fr1->foot_ref.push_back({});
    CHECK(refused_with("phase 1: reference tables must match the horizon"));
    fr1->foot_ref.pop_back();
    tc1->u_ref.resize(1);
    CHECK(refused_with("phase 1: reference tables must match the horizon"));
    tc1->u_ref.resize(2);  // u_ref needs N rows (the last state slot's control reference is unused)
    CHECK(ws.describe().shooting[0] == 5);

    // dynamics / reset callbacks: exactly the HKD::Model / HKDReset registration (std::bind forwards
    // the solver's own objects) is accepted; a callback that transforms its inputs or post-processes
    // the model's result would be dropped by the device solve, so it is refused
    namespace pc = std::placeholders;
    typedef SinglePhase<double, 24, 24, 0> Ph;
    HKD::Model<double> model;
    VecM<int, 4> cv;
    for (int l = 0; l < 4; ++l) cv[l] = trot_a[l];
    double dtb = 0.01;
    s0->set_dynamics(std::bind(&HKD::Model<double>::dynamics, &model, pc::_1, pc::_2, pc::_3, pc::_4, pc::_5, cv, dtb));
    CHECK(ws.describe().shooting[0] == 5);
    s0->set_dynamics([&](Ph::State &xn, Ph::Output &y, Ph::State &x, Ph::Contrl &u, double t) {
        model.dynamics(xn, y, x, u, t, cv, dtb);
        xn[5] = std::max(xn[5], 0.0);  // user post-processing
    });
    CHECK(refused_with("phase 0: Dynamics is not the HKD registration"));
    s0->set_dynamics([&](Ph::State &xn, Ph::Output &y, Ph::State &x, Ph::Contrl &u, double t) {
        Ph::Contrl u2 = u;  // user-transformed input
        u2[2] += 1;
        model.dynamics(xn, y, x, u2, t, cv, dtb);
    });
    CHECK(refused_with("phase 0: Dynamics is not the HKD registration"));
    s0->set_dynamics([&](Ph::State &xn, Ph::Output &y, Ph::State &x, Ph::Contrl &u, double t) {
        model.dynamics(xn, y, x, u, t, cv, dtb);  // a plain forwarding lambda is the registration
    });
    CHECK(ws.describe().shooting[0] == 5);
    HKDReset<double> reset;
    s0->set_resetmap([&](DVec<double> &xn, DVec<double> &x) {
        reset.resetmap(xn, x, cv, cv);
        xn[0] = 0;
    });
    CHECK(refused_with("phase 0: resetmap / resetmap_partial is not the HKD registration"));
    s0->set_resetmap(std::bind(&HKDReset<double>::resetmap, &reset, pc::_1, pc::_2, cv, cv));
    s0->set_resetmap_partial(std::bind(&HKDReset<double>::resetmap_partial, &reset, pc::_1, pc::_2, cv, cv));
    CHECK(ws.describe().shooting[0] == 5);
    return 0;
}

// the hkd:: plugins' virtuals against the batched primitives they call (one point)
static int device_checks()
{
    hkd::TrackingCost track;
    hkd::FootPlaceReg foot;
    std::array<double, 24> xr{}, ur{};
    std::array<double, 12> pf{};
    for (int j = 0; j < 24; ++j) { xr[j] = 0.01 * j; ur[j] = 0.02 * (j % 5); }
    for (int j = 0; j < 12; ++j) pf[j] = 0.1 * (j % 3) - 0.05;
    for (auto *c : {(hkd::HKDCostRefs *)&track, (hkd::HKDCostRefs *)&foot}) {
        c->contact = {{1, 0, 0, 1}};
        c->x_ref.assign(3, xr);
        c->u_ref.assign(3, ur);
        c->foot_ref.assign(3, pf);
        c->t_start = 0.5f;
        c->knot_dt = 0.01;
    }
    VecM<double, 24> x, u;
    VecM<double, 0> y;
    for (int j = 0; j < 24; ++j) { x[j] = 0.03 * j - 0.2; u[j] = 5.0 + 0.1 * j; }
    RCostData<double, 24, 24, 0> a, b;
    track.running_cost(a, x, u, y, 0.01, 0.51f);
    track.running_cost_par(a, x, u, y, 0.01, 0.51f);
    foot.running_cost(b, x, u, y, 0.01, 0.51f);
    foot.running_cost_par(b, x, u, y, 0.01, 0.51f);
    // the same terms in one primitive call
    const int c[4] = {1, 0, 0, 1};
    double l = 0, lx[24], lu[24], lxx[576], luu[576];
    hkd::detail::on_device({{x.data(), 192}, {u.data(), 192}, {c, 16}, {xr.data(), 192}, {ur.data(), 192}, {pf.data(), 96}},
                           {{&l, 8}, {lx, 192}, {lu, 192}, {lxx, 4608}, {luu, 4608}},
                           [&](std::vector<void *> &i, std::vector<void *> &o) {
                               return hsddp_hkd_running_cost((double *)i[0], (double *)i[1], (int *)i[2], (double *)i[3],
                                                             (double *)i[4], (double *)i[5], &track.weights, 0.01,
                                                             HSDDP_TERM_TRACKING | HSDDP_TERM_FOOT, (double *)o[0],
                                                             (double *)o[1], (double *)o[2], (double *)o[3],
                                                             (double *)o[4], 1, nullptr);
                           });
    CHECK(close(a.l + b.l, l));
    for (int j = 0; j < 24; ++j) CHECK(close(a.lx[j] + b.lx[j], lx[j]) && close(a.lu[j] + b.lu[j], lu[j]));
    for (int e = 0; e < 576; ++e) CHECK(close(a.lxx.data()[e] + b.lxx.data()[e], lxx[e]) && close(a.luu.data()[e] + b.luu.data()[e], luu[e]));
    TCostData<double, 24> ta, tb;
    track.terminal_cost(ta, x, 0.52f);
    track.terminal_cost_par(ta, x, 0.52f);
    foot.terminal_cost(tb, x, 0.52f);
    CHECK(ta.Phi > 0 && tb.Phi > 0 && ta.Phixx(0, 0) > 0);
    // GRF rows: stance legs 0 and 3, 5 rows each (HKDConstraints.cpp:7-33)
    hkd::GRFConstraint grf(std::array<int, 4>{{1, 0, 0, 1}});
    grf.update_horizon_len(1);
    grf.create_data();
    grf.initialize_params();
    grf.compute_violation(x, u, y, 0);
    grf.compute_partial(x, u, y, 0);
    CHECK(grf.size == 10 && close(grf.data[0][0].g, u[2]) && close(grf.data[0][5].g, u[11]) && grf.data[0][6].gu[9] == -1.0);
    // touchdown of legs 1 and 2
    hkd::TouchDownConstraint td(std::array<int, 4>{{0, 1, 1, 0}});
    td.create_data();
    td.initialize_params();
    td.compute_violation(x);
    td.compute_partial(x);
    CHECK(td.size == 2 && td.data[0].hx[5] == 1.0 && td.max_violation >= 0);
    return 0;
}

int main(int argc, char **argv)
{
    try {
        if (host_checks()) return 1;
        if (argc > 1 && std::string(argv[1]) == "gpu" && device_checks()) return 1;
    } catch (const std::exception &e) {
        std::fprintf(stderr, "error: %s\n", e.what());
        return 1;
    }
    std::printf("plugin_check ok\n");
    return 0;
}
