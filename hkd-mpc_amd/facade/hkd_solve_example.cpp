// hkd_solve_example — the HKD-MPC call sequence through the C++ facade (hsddp_facade.hpp):
// build the phases as HKDProblem::initialization / create_problem_one_phase do
// (HKDProblem.cpp:15-111, 225-310), then set_multiPhaseProblem -> set_initial_condition -> solve
// (HKDMPC.cpp:57-69), and write the trajectories back out.
//
//   hkd_solve_example <dir> [max_AL_iter max_DDP_iter [ddp_setting.info]]
//   <dir>/problem.txt : P dt N_0 .. N_{P-1}
//   <dir>/contacts.i32 [(P+1)][4], x0.f64 [24], ref_x.f64 [S][24], ref_u.f64 [S][24], ref_foot.f64 [S][12]
//   writes <dir>/Xbar.f64 [S][24], Ubar.f64 [Kc][24], K.f64 [Kc][24][24] (row-major), info.txt, and
//   the Trajectory exports: Xsim.f64 [S][24], A.f64 [Kc][24][24], l.f64 / lx.f64 / luu.f64 (rcostData),
//   Phix.f64 [P][24] (tcostData), G0.f64 [P][24], H0.f64 [P][24][24] (get_value_approx),
//   phase_cost.f64 [P], solver_info.f32 [n][4] (get_solver_info)
#include <cstdio>
#include <fstream>
#include <iostream>

#include "hsddp_facade.hpp"

template <typename V>
static void read_bin(const std::string &path, std::vector<V> &v)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot read " + path);
    f.read((char *)v.data(), (std::streamsize)(v.size() * sizeof(V)));
    if (!f) throw std::runtime_error("short read " + path);
}
template <typename V>
static void write_bin(const std::string &path, const std::vector<V> &v)
{
    std::ofstream f(path, std::ios::binary);
    f.write((const char *)v.data(), (std::streamsize)(v.size() * sizeof(V)));
}

int main(int argc, char **argv)
{
    if (argc < 2) {
        std::cerr << "usage: hkd_solve_example <dir> [max_AL_iter max_DDP_iter]\n";
        return 2;
    }
    try {
        const std::string dir = argv[1];
        std::ifstream pf(dir + "/problem.txt");
        int P;
        double dt;
        pf >> P >> dt;
        std::vector<int> N(P);
        int S = 0;
        for (int i = 0; i < P; ++i) { pf >> N[i]; S += N[i] + 1; }
        std::vector<int> contacts(4 * (P + 1));
        std::vector<double> x0(24), rx(24 * S), ru(24 * S), rf(12 * S);
        read_bin(dir + "/contacts.i32", contacts);
        read_bin(dir + "/x0.f64", x0);
        read_bin(dir + "/ref_x.f64", rx);
        read_bin(dir + "/ref_u.f64", ru);
        read_bin(dir + "/ref_foot.f64", rf);

        std::deque<std::shared_ptr<SinglePhaseBase<double>>> phases;
        std::vector<std::shared_ptr<Trajectory<double, 24, 24, 0>>> trajs;
        int s = 0;
        for (int i = 0; i < P; ++i) {
            auto phase = std::make_shared<SinglePhase<double, 24, 24, 0>>();
            auto traj = std::make_shared<Trajectory<double, 24, 24, 0>>(dt, N[i]);
            auto track = std::make_shared<hkd::TrackingCost>();
            auto foot = std::make_shared<hkd::FootPlaceReg>();
            for (int k = 0; k <= N[i]; ++k) {
                std::array<double, 24> xr, ur;
                std::array<double, 12> fr;
                for (int j = 0; j < 24; ++j) { xr[j] = rx[24 * (s + k) + j]; ur[j] = ru[24 * (s + k) + j]; }
                for (int j = 0; j < 12; ++j) fr[j] = rf[12 * (s + k) + j];
                track->x_ref.push_back(xr);
                track->u_ref.push_back(ur);
                foot->foot_ref.push_back(fr);
                for (int j = 0; j < 24; ++j) traj->Xbar[k][j] = traj->X[k][j] = xr[j];  // HKDProblem.cpp:84-90
            }
            s += N[i] + 1;
            hkd::Dynamics dyn;
            hkd::DynamicsPartial dpar;
            hkd::Resetmap rm;
            hkd::ResetmapPartial rmp;
            hkd::TouchDownConstraint td_proto;
            std::array<int, 4> phase_contact;
            for (int l = 0; l < 4; ++l) {
                phase_contact[l] = dyn.contact[l] = dpar.contact[l] = rm.contact[l] = rmp.contact[l] = td_proto.contact[l] =
                    contacts[4 * i + l];
                rm.next_contact[l] = rmp.next_contact[l] = td_proto.next_contact[l] = contacts[4 * (i + 1) + l];
            }
            dyn.dt = dpar.dt = dt;
            phase->set_trajectory(traj);
            phase->set_dynamics(dyn);
            phase->set_dynamics_partial(dpar);
            phase->set_resetmap(rm);
            phase->set_resetmap_partial(rmp);
            phase->add_cost(track);
            phase->add_cost(foot);
            if (phase_contact[0] + phase_contact[1] + phase_contact[2] + phase_contact[3] > 0)  // HKDProblem.cpp:255-263
                phase->add_pathConstraint(std::make_shared<hkd::GRFConstraint>(phase_contact));
            phase->add_terminalConstraint(std::make_shared<hkd::TouchDownConstraint>(td_proto));
            phase->update_SS_config(N[i] + 1);  // every state a shooting state (HKDProblem.cpp:104)
            phases.push_back(phase);
            trajs.push_back(traj);
        }
        HSDDP_OPTION option;
        if (argc >= 5) loadHSDDPSetting(argv[4], option);  // as HKDMPC does before solving
        if (argc >= 4) {
            option.max_AL_iter = std::atoi(argv[2]);
            option.max_DDP_iter = std::atoi(argv[3]);
        }
        DVec<double> x0v(24);
        for (int j = 0; j < 24; ++j) x0v[j] = x0[j];

        MultiPhaseDDP<double> solver;
        solver.set_multiPhaseProblem(phases);
        solver.set_initial_condition(x0v);
        solver.solve(option);

        std::vector<double> Xb, Ub, K;
        for (int i = 0; i < P; ++i) {
            auto &tr = *trajs[i];
            for (int k = 0; k <= N[i]; ++k)
                for (int j = 0; j < 24; ++j) Xb.push_back(tr.Xbar[k][j]);
            for (int k = 0; k < N[i]; ++k) {
                for (int j = 0; j < 24; ++j) Ub.push_back(tr.Ubar[k][j]);
                for (int a = 0; a < 24; ++a)
                    for (int b = 0; b < 24; ++b) K.push_back(tr.K[k](a, b));
            }
        }
        std::vector<double> Xsim, A, l, lx, luu, Phix, G0, H0, pc;
        for (int i = 0; i < P; ++i) {
            auto &tr = *trajs[i];
            for (int k = 0; k <= N[i]; ++k)
                for (int j = 0; j < 24; ++j) Xsim.push_back(tr.Xsim[k][j]);
            for (int k = 0; k < N[i]; ++k) {
                l.push_back(tr.rcostData[k].l);
                for (int a = 0; a < 24; ++a) {
                    lx.push_back(tr.rcostData[k].lx[a]);
                    for (int b = 0; b < 24; ++b) { A.push_back(tr.A[k](a, b)); luu.push_back(tr.rcostData[k].luu(a, b)); }
                }
            }
            DVec<double> G;
            DMat<double> H;
            phases[i]->get_value_approx(G, H);
            for (int a = 0; a < 24; ++a) {
                Phix.push_back(tr.tcostData.Phix[a]);
                G0.push_back(G[a]);
                for (int b = 0; b < 24; ++b) H0.push_back(H(a, b));
            }
            pc.push_back(phases[i]->get_actual_cost());
        }
        write_bin(dir + "/Xsim.f64", Xsim);
        write_bin(dir + "/A.f64", A);
        write_bin(dir + "/l.f64", l);
        write_bin(dir + "/lx.f64", lx);
        write_bin(dir + "/luu.f64", luu);
        write_bin(dir + "/Phix.f64", Phix);
        write_bin(dir + "/G0.f64", G0);
        write_bin(dir + "/H0.f64", H0);
        write_bin(dir + "/phase_cost.f64", pc);
        write_bin(dir + "/Xbar.f64", Xb);
        write_bin(dir + "/Ubar.f64", Ub);
        write_bin(dir + "/K.f64", K);
        std::vector<float> c, f, e, q, hist;
        solver.get_solver_info(c, f, e, q);
        for (size_t n = 0; n < c.size(); ++n) hist.insert(hist.end(), {c[n], f[n], e[n], q[n]});
        write_bin(dir + "/solver_info.f32", hist);
        const hsddp_element_info &info = solver.element_info();
        std::ofstream out(dir + "/info.txt");
        out.precision(17);
        out << solver.get_actual_cost() << " " << solver.measure_dynamics_feasibility() << " " << info.iters << " " << info.outer_iters << " "
            << info.status << " " << info.n_ls_trials << "\n";
        std::printf("facade solve ok: cost %.17g iters %d\n", solver.get_actual_cost(), info.iters);
    } catch (const std::exception &ex) {
        std::cerr << "error: " << ex.what() << "\n";
        return 1;
    }
    return 0;
}
