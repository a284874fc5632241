// hkd_mpc.hpp — HKDMPCSolver (HKDMPC/HKDMPC.h:22-100, HKDMPC.cpp:18-298) over the C-ABI, for a
// batch of B robots on one GPU, with the reference's member names and call sequence:
//
//   HKDMPCSolver(reference_file)      loads the quad_reference.csv     (HKDMPC.h:26-31)
//   initialize()                      HKDProblem::initialization + first solve (HKDMPC.cpp:20-94)
//   mpcdata_lcm_handler(msgs)         copies the robot states, starts update() on a worker
//                                     thread (HKDMPC.cpp:166-200)
//   update()                          HKDProblem::update + re-solve with max_AL_iter = 2,
//                                     max_DDP_iter = 1 + update_foot_placement + publish_mpc_cmd
//                                     (HKDMPC.cpp:96-165, 207-298)
//
// Device-side: the phase bookkeeping, warm-start shift, per-knot references, solve and command
// extraction (hsddp_advance, hsddp_solve, hsddp_extract_commands); per tick only the B robot
// states go up and the B commands come back.  LCM is not available on this platform: a message
// is the hkd_data_lcmt struct below and publishing calls a user callback with the
// hkd_command_lcmt records (hsddp_mpc_command).  The worker serialises updates as mpc_mutex does
// in the reference (a new request waits for the running update); wait() joins it.
#ifndef HKD_MPC_HPP
#define HKD_MPC_HPP

#include <chrono>
#include <cmath>
#include <exception>
#include <functional>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../../include/hsddp.h"

namespace hkd {

// hkd_data_lcmt (lcmtypes/hkd_data_lcmt.lcm:1-12), one robot
struct hkd_data_lcmt {
    bool reset_mpc;
    bool MS;
    double mpctime;
    int contact[4];
    float p[3], vWorld[3], rpy[3], omegaBody[3], qJ[12], foot_placements[12];
};

// HKDProblem's configuration (HKDMPC.cpp:26-29)
struct MPCConfig {
    float plan_duration = 0.6f;
    int nsteps_between_mpc = 1;
    float timeStep = 0.01f;
};

class HKDMPCSolver {
public:
    using Publisher = std::function<void(const std::vector<hsddp_mpc_command> &)>;

    // reference_file: quad_reference.csv; batch: robots solved together; settings: ddp_setting.info
    HKDMPCSolver(const std::string &reference_file, int batch, const std::string &settings, int device = 0)
        : B(batch), dev(device), settings_file(settings)
    {
        const int n = hsddp_load_quad_reference(reference_file.c_str(), 0, &dt_ref, nullptr, 0);
        if (n <= 0) throw std::runtime_error(std::string("reference: ") + hsddp_last_error());
        quad_reference.resize(n);
        hsddp_load_quad_reference(reference_file.c_str(), 0, &dt_ref, quad_reference.data(), n);
        hkd_data.resize(B);
        solve_time = 0;
    }
    ~HKDMPCSolver()
    {
        if (worker.joinable()) worker.join();
        if (h) hsddp_destroy(h);
    }
    HKDMPCSolver(const HKDMPCSolver &) = delete;
    HKDMPCSolver &operator=(const HKDMPCSolver &) = delete;

    void set_publisher(Publisher p) { publish = std::move(p); }

    // HKDMPCSolver::initialize (HKDMPC.cpp:20-94): options from the INFO file, the phase plan of
    // the window at the reference's start (QuadReference::initialize), references on the device,
    // the nominal initial state, one full solve
    void initialize()
    {
        std::lock_guard<std::mutex> lk(mpc_mutex);
        hsddp_default_options(&ddp_options);
        chk(hsddp_load_settings(settings_file.c_str(), &ddp_options));
        const int n_win = (int)std::lround(mpc_config.plan_duration / dt_ref) + 2;
        if ((int)quad_reference.size() < n_win) throw std::runtime_error("reference shorter than the plan window");
        dt_mpc = mpc_config.timeStep * mpc_config.nsteps_between_mpc;
        hsddp_phase_plan plan;
        chk(hsddp_plan_phases(quad_reference.data(), n_win, dt_ref, mpc_config.plan_duration, mpc_config.timeStep,
                              dt_mpc, &plan));
        if (h) { hsddp_destroy(h); h = nullptr; }
        hsddp_problem_desc desc{};
        desc.device = dev;
        desc.batch = B;
        desc.n_phases = plan.n_phases;
        for (int i = 0; i < plan.n_phases; ++i) desc.horizons[i] = plan.horizons[i];
        desc.dt = mpc_config.timeStep;
        desc.ref_per_element = 0;
        hsddp_default_weights(&desc.weights);
        hsddp_default_constraint_params(&desc.cparams);
        chk(hsddp_create(&desc, &h));
        chk(hsddp_set_options(h, &ddp_options));
        chk(hsddp_set_reference_table(h, quad_reference.data(), (int)quad_reference.size(), dt_ref));
        const int ws = 0;
        chk(hsddp_build_references(h, &ws, n_win, nullptr, mpc_config.timeStep));
        P = plan.n_phases;
        std::vector<int> contacts((size_t)B * (P + 1) * 4);
        for (int b = 0; b < B; ++b)
            for (int i = 0; i <= P; ++i)
                for (int l = 0; l < 4; ++l) contacts[((size_t)b * (P + 1) + i) * 4 + l] = plan.contacts[i][l];
        // xinit = [body, qdummy]: body = (eul 0, pos (0, 0, 0.2486), 0, 0), qJ = (0, -0.8, 1.6) x 4
        // (HKDMPC.cpp:44-55)
        std::vector<double> x0((size_t)B * 24, 0.0);
        for (int b = 0; b < B; ++b) {
            double *x = &x0[(size_t)b * 24];
            x[5] = 0.2486;
            for (int j = 0; j < 12; ++j) x[12 + j] = j % 3 == 0 ? 0.0 : (j % 3 == 1 ? -0.8 : 1.6);
        }
        compute_hkd_state(x0, contacts, P);
        chk(hsddp_upload_problem(h, contacts.data(), x0.data(), nullptr, nullptr, nullptr));
        hsddp_stats st;
        chk(hsddp_solve(h, &st));
        mpc_time = 0;
        mpc_time_prev = 0;
        mpc_iter = 0;
    }

    // HKDMPCSolver::mpcdata_lcm_handler (HKDMPC.cpp:166-200): msgs[B]
    void mpcdata_lcm_handler(const std::vector<hkd_data_lcmt> &msgs)
    {
        if ((int)msgs.size() != B) throw std::runtime_error("one message per robot");
        wait();  // mpc_mutex: the previous update finishes first
        if (msgs[0].reset_mpc) {
            ddp_options.MS = msgs[0].MS;
            initialize();
            return;
        }
        {
            std::lock_guard<std::mutex> lk(mpc_mutex);
            hkd_data = msgs;
            mpc_time_prev = mpc_time;
            mpc_time = msgs[0].mpctime;
        }
        worker = std::thread([this] {
            try {
                update();
            } catch (...) {
                worker_error = std::current_exception();
            }
        });
    }

    // joins the running update; rethrows its failure
    void wait()
    {
        if (worker.joinable()) worker.join();
        if (worker_error) {
            std::exception_ptr e = worker_error;
            worker_error = nullptr;
            std::rethrow_exception(e);
        }
    }

    // HKDMPCSolver::update (HKDMPC.cpp:96-165)
    void update()
    {
        std::lock_guard<std::mutex> lk(mpc_mutex);
        hsddp_options o = ddp_options;
        o.max_AL_iter = 2;  // quirk A17
        o.max_DDP_iter = 1;
        chk(hsddp_set_options(h, &o));
        mpc_iter++;
        // opt_problem.update(): layout, warm start, references; inputs pending until x0 is known
        std::vector<int> flags(mpc_config.nsteps_between_mpc);
        chk(hsddp_advance(h, mpc_config.nsteps_between_mpc, mpc_config.plan_duration, dt_mpc, nullptr, flags.data()));
        int hz[HSDDP_MAX_PHASES];
        chk(hsddp_get_layout(h, &P, hz, nullptr, nullptr));
        std::vector<int> contacts((size_t)B * (P + 1) * 4);
        durations.assign((size_t)B * P * 4, 0.0);
        chk(hsddp_get_phase_info(h, contacts.data(), durations.data()));
        // xinit = [eul, pos, omega, vel, qdummy] from the robot state (HKDMPC.cpp:121-134)
        std::vector<double> x0((size_t)B * 24);
        for (int b = 0; b < B; ++b) {
            const hkd_data_lcmt &m = hkd_data[b];
            double *x = &x0[(size_t)b * 24];
            for (int a = 0; a < 3; ++a) {
                x[a] = m.rpy[2 - a];
                x[3 + a] = m.p[a];
                x[6 + a] = m.omegaBody[a];
                x[9 + a] = m.vWorld[a];
            }
            for (int j = 0; j < 12; ++j) x[12 + j] = m.qJ[j];
        }
        compute_hkd_state(x0, contacts, P);
        chk(hsddp_update_problem(h, nullptr, x0.data(), nullptr, nullptr, nullptr));
        const auto t0 = std::chrono::high_resolution_clock::now();
        hsddp_stats st;
        chk(hsddp_solve(h, &st));
        const auto t1 = std::chrono::high_resolution_clock::now();
        solve_time = (float)std::chrono::duration<double, std::milli>(t1 - t0).count();
        // update_foot_placement + publish_mpc_cmd (HKDMPC.cpp:207-298)
        std::vector<float> pf((size_t)B * 12);
        for (int b = 0; b < B; ++b)
            for (int j = 0; j < 12; ++j) pf[(size_t)b * 12 + j] = hkd_data[b].foot_placements[j];
        commands.resize(B);
        chk(hsddp_extract_commands(h, mpc_config.nsteps_between_mpc, mpc_time, dt_mpc, durations.data(), 1, pf.data(),
                                   1, solve_time, commands.data()));
        if (publish) publish(commands);
    }

    // per-element results of the last solve
    std::vector<hsddp_element_info> solver_info() const
    {
        std::vector<hsddp_element_info> info(B);
        chk(hsddp_download_element_info(h, info.data()));
        return info;
    }

    int B, dev;
    std::string settings_file;
    MPCConfig mpc_config;
    hsddp_options ddp_options{};
    std::vector<hsddp_quad_state> quad_reference;
    float dt_ref = 0, dt_mpc = 0.01f;
    std::vector<hkd_data_lcmt> hkd_data;
    std::vector<hsddp_mpc_command> commands;
    std::vector<double> durations;
    double mpc_time = 0, mpc_time_prev = 0;
    float solve_time;
    int mpc_iter = 0, P = 0;
    hsddp_handle h = nullptr;

private:
    static void chk(int rc)
    {
        if (rc != HSDDP_OK) throw std::runtime_error(std::string("hsddp: ") + hsddp_last_error());
    }

    // compute_hkd_state (HKD-TrajOpt/HKDModel.h:65-96) for every robot: the qdummy of a stance leg
    // of the first phase is its foot position, computed on the device (hsddp_hkd_foot_position);
    // of a swing leg the joint angles already in x
    void compute_hkd_state(std::vector<double> &x0, const std::vector<int> &contacts, int n_phases)
    {
        const size_t n = (size_t)B * 4;
        std::vector<int> leg(n);
        std::vector<double> xs(n * 24), pfo(n * 3);
        for (int b = 0; b < B; ++b)
            for (int l = 0; l < 4; ++l) {
                leg[(size_t)b * 4 + l] = l;
                std::copy(&x0[(size_t)b * 24], &x0[(size_t)b * 24] + 24, &xs[((size_t)b * 4 + l) * 24]);
            }
        void *dx = hsddp_device_alloc(xs.size() * 8, dev), *dl = hsddp_device_alloc(n * 4, dev),
             *dp = hsddp_device_alloc(pfo.size() * 8, dev);
        int rc = (!dx || !dl || !dp) ? HSDDP_ERR_ALLOC : HSDDP_OK;
        if (!rc) rc = hsddp_memcpy_h2d(dx, xs.data(), xs.size() * 8);
        if (!rc) rc = hsddp_memcpy_h2d(dl, leg.data(), n * 4);
        if (!rc) rc = hsddp_hkd_foot_position((const double *)dx, (const int *)dl, (double *)dp, (int)n, nullptr);
        if (!rc) rc = hsddp_device_synchronize(dev);
        if (!rc) rc = hsddp_memcpy_d2h(pfo.data(), dp, pfo.size() * 8);
        hsddp_device_free(dx); hsddp_device_free(dl); hsddp_device_free(dp);
        chk(rc);
        for (int b = 0; b < B; ++b)
            for (int l = 0; l < 4; ++l)
                if (contacts[((size_t)b * (n_phases + 1)) * 4 + l])
                    for (int a = 0; a < 3; ++a) x0[(size_t)b * 24 + 12 + 3 * l + a] = pfo[((size_t)b * 4 + l) * 3 + a];
    }

    std::mutex mpc_mutex;
    std::thread worker;
    std::exception_ptr worker_error;
    Publisher publish;
};

}  // namespace hkd

#endif
