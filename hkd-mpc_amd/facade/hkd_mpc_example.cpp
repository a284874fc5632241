// hkd_mpc_example — the HKD-MPC application loop (hkdmpc_run: HKDMPCSolver, HKDMPC.cpp) for a
// batch of robots through hkd_mpc.hpp: initialize() from a quad_reference.csv, then `ticks`
// robot-state messages, each answered by update() on the worker thread with one command per robot.
// The robot states are a deterministic synthetic stream (float arithmetic only, reproducible in
// any language); the commands are written out for comparison.
//
//   hkd_mpc_example <quad_reference.csv> <ddp_setting.info> <out_dir> <batch> <ticks>
//   writes <out_dir>/commands.bin: ticks x batch hsddp_mpc_command records,
//          <out_dir>/layout.txt:   per tick the horizons and the solve time (ms)
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iostream>

#include "hkd_mpc.hpp"

// message of robot b at tick t (t >= 1)
static hkd::hkd_data_lcmt message(int t, int b)
{
    hkd::hkd_data_lcmt m{};
    const float ft = (float)t, fb = (float)b;
    m.reset_mpc = false;
    m.MS = true;
    m.mpctime = 0.01 * t;
    m.p[0] = 0.001f * ft + 0.002f * fb; m.p[1] = 0.0005f * fb; m.p[2] = 0.25f;
    m.vWorld[0] = 0.1f;
    m.rpy[0] = 0.002f * fb; m.rpy[1] = 0.001f * ft;
    m.omegaBody[2] = 0.01f * fb;
    const float dq = 0.001f * (float)(t % 5);
    for (int l = 0; l < 4; ++l) {
        m.qJ[3 * l] = dq; m.qJ[3 * l + 1] = -0.8f + dq; m.qJ[3 * l + 2] = 1.6f - dq;
        m.foot_placements[3 * l] = (l < 2 ? 0.2f : -0.2f) + 0.001f * ft;
        m.foot_placements[3 * l + 1] = (l % 2 ? 0.14f : -0.14f);
        m.foot_placements[3 * l + 2] = 0.f;
    }
    return m;
}

int main(int argc, char **argv)
{
    if (argc < 6) {
        std::cerr << "usage: hkd_mpc_example <quad_reference.csv> <ddp_setting.info> <out_dir> <batch> <ticks>\n";
        return 2;
    }
    try {
        const std::string out = argv[3];
        const int B = std::atoi(argv[4]), ticks = std::atoi(argv[5]);
        hkd::HKDMPCSolver mpc(argv[1], B, argv[2]);
        std::ofstream cf(out + "/commands.bin", std::ios::binary), lf(out + "/layout.txt");
        mpc.set_publisher([&](const std::vector<hsddp_mpc_command> &cmds) {
            cf.write((const char *)cmds.data(), (std::streamsize)(cmds.size() * sizeof(hsddp_mpc_command)));
        });
        mpc.initialize();
        for (int t = 1; t <= ticks; ++t) {
            std::vector<hkd::hkd_data_lcmt> msgs(B);
            for (int b = 0; b < B; ++b) msgs[b] = message(t, b);
            mpc.mpcdata_lcm_handler(msgs);
            mpc.wait();
            int P, hz[HSDDP_MAX_PHASES];
            hsddp_get_layout(mpc.h, &P, hz, nullptr, nullptr);
            for (int i = 0; i < P; ++i) lf << hz[i] << (i + 1 < P ? " " : "");
            lf << " | " << mpc.solve_time << "\n";
        }
        const auto info = mpc.solver_info();
        int bad = 0;
        for (const auto &e : info) bad += !(e.cost == e.cost);
        std::printf("hkd_mpc_example: %d robots, %d ticks, last solve %.3f ms, non-finite costs %d\n", B, ticks,
                    mpc.solve_time, bad);
        return bad ? 1 : 0;
    } catch (const std::exception &e) {
        std::cerr << "hkd_mpc_example: " << e.what() << "\n";
        return 1;
    }
}
