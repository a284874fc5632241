// facade_check — host-only checks of the C++ facade (no device needed): option defaults and the
// INFO loader round-trip through the C-ABI, and a phase with a non-HKD plugin is rejected before
// any device work (no CPU fallback exists).
#include <cstdio>

#include "hsddp_facade.hpp"

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            std::fprintf(stderr, "check failed: %s (line %d)\n", #c, __LINE__); \
            return 1;                                                    \
        }                                                                \
    } while (0)

int main(int argc, char **argv)
{
    HSDDP_OPTION o;
    hsddp_options c;
    hsddp_default_options(&c);
    CHECK(o.alpha == c.alpha && o.gamma == c.gamma && o.max_DDP_iter == c.max_DDP_iter);
    CHECK(o.update_regularization == c.update_regularization && o.MS == (bool)c.MS);
    if (argc > 1) {  // settings/ddp_setting.info
        HSDDP_OPTION f;
        loadHSDDPSetting(argv[1], f);
        hsddp_options cf;
        hsddp_default_options(&cf);
        CHECK(hsddp_load_settings(argv[1], &cf) == HSDDP_OK);
        CHECK(f.max_AL_iter == cf.max_AL_iter && f.cost_thresh == cf.cost_thresh && f.merit_offset == cf.merit_offset);
    }
    // a user-defined dynamics callback cannot run on the device: solve() must refuse it
    auto phase = std::make_shared<SinglePhase<double, 24, 24, 0>>();
    phase->set_trajectory(std::make_shared<Trajectory<double, 24, 24, 0>>(0.01, 5));
    phase->set_dynamics([](SinglePhase<double, 24, 24, 0>::State &, SinglePhase<double, 24, 24, 0>::Output &,
                           SinglePhase<double, 24, 24, 0>::State &, SinglePhase<double, 24, 24, 0>::Contrl &,
                           double) {});
    MultiPhaseDDP<double> solver;
    solver.set_multiPhaseProblem({phase});
    solver.set_initial_condition(DVec<double>(24));
    bool threw = false;
    try {
        solver.solve(o);
    } catch (const std::runtime_error &e) {
        threw = std::string(e.what()).find("Dynamics is not the HKD registration") != std::string::npos;
    }
    CHECK(threw);
    std::printf("facade_check ok\n");
    return 0;
}
