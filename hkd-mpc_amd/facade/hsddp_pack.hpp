// hsddp_pack.hpp — packing between the reference's per-phase Trajectory objects and the C-ABI's
// flat arrays (include/hsddp.h: state slots phase-major, S = sum(N_i + 1); control slots
// Kc = sum N_i; matrices row-major).
//
// Templates over the trajectory type: they use only the member names and element access of the
// reference's Trajectory (TrajectoryManagement.h:49-81: deques Xbar, X, Ubar, U, Defect, dX, dU,
// A, B, K, rcostData with v[j] / m(a, b) access), so the same code packs the facade's Trajectory
// (hsddp_facade.hpp, used by MultiPhaseDDP::solve there) and the reference's Eigen-based one (the
// binding in INTEGRATION.md §1).  Eigen stores matrices column-major; m(a, b) reads it in place.
#ifndef HSDDP_PACK_HPP
#define HSDDP_PACK_HPP

#include <stdexcept>
#include <vector>

namespace hsddp_pack {

constexpr int NX = 24, NU = 24;

// horizons (N_i = horizon), dt (the first phase's timeStep), S and Kc of a phase list
template <class TrajPtr>
void layout(const std::vector<TrajPtr> &trajs, int *horizons, double &dt, int &S, int &Kc)
{
    S = Kc = 0;
    for (size_t i = 0; i < trajs.size(); ++i) {
        if (!trajs[i]) throw std::runtime_error("phase " + std::to_string(i) + " has no trajectory");
        horizons[i] = trajs[i]->horizon;
        S += horizons[i] + 1;
        Kc += horizons[i];
    }
    dt = trajs.empty() ? 0.0 : (double)trajs[0]->timeStep;
}

// Xbar [S][24], Ubar [Kc][24], K [Kc][24][24] (row-major) from the trajectories (warm start)
template <class TrajPtr>
void pack_trajectories(const std::vector<TrajPtr> &trajs, std::vector<double> &Xbar, std::vector<double> &Ubar,
                       std::vector<double> &K)
{
    Xbar.clear(); Ubar.clear(); K.clear();
    for (auto &t : trajs) {
        for (int k = 0; k <= t->horizon; ++k)
            for (int j = 0; j < NX; ++j) Xbar.push_back(t->Xbar[k][j]);
        for (int k = 0; k < t->horizon; ++k) {
            for (int j = 0; j < NU; ++j) Ubar.push_back(t->Ubar[k][j]);
            for (int a = 0; a < NU; ++a)
                for (int b = 0; b < NX; ++b) K.push_back(t->K[k](a, b));
        }
    }
}

// the solution back into the trajectories (hsddp_download_trajectory layout)
template <class TrajPtr>
void unpack_trajectories(const std::vector<TrajPtr> &trajs, const double *Xbar, const double *Ubar, const double *K)
{
    size_t s = 0, kc = 0;
    for (auto &t : trajs) {
        for (int k = 0; k <= t->horizon; ++k, ++s)
            for (int j = 0; j < NX; ++j) t->Xbar[k][j] = Xbar[NX * s + j];
        for (int k = 0; k < t->horizon; ++k, ++kc) {
            for (int j = 0; j < NU; ++j) t->Ubar[k][j] = Ubar[NU * kc + j];
            for (int a = 0; a < NU; ++a)
                for (int b = 0; b < NX; ++b) t->K[k](a, b) = K[NU * NX * kc + NX * a + b];
        }
    }
}

// the working trajectory (hsddp_download_working): X, Defect, dX per state slot, U, dU per control
// slot; Xsim = X + Defect (Defect = Xsim - X, TrajectoryManagement.cpp:193-199)
template <class TrajPtr>
void unpack_working(const std::vector<TrajPtr> &trajs, const double *X, const double *U, const double *D,
                    const double *dX, const double *dU)
{
    size_t s = 0, kc = 0;
    for (auto &t : trajs) {
        for (int k = 0; k <= t->horizon; ++k, ++s)
            for (int j = 0; j < NX; ++j) {
                t->X[k][j] = X[NX * s + j];
                t->Defect[k][j] = D[NX * s + j];
                t->Xsim[k][j] = X[NX * s + j] + D[NX * s + j];
                t->dX[k][j] = dX[NX * s + j];
            }
        for (int k = 0; k < t->horizon; ++k, ++kc)
            for (int j = 0; j < NU; ++j) {
                t->U[k][j] = U[NU * kc + j];
                t->dU[k][j] = dU[NU * kc + j];
            }
    }
}

// the LQ model (hsddp_download_lq, row-major) into Trajectory::A, B and rcostData (l, lx, lu, lxx,
// luu; lux = 0)
template <class TrajPtr>
void unpack_lq(const std::vector<TrajPtr> &trajs, const double *A, const double *B, const double *l, const double *lx,
               const double *lu, const double *lxx, const double *luu)
{
    size_t kc = 0;
    for (auto &t : trajs)
        for (int k = 0; k < t->horizon; ++k, ++kc) {
            auto &r = t->rcostData[k];
            r.l = l[kc];
            for (int a = 0; a < NX; ++a) {
                r.lx[a] = lx[NX * kc + a];
                r.lu[a] = lu[NU * kc + a];
                for (int b = 0; b < NX; ++b) {
                    t->A[k](a, b) = A[NX * NX * kc + NX * a + b];
                    t->B[k](a, b) = B[NX * NU * kc + NU * a + b];
                    r.lxx(a, b) = lxx[NX * NX * kc + NX * a + b];
                    r.luu(a, b) = luu[NU * NU * kc + NU * a + b];
                    r.lux(a, b) = 0;
                }
            }
        }
}

// terminal data (hsddp_download_terminal) into Trajectory::tcostData and the value function at
// each phase start (hsddp_download_value) into G[0], H[0]; either of G, H may be null
template <class TrajPtr>
void unpack_terminal_value(const std::vector<TrajPtr> &trajs, const double *Phi, const double *Phix,
                           const double *Phixx, const double *G, const double *H)
{
    for (size_t i = 0; i < trajs.size(); ++i) {
        auto &t = trajs[i];
        t->tcostData.Phi = Phi[i];
        for (int a = 0; a < NX; ++a) {
            t->tcostData.Phix[a] = Phix[NX * i + a];
            if (G) t->G[0][a] = G[NX * i + a];
            for (int b = 0; b < NX; ++b) {
                t->tcostData.Phixx(a, b) = Phixx[NX * NX * i + NX * a + b];
                if (H) t->H[0](a, b) = H[NX * NX * i + NX * a + b];
            }
        }
    }
}

// per-slot references rx, ru [S][24], rf [S][12] from get(i, k, xr, ur, pf) for every knot k = 0..N_i
// of every phase (the reference's HKDSinglePhaseReference::get_reference_at_t, HKDReference.cpp:8-57)
template <class F>
void pack_references(int n_phases, const int *horizons, F get, std::vector<double> &rx, std::vector<double> &ru,
                     std::vector<double> &rf)
{
    rx.clear(); ru.clear(); rf.clear();
    double xr[NX], ur[NU], pf[12];
    for (int i = 0; i < n_phases; ++i)
        for (int k = 0; k <= horizons[i]; ++k) {
            get(i, k, xr, ur, pf);
            rx.insert(rx.end(), xr, xr + NX);
            ru.insert(ru.end(), ur, ur + NU);
            rf.insert(rf.end(), pf, pf + 12);
        }
}

}  // namespace hsddp_pack

#endif  // HSDDP_PACK_HPP
