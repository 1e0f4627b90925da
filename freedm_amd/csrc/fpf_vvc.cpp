// fpf_vvc.cpp -- the VVC module's step-size search as one batched solve
// (include/freedm_pf.h: fpf_vvc_line_search).
//
// The reference (Broker/src/vvc/VoltVarCtrl.cpp:1316-1542) walks the step sizes
// c_m = c0 * alpha^m one at a time and calls DPF_return7 twice per step (the
// current and the next size; half the calls repeat the previous step's).  Every
// candidate is independent, so all m_max + 1 of them go to the GPU as one batch
// and the reference's stop rule runs over the returned losses.
#include "../../include/freedm_pf.h"
#include "fpf_internal.h"

#include <cmath>
#include <cstring>
#include <vector>

#pragma clang fp contract(off)

double fpf_feeder_bkva(const fpf_feeder *f);   // fpf_api.cpp

namespace fpf {
// The step-size search; lazy > 0 (fpf_vvc_round): the candidates in batches, the
// first of `lazy` sizes, the rest only when the stop rule did not fire inside the
// first -- the reference itself never solves a candidate past stop + 1, and the
// large sizes are the slow ones (the demo feeder's candidates 0..31 take 5 sweeps,
// its last ones 14-20; a wavefront sweeps until its slowest scenario is done).
// Candidates not solved get NaN losses / extremes and count as neither converged
// nor not.
int vvc_line_search(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *g,
                    const double *load_nodes, const int *n_loads, int ld, double c0, double alpha, int m_max,
                    double ploss_orig, fpf_line_search *res, int lazy) {
    if (!feeder || !ctrl_dl || !g || !load_nodes || !n_loads || !res || !res->loss || m_max < 1 || ld < 0 ||
        ncols < 12)
        return FPF_ERR_ARG;
    fpf_feeder_info in;
    if (fpf_feeder_get_info(feeder, &in) != FPF_OK || in.nl != nl) return FPF_ERR_ARG;
    for (int x = 0; x < 3; ++x)
        if (n_loads[x] < 0 || n_loads[x] > ld) return FPF_ERR_ARG;
    const double bkva = fpf_feeder_bkva(feeder);   // sysinfo.bkva of the candidate update (:1360)
    const int M = m_max + 1;
    const size_t nlz = (size_t)nl;
    // c_m = c0 alpha^m as the reference forms it, one product per step (:1420-1422)
    std::vector<double> cv(M);
    cv[0] = c0;
    for (int m = 1; m < M; ++m) cv[m] = alpha * cv[m - 1];
    // the rows each load node's Q update goes to
    std::vector<std::vector<size_t>> rows_of(3 * (size_t)std::max(ld, 1));
    for (int x = 0; x < 3; ++x)
        for (int i = 0; i < n_loads[x]; ++i)
            for (size_t r = 0; r < nlz; ++r)
                if (ctrl_dl[r + 2 * nlz] == load_nodes[(size_t)x * ld + i]) rows_of[(size_t)x * ld + i].push_back(r);
    std::vector<signed char> status(M, (signed char)-1);
    std::vector<int> iters(M, 0);
    std::vector<double> pq;
    // solve candidates [m0, m1): [6][Nl][m1 - m0], every candidate starting as
    // ctrl_o's loads (Dl_new persists across iterations and only the SST rows
    // change, :1320-1372)
    auto solve = [&](int m0, int m1) -> int {
        const size_t K = (size_t)(m1 - m0);
        pq.assign((size_t)6 * nlz * K, 0.0);
        for (int c = 0; c < 6; ++c)
            for (size_t r = 0; r < nlz; ++r) {
                const double v = ctrl_dl[r + (size_t)(6 + c) * nlz];
                double *dst = &pq[((size_t)c * nlz + r) * K];
                for (size_t m = 0; m < K; ++m) dst[m] = v;
            }
        for (int m = m0; m < m1; ++m)
            for (int x = 0; x < 3; ++x) {
                const int col = 7 + 2 * x;   // Q of phase x
                for (int i = 0; i < n_loads[x]; ++i) {
                    const double gupdate = g[(size_t)x * ld + i] * (bkva / 3) * cv[m];
                    for (size_t r : rows_of[(size_t)x * ld + i])
                        pq[((size_t)(col - 6) * nlz + r) * K + (m - m0)] = ctrl_dl[r + (size_t)col * nlz] - gupdate;
                }
            }
        fpf_outputs out;
        std::memset(&out, 0, sizeof(out));
        out.iters = iters.data() + m0;
        out.status = status.data() + m0;
        out.loss = res->loss + m0;
        out.vmin = res->vmin ? res->vmin + m0 : nullptr;
        out.vmax = res->vmax ? res->vmax + m0 : nullptr;
        return fpf::solve_batch_host(feeder, (int)K, pq.data(), &out, nullptr, FPF_LAYOUT_SCEN_FASTEST);
    };
    // the reference's loop (:1330-1540) over the solved candidates [0, solved):
    // keep c_m while the next size lowers the loss
    res->stop = -1;
    res->reverse = 0;
    int solved = 0, m = 0, rc = 0;
    const int first = lazy > 1 && lazy < M ? lazy : M;
    while (solved < M) {
        const int m1 = solved == 0 ? first : M;
        const int r = solve(solved, m1);
        if (r < 0) return r;
        rc += r;
        solved = m1;
        for (; m < m_max && m + 1 < solved; ++m) {
            if (res->loss[m + 1] > res->loss[m]) {
                res->stop = m;
                break;
            }
            if (res->loss[m] > ploss_orig) res->reverse = 1;   // Ploss_aftter_ctrl > Ploss_orig
        }
        if (res->stop >= 0) break;
    }
    for (int k = solved; k < M; ++k) {
        res->loss[k] = NAN;
        if (res->vmin) res->vmin[k] = NAN;
        if (res->vmax) res->vmax[k] = NAN;
    }
    res->first_nonconv = -1;
    for (int k = 0; k < solved; ++k)
        if (status[k] != FPF_CONVERGED) {
            res->first_nonconv = k;
            break;
        }
    return rc;
}
}  // namespace fpf

extern "C" int fpf_vvc_line_search(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *g,
                                   const double *load_nodes, const int *n_loads, int ld, double c0, double alpha,
                                   int m_max, double ploss_orig, fpf_line_search *res) {
    return fpf::vvc_line_search(feeder, ctrl_dl, nl, ncols, g, load_nodes, n_loads, ld, c0, alpha, m_max, ploss_orig,
                                res, 0);
}
