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

#include <cstring>
#include <vector>

#pragma clang fp contract(off)

double fpf_feeder_bkva(const fpf_feeder *f);   // fpf_api.cpp

extern "C" int fpf_vvc_line_search(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *g,
                                   const double *load_nodes, const int *n_loads, int ld, double c0, double alpha,
                                   int m_max, double ploss_orig, fpf_line_search *res) {
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
    // [6][Nl][M]: every candidate starts as ctrl_o's loads (Dl_new persists
    // across iterations and only the SST rows change, :1320-1372)
    std::vector<double> pq((size_t)6 * nlz * M);
    for (int c = 0; c < 6; ++c)
        for (size_t r = 0; r < nlz; ++r) {
            const double v = ctrl_dl[r + (size_t)(6 + c) * nlz];
            double *dst = &pq[((size_t)c * nlz + r) * M];
            for (int m = 0; m < M; ++m) dst[m] = v;
        }
    double cvq = c0;
    for (int m = 0; m < M; ++m) {
        for (int x = 0; x < 3; ++x) {
            const int col = 7 + 2 * x;   // Q of phase x
            for (int i = 0; i < n_loads[x]; ++i) {
                const double node = load_nodes[(size_t)x * ld + i];
                const double gupdate = g[(size_t)x * ld + i] * (bkva / 3) * cvq;
                for (size_t r = 0; r < nlz; ++r)
                    if (ctrl_dl[r + 2 * nlz] == node)
                        pq[((size_t)(col - 6) * nlz + r) * M + m] = ctrl_dl[r + (size_t)col * nlz] - gupdate;
            }
        }
        cvq = alpha * cvq;   // :1420-1422
    }
    std::vector<signed char> status(M);
    std::vector<int> iters(M);
    fpf_outputs out;
    std::memset(&out, 0, sizeof(out));
    out.iters = iters.data();
    out.status = status.data();
    out.loss = res->loss;
    out.vmin = res->vmin;
    out.vmax = res->vmax;
    const int rc = fpf::solve_batch_host(feeder, M, pq.data(), &out, nullptr, FPF_LAYOUT_SCEN_FASTEST);
    if (rc < 0) return rc;
    res->first_nonconv = -1;
    for (int m = 0; m < M; ++m)
        if (status[m] != FPF_CONVERGED) {
            res->first_nonconv = m;
            break;
        }
    // the reference's loop (:1330-1540): keep c_m while the next size lowers the loss
    res->stop = -1;
    res->reverse = 0;
    for (int m = 0; m < m_max; ++m) {
        if (res->loss[m + 1] > res->loss[m]) {
            res->stop = m;
            break;
        }
        if (res->loss[m] > ploss_orig) res->reverse = 1;   // Ploss_aftter_ctrl > Ploss_orig
    }
    return rc;
}
