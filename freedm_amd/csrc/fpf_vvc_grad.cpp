// fpf_vvc_grad.cpp -- the VVC module's gradient stage and its whole round
// (include/freedm_pf.h: fpf_vvc_gradient, fpf_vvc_round).
//
// The reference runs once per VVC round, after the base DPF
// (Broker/src/vvc/VoltVarCtrl.cpp:1141-1325):
//   per phase x, over the branches whose self impedance is nonzero
//   (form_Yabc.cpp:8-260) -- the admittance matrix Y_x of the self
//   impedances, the bus voltages in polar form (V_abc_list.cpp), the
//   branches renamed to V-list positions (rename_brn.cpp), dF/dtheta and dF/dV
//   of the loss F (form_Ftheta.cpp, form_Fv.cpp), the polar power-flow
//   Jacobian J = [H N; K L] (form_J.cpp), lambda = -inv(J^T) Fx, and the
//   gradient with respect to the SST reactive injections, g = -gu^T lambda.
// It is a few hundred buses solved once per 9 s round with long double
// accumulators (the F and J sums), so it runs on the host in x87 extended
// precision exactly like the reference's build; the DPF solves around it run
// on the GPU.  inv() is LAPACK in the reference; here one LU solve with partial
// pivoting (agreement to rounding: tests/test_vvc_round.py).
#include "../../include/freedm_pf.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <complex>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "fpf_gradb.h"
#include "fpf_internal.h"

#pragma clang fp contract(off)

namespace {

typedef std::complex<double> cplx;
const double kPi = 3.14159265358979323846;   // form_Ftheta.cpp:11

struct Table {   // column-major Dl view
    const double *d;
    int nl;
    double operator()(int r, int c) const { return d[(size_t)c * nl + r]; }
};

// One phase's network as the gradient sees it.
struct PhaseNet {
    int lnum = 0;                       // Lnum_x: branches with a nonzero self impedance
    std::vector<cplx> sbus, rbus, zself; // rows of brnches for this phase (VoltVarCtrl.cpp:408-433)
    std::vector<cplx> Y;                // (lnum+1)^2, column-major (form_Yabc.cpp:118-220)
    std::vector<double> V, theta, node; // V_abc_list (lnum+1 each)
    std::vector<int> vrow;              // the Vpolar row of each V_abc_list entry (-1: none, V = 0)
    int scan_end = 0;                   // V_abc_list scanned Vpolar rows [0, scan_end)
    std::vector<int> s, r;              // renamed branch ends (rename_brn.cpp)
    cplx y(int a, int b) const { return Y[(size_t)a + (size_t)b * (lnum + 1)]; }
};

// Solve A x = b by LU with partial pivoting (A n x n column-major, b -> x).
// lambda = -inv(J^T) Fx needs one solve, not the inverse the reference forms
// (LAPACK getri, then a product): n^3 / 3 operations instead of n^3, the same
// result to rounding (1e-10 against the oracle's inverse, tests/test_vvc_round.py).
// The elimination runs column by column (contiguous in column-major storage).
bool lu_solve(std::vector<double> a, int n, std::vector<double> &x) {
    auto A = [&](int r, int c) -> double & { return a[(size_t)r + (size_t)c * n]; };
    for (int k = 0; k < n; ++k) {
        int p = k;
        double best = std::fabs(A(k, k));
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(A(i, k)) > best) {
                best = std::fabs(A(i, k));
                p = i;
            }
        if (best == 0) return false;
        if (p != k) {
            for (int j = 0; j < n; ++j) std::swap(A(k, j), A(p, j));
            std::swap(x[k], x[p]);
        }
        const double piv = A(k, k);
        double *ck = &A(0, k);
        for (int i = k + 1; i < n; ++i) ck[i] /= piv;
        for (int j = k + 1; j < n; ++j) {
            const double akj = A(k, j);
            if (akj == 0) continue;
            double *cj = &A(0, j);
            for (int i = k + 1; i < n; ++i) cj[i] -= ck[i] * akj;
        }
        const double xk = x[k];
        if (xk != 0)
            for (int i = k + 1; i < n; ++i) x[i] -= ck[i] * xk;
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = x[i];
        for (int k = i + 1; k < n; ++k) v -= A(i, k) * x[k];
        x[i] = v / A(i, i);
    }
    return true;
}

}  // namespace

// Everything of the gradient but the numbers that depend on the voltages'
// values: the load lists, the per-phase branch lists and Y, the V_abc_list rows
// (from vpolar's nonzero pattern) and the renamed branch ends; P.V / P.theta are
// filled from vpolar as well (the host path).
struct GradPlan {
    int cnt_nodes = 0, lload[3] = {0, 0, 0};
    std::vector<double> node_f, loads[3];
    PhaseNet ph[3];
};

namespace {
int build_plan(const Table &t, int ncols, const double *z, int z_rows, const double *vpolar, int nn, double bkva,
               double bkv, GradPlan &plan, std::string *err) {
    const int nl = t.nl;
    if (ncols < 12) return FPF_ERR_ARG;
    // ---- Node_f and Load_a/b/c (VoltVarCtrl.cpp:354-398): (int) tests, and the scan
    // stops at the first full counter
    int cnt_nodes = 1;
    int *const lload = plan.lload;
    for (int i = 0; i < nl; ++i) {
        if ((int)t(i, 0) != 0) ++cnt_nodes;
        for (int x = 0; x < 3; ++x)
            if ((int)t(i, 6 + 2 * x) != 0) ++lload[x];
    }
    plan.cnt_nodes = cnt_nodes;
    std::vector<double> &node_f = plan.node_f;
    std::vector<double> *const loads = plan.loads;
    node_f.assign(cnt_nodes, 0.0);
    for (int x = 0; x < 3; ++x) loads[x].assign(lload[x], 0.0);
    {
        int jn = 1, jl[3] = {0, 0, 0};
        for (int i = 0; i < nl && jn < cnt_nodes && jl[0] < lload[0] && jl[1] < lload[1] && jl[2] < lload[2]; ++i) {
            if ((int)t(i, 2) != 0) node_f[jn++] = t(i, 2);
            for (int x = 0; x < 3; ++x)
                if ((int)t(i, 6 + 2 * x) != 0) loads[x][jl[x]++] = t(i, 2);
        }
    }
    // ---- branches with the self impedances of each phase (form_Yabc.cpp:11-45)
    const double Zb = std::pow(bkv, 2) / bkva * 1000;
    struct Br { cplx s, r, z[3]; };
    std::vector<Br> br;
    size_t lbr = 0;   // Lbr: rows with ln > 0 (form_Yabc.cpp:15-16)
    for (int i = 0; i < nl; ++i)
        if (t(i, 0) > 0) ++lbr;
    for (int i = 0; i < nl && br.size() < lbr; ++i) {
        if ((int)t(i, 0) == 0) continue;
        const int code = (int)t(i, 3), idx = 3 * (code - 1);
        if (idx < 0 || idx + 2 >= z_rows) {
            *err = "line code " + std::to_string(code) + " outside Z";
            return FPF_ERR_TOPOLOGY;
        }
        Br b;
        b.s = t(i, 1);
        b.r = t(i, 2);
        for (int x = 0; x < 3; ++x) {
            const size_t zi = (size_t)(idx + x) + (size_t)x * z_rows;
            const cplx zz(z[2 * zi], z[2 * zi + 1]);
            b.z[x] = code == 7 ? zz : t(i, 4) * zz / Zb;
        }
        br.push_back(b);
    }
    PhaseNet *const ph = plan.ph;
    for (int x = 0; x < 3; ++x)
        for (const Br &b : br)
            if (std::abs(b.z[x]) > 0) ++ph[x].lnum;
    {
        size_t fill[3] = {0, 0, 0};
        for (int x = 0; x < 3; ++x) {
            ph[x].sbus.assign(ph[x].lnum, 0.0);
            ph[x].rbus.assign(ph[x].lnum, 0.0);
            ph[x].zself.assign(ph[x].lnum, 0.0);
        }
        for (size_t i = 0; i < br.size() && fill[0] < (size_t)ph[0].lnum && fill[1] < (size_t)ph[1].lnum &&
                           fill[2] < (size_t)ph[2].lnum;
             ++i)
            for (int x = 0; x < 3; ++x)
                if (std::abs(br[i].z[x]) != 0) {
                    ph[x].sbus[fill[x]] = br[i].s;
                    ph[x].rbus[fill[x]] = br[i].r;
                    ph[x].zself[fill[x]] = br[i].z[x];
                    ++fill[x];
                }
    }
    for (int x = 0; x < 3; ++x) {
        PhaseNet &P = ph[x];
        const int L = P.lnum, n = L + 1;
        if (L == 0) {
            *err = "a phase without branches";
            return FPF_ERR_TOPOLOGY;
        }
        // Y over ka = [first sbus, every rbus] (form_Yabc.cpp:118-156)
        std::vector<cplx> yy(L);
        for (int i = 0; i < L; ++i) yy[i] = cplx(1.0, 0.0) / P.zself[i];
        std::vector<int> ka(n);
        ka[0] = (int)P.sbus[0].real();
        for (int i = 0; i < L; ++i) ka[i + 1] = (int)P.rbus[i].real();
        // (form_Yabc's loops visit, per entry, the branches in order: the diagonal
        // adds every branch touching ka[m], an off-diagonal subtracts first the
        // branches s -> r, then those r -> s.  Assembled here branch by branch from
        // the positions of each bus in ka -- the same additions per entry in the same
        // order, O(L) instead of O(n^2 L))
        P.Y.assign((size_t)n * n, 0.0);
        {
            std::vector<std::vector<int>> at_node;
            auto pos = [&](int node) -> const std::vector<int> & {
                static const std::vector<int> none;
                return node >= 0 && node < (int)at_node.size() ? at_node[node] : none;
            };
            int mx = 0;
            for (int m = 0; m < n; ++m) mx = std::max(mx, ka[m]);
            at_node.resize((size_t)mx + 1);
            for (int m = 0; m < n; ++m)
                if (ka[m] >= 0) at_node[ka[m]].push_back(m);
            for (int i = 0; i < L; ++i) {
                const int si = (int)P.sbus[i].real(), ri = (int)P.rbus[i].real();
                // diagonal: once per m with ka[m] == si or ka[m] == ri
                for (int m : pos(si)) P.Y[(size_t)m + (size_t)m * n] += yy[i];
                if (ri != si)
                    for (int m : pos(ri)) P.Y[(size_t)m + (size_t)m * n] += yy[i];
            }
            // off-diagonal: all s -> r contributions of an entry precede its r -> s ones
            for (int pass = 0; pass < 2; ++pass)
                for (int i = 0; i < L; ++i) {
                    const int si = (int)P.sbus[i].real(), ri = (int)P.rbus[i].real();
                    const int a = pass == 0 ? si : ri, b = pass == 0 ? ri : si;
                    for (int m : pos(a))
                        for (int q : pos(b))
                            if (m != q) P.Y[(size_t)m + (size_t)q * n] -= yy[i];
                }
        }
        // V_abc_list (V_abc_list.cpp): the first n rows with a nonzero |V| of this phase
        P.V.assign(n, 0.0);
        P.theta.assign(n, 0.0);
        P.node.assign(n, 0.0);
        P.vrow.assign(n, -1);
        {
            int i = 0;
            for (int j = 0; i < nn && j < n; ++i) {
                const double mag = vpolar[i + (size_t)(2 * x) * nn];
                if (mag != 0) {
                    P.V[j] = mag;
                    P.theta[j] = vpolar[i + (size_t)(2 * x + 1) * nn];
                    P.node[j] = i < cnt_nodes ? node_f[i] : 0.0;
                    P.vrow[j] = i;
                    ++j;
                }
            }
            P.scan_end = i;
        }
        // rename_brn: each end to its position in the V list (the last match wins)
        P.s.assign(L, 0);
        P.r.assign(L, 0);
        for (int i = 0; i < L; ++i) {
            double s_new = P.sbus[i].real(), r_new = P.rbus[i].real();
            for (int j = 0; j < n; ++j) {
                if (std::round(P.sbus[i].real()) == std::round(P.node[j])) s_new = j;
                else if (std::round(P.rbus[i].real()) == std::round(P.node[j])) r_new = j;
            }
            P.s[i] = (int)s_new;
            P.r[i] = (int)r_new;
        }
    }
    return FPF_OK;
}

// The numbers at the plan's voltages (P.V, P.theta): Fx, J, lambda, g (host).
int numeric(GradPlan &plan, double bkva, double beta0, int ld, double *g, double *load_nodes, int *n_loads,
            double *stats, std::string *err) {
    const int *const lload = plan.lload;
    const std::vector<double> *const loads = plan.loads;
    double gmin = INFINITY, gmax = -INFINITY;
    for (int x = 0; x < 3; ++x) {
        PhaseNet &P = plan.ph[x];
        const int L = P.lnum, n = L + 1;
        // Fx = [dF/dtheta; dF/dV] over the n-1 non-reference buses
        const int m1 = n - 1, nf = 2 * m1;
        std::vector<double> Fx(nf, 0.0);
        for (int i = 0; i < m1; ++i) {
            long double Rt = 0, Rv = 0;
            for (int j = 0; j < L; ++j) {
                const int s = P.s[j], r = P.r[j];
                if (s != i + 1 && r != i + 1) continue;   // (no term: no sin / cos to evaluate)
                const double d = (P.theta[s] - P.theta[r]) * kPi / 180;
                if (s == i + 1) {
                    Rt = Rt - 2 * (-P.y(s, r).real()) * P.V[s] * P.V[r] * (-std::sin(d));
                    Rv = Rv + 2 * (-P.y(s, r).real()) * (P.V[s] - P.V[r] * std::cos(d));
                }
                if (r == i + 1) {
                    Rt = Rt - 2 * (-P.y(s, r).real()) * P.V[s] * P.V[r] * std::sin(d);
                    Rv = Rv + 2 * (-P.y(s, r).real()) * (P.V[r] - P.V[s] * std::cos(d));
                }
            }
            Fx[i] = (double)Rt;
            Fx[m1 + i] = (double)Rv;
        }
        // J = [H N; K L] (form_J.cpp), stored transposed for lambda = -inv(J^T) Fx
        std::vector<double> Jt((size_t)nf * nf, 0.0);
        auto put = [&](int row, int col, double v) { Jt[(size_t)col + (size_t)row * nf] = v; };
        for (int a = 1; a < n; ++a) {
            long double Rs = 0, Rc = 0;   // sum over m != a of V_m (G sin - B cos), V_m (G cos + B sin)
            // (a zero admittance contributes +-0 to these sums and +-0 entries to J: both
            // skipped -- J starts zero, and a signed zero leaves a nonzero sum unchanged;
            // Y of a radial feeder has a few nonzeros per row, so this is O(L), not O(L^2))
            for (int m = 0; m < n; ++m) {
                const cplx yam = P.y(a, m);
                if (m == a || (yam.real() == 0 && yam.imag() == 0)) continue;
                const double d = (P.theta[a] - P.theta[m]) * kPi / 180;
                Rs = Rs + P.V[m] * (yam.real() * std::sin(d) - yam.imag() * std::cos(d));
                Rc = Rc + P.V[m] * (yam.real() * std::cos(d) + yam.imag() * std::sin(d));
            }
            for (int b = 1; b < n; ++b) {
                const cplx yab = P.y(a, b);
                if (a != b && yab.real() == 0 && yab.imag() == 0) continue;
                if (a != b) {
                    const double d = (P.theta[a] - P.theta[b]) * kPi / 180;
                    const double sn = yab.real() * std::sin(d) - yab.imag() * std::cos(d);
                    const double cs = yab.real() * std::cos(d) + yab.imag() * std::sin(d);
                    put(a - 1, b - 1, P.V[a] * P.V[b] * sn);
                    put(a - 1, m1 + b - 1, P.V[a] * cs);
                    put(m1 + a - 1, b - 1, -P.V[a] * P.V[b] * cs);
                    put(m1 + a - 1, m1 + b - 1, P.V[a] * sn);
                } else {
                    put(a - 1, b - 1, (double)(-P.V[a] * Rs));
                    put(a - 1, m1 + b - 1, (double)(Rc + 2 * P.V[a] * yab.real()));
                    put(m1 + a - 1, b - 1, (double)(P.V[a] * Rc));
                    put(m1 + a - 1, m1 + b - 1, (double)(-2 * P.V[a] * yab.imag() + Rs));
                }
            }
        }
        std::vector<double> lam(Fx);
        if (!lu_solve(Jt, nf, lam)) {
            *err = "singular Jacobian";
            return FPF_ERR_TOPOLOGY;
        }
        for (double &v : lam) v = -v;
        // g_vq = -gu^T lambda, gu = [0; Gqq], Gqq(ia, ja) = -1 where V-list bus ia+1 is load ja
        n_loads[x] = std::min(lload[x], ld);
        double gx_min = INFINITY, gx_max = 0.0;
        for (int j = 0; j < lload[x] && j < ld; ++j) {
            double acc = 0;
            for (int ia = 0; ia < L; ++ia)
                if (P.node[ia + 1] == loads[x][j]) acc += lam[L + ia];
            g[(size_t)x * ld + j] = acc;
            load_nodes[(size_t)x * ld + j] = loads[x][j];
            gx_min = std::min(gx_min, std::fabs(acc));
            gx_max = std::max(gx_max, std::fabs(acc));
        }
        gmin = std::min(gmin, gx_min);
        gmax = std::max(gmax, gx_max);
    }
    if (stats) {
        stats[0] = gmin;
        stats[1] = gmax;
        stats[2] = gmin;                          // gabs_min (:1319) = the smallest |g| of all phases
        stats[3] = beta0 / (bkva / 3) / gmin;     // cvq (:1323)
    }
    return FPF_OK;
}

// The gradient at the DPF result vpolar (nn x 6) of table t.
int gradient(const Table &t, int ncols, const double *z, int z_rows, const double *vpolar, int nn, double bkva,
             double bkv, double beta0, int ld, double *g, double *load_nodes, int *n_loads, double *stats,
             std::string *err) {
    GradPlan plan;
    const int rc = build_plan(t, ncols, z, z_rows, vpolar, nn, bkva, bkv, plan, err);
    if (rc != FPF_OK) return rc;
    return numeric(plan, bkva, beta0, ld, g, load_nodes, n_loads, stats, err);
}

}  // namespace

double fpf_feeder_bkva(const fpf_feeder *f);   // fpf_api.cpp
double fpf_feeder_bkv(const fpf_feeder *f);

extern "C" int fpf_vvc_gradient(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *z,
                                int z_rows, int z_cols, double beta0, int ld, double *g, double *load_nodes,
                                int *n_loads, double *stats) {
    (void)z_cols;
    if (!feeder || !ctrl_dl || !z || !g || !load_nodes || !n_loads || ld < 1 || ncols < 12) return FPF_ERR_ARG;
    fpf_feeder_info in;
    if (fpf_feeder_get_info(feeder, &in) != FPF_OK || in.nl != nl) return FPF_ERR_ARG;
    const int nn = in.nn;
    // the base DPF of this control on the device (VoltVarCtrl.cpp:1141)
    std::vector<double> vpolar((size_t)6 * nn), pqb((size_t)6 * nn), pql((size_t)6 * nn);
    int iters = 0;
    signed char status = 0;
    double loss = 0, vmin = 0, vmax = 0;
    fpf_outputs o;
    std::memset(&o, 0, sizeof(o));
    o.vpolar = vpolar.data();
    o.iters = &iters;
    o.status = &status;
    o.loss = &loss;
    o.vmin = &vmin;
    o.vmax = &vmax;
    static const bool trace = getenv("FPF_VVC_TRACE") && atoi(getenv("FPF_VVC_TRACE")) != 0;   // (diagnostics)
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = fpf_solve_batch(feeder, 1, ctrl_dl + (size_t)6 * nl, &o, nullptr);
    if (rc < 0) return rc;
    if (status != FPF_CONVERGED) return FPF_ERR_UNSUPPORTED;   // the reference throws (DPF_return7.cpp:242)
    const auto t1 = std::chrono::steady_clock::now();
    std::string err;
    double st[4] = {0, 0, 0, 0};
    const int gr = gradient(Table{ctrl_dl, nl}, ncols, z, z_rows, vpolar.data(), nn, fpf_feeder_bkva(feeder),
                            fpf_feeder_bkv(feeder), beta0, ld, g, load_nodes, n_loads, st, &err);
    if (trace)
        fprintf(stderr, "vvc_gradient: base solve %.1f us, host gradient %.1f us\n",
                std::chrono::duration<double, std::micro>(t1 - t0).count(),
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count());
    if (gr != FPF_OK) return gr;
    if (stats) {
        stats[0] = st[0];
        stats[1] = st[1];
        stats[2] = st[2];
        stats[3] = st[3];
        stats[4] = loss;   // Ploss_orig (:1152-1161)
        stats[5] = vmin;   // Vmin_orig / Vmax_orig (:1201-1207)
        stats[6] = vmax;
        stats[7] = iters;
    }
    return FPF_OK;
}

extern "C" int fpf_vvc_gradient_at(const double *ctrl_dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
                                   const double *vpolar, int nn, double bkva, double bkv, double beta0, int ld,
                                   double *g, double *load_nodes, int *n_loads, double *stats) {
    (void)z_cols;
    if (!ctrl_dl || !z || !vpolar || !g || !load_nodes || !n_loads || ld < 1 || ncols < 12 || nn < 2 ||
        !(bkva > 0) || !(bkv > 0))
        return FPF_ERR_ARG;
    std::string err;
    double st[4] = {0, 0, 0, 0};
    const int gr = gradient(Table{ctrl_dl, nl}, ncols, z, z_rows, vpolar, nn, bkva, bkv, beta0, ld, g, load_nodes,
                            n_loads, st, &err);
    if (gr != FPF_OK) return gr;
    if (stats)
        for (int i = 0; i < 4; ++i) stats[i] = st[i];
    return FPF_OK;
}

// the host-synchronous round's first batch of step sizes: the stop of the config-1
// feeders' rounds falls at m = 0 (123-bus), 23 (Dl_new) and 28 (demo), and the
// demo's candidates up to 31 converge in 5 sweeps where its last ones take 14-20
// (one batch of all 101: 41 us of kernel, profiles/r06s2_vvc)
constexpr int VVC_LAZY_FIRST = 32;

extern "C" int fpf_vvc_round(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *z, int z_rows,
                             int z_cols, double beta0, double alpha, int m_max, int ld, double *g, double *load_nodes,
                             int *n_loads, double *loss_fwd, double *loss_rev, double *dl_out, double *res) {
    if (!loss_fwd || !dl_out || m_max < 1) return FPF_ERR_ARG;
    double st[8];
    int rc = fpf_vvc_gradient(feeder, ctrl_dl, nl, ncols, z, z_rows, z_cols, beta0, ld, g, load_nodes, n_loads, st);
    if (rc != FPF_OK) return rc;
    const double ploss_orig = st[4];
    std::memcpy(dl_out, ctrl_dl, sizeof(double) * (size_t)nl * ncols);
    const double bkva = fpf_feeder_bkva(feeder);
    int stop[2] = {-1, -1}, reversed = 0, sent = 0, nonconv = 0;
    double after = 0;
    for (int pass = 0; pass < 2; ++pass) {
        if (pass == 1 && !reversed) break;
        // c0 (:1323) and the reversed start -beta0/(bkva/3)/gabs_min (:1546)
        const double c0 = pass == 0 ? st[3] : -beta0 / (bkva / 3) / st[2];
        double *lossv = pass == 0 ? loss_fwd : loss_rev;
        std::vector<double> tmp;
        if (!lossv) {
            tmp.assign((size_t)m_max + 1, 0.0);
            lossv = tmp.data();
        }
        fpf_line_search ls;
        std::memset(&ls, 0, sizeof(ls));
        ls.loss = lossv;
        // the first VVC_LAZY_FIRST step sizes as one batch, the rest only if the
        // stop rule has not fired among them (fpf_vvc.cpp: vvc_line_search)
        static const bool trace = getenv("FPF_VVC_TRACE") && atoi(getenv("FPF_VVC_TRACE")) != 0;   // (diagnostics)
        const auto t0 = std::chrono::steady_clock::now();
        rc = fpf::vvc_line_search(feeder, ctrl_dl, nl, ncols, g, load_nodes, n_loads, ld, c0, alpha, m_max,
                                  ploss_orig, &ls, VVC_LAZY_FIRST);
        if (rc < 0) return rc;
        if (trace)
            fprintf(stderr, "vvc_round: search pass %d %.1f us (stop %d)\n", pass,
                    std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count(), ls.stop);
        // the reference solves candidates 0 .. stop + 1 (two per step) and throws
        // at the first that does not converge
        const int last = ls.stop >= 0 ? ls.stop + 1 : m_max;
        if (ls.first_nonconv >= 0 && ls.first_nonconv <= last) nonconv = 1;
        stop[pass] = ls.stop;
        if (pass == 0) reversed = ls.reverse;
        if (ls.stop >= 0) {
            after = lossv[ls.stop];
            // Dl = Dl_osize (:1486): the kept candidate's Q set-points, c_stop = c0 alpha^stop
            double c = c0;
            for (int m = 0; m < ls.stop; ++m) c = alpha * c;
            for (int x = 0; x < 3; ++x)
                for (int i = 0; i < n_loads[x]; ++i) {
                    const double gup = g[(size_t)x * ld + i] * (bkva / 3) * c;
                    for (int r = 0; r < nl; ++r)
                        if (ctrl_dl[r + 2 * (size_t)nl] == load_nodes[(size_t)x * ld + i])
                            dl_out[r + (size_t)(7 + 2 * x) * nl] = ctrl_dl[r + (size_t)(7 + 2 * x) * nl] - gup;
                }
            if (lossv[ls.stop] < ploss_orig) sent = 1;   // :1495
        } else if (m_max > 0) {
            after = lossv[m_max - 1];
        }
    }
    if (res) {
        const double v[13] = {ploss_orig, st[5], st[6], st[3], (double)stop[0], (double)stop[1], (double)reversed,
                              (double)sent, after, st[0], st[1], st[2], (double)nonconv};
        std::memcpy(res, v, sizeof(v));
    }
    return nonconv ? 1 : 0;
}

// ---------------------------------------------------------------------------
// The batched gradient (VoltVarCtrl.cpp:1141-1325 for B scenarios of one control
// table): base solves, V lists, Fx, J^T, the LU solves (fpf_vvc_gradb.hip: partial
// pivoting, the host lu_solve's steps) and g all on the device;
// the plan (load lists, branch lists, Y, V_abc_list rows, renamed branch ends)
// on the host once per batch, from the first converged scenario.

namespace {
// the cached scratch slots of the batch paths (fpf::feeder_buf): reused call after
// call, so a repeated call allocates nothing and uploads its plan in one copy per
// phase -- the per-array hipMalloc / hipMemcpy / hipFree of the first version cost
// more than the whole device work on the small feeders (profiles/r06s2_vvcb)
enum : int {
    SB_PQ = 0,      // the batch's loads [6][Nl][B] (fpf_vvc_round_batch reads them again)
    SB_VP,          // Vpolar of the base solves
    SB_RES,         // iters | status | loss | vmin | vmax of the base solves
    SB_FLAGS,       // gstatus | singular flags of the three phases
    SB_G,           // g [B][3][ld]
    SB_PLAN0,       // + x: phase x's plan arrays (device)
    SB_A0 = SB_PLAN0 + 3,   // + x: phase x's J^T chunk
    SB_RHS0 = SB_A0 + 3,    // + x: its right-hand sides
    SB_RB_G = SB_RHS0 + 3,  // fpf_vvc_round_batch: g, the Q-update triples, the pass lists
    SB_RB_TRI,
    SB_RB_TODO,
    SB_RB_CAND,
    SB_RB_OUT,      // candidates' loss | status
    SB_HOST_PLAN0 = 0,      // pinned host slots: + x, phase x's plan arrays
    SB_HOST_RES = 3,        // the base solves' scalars, the flags
};
constexpr size_t al256(size_t n) { return (n + 255) & ~(size_t)255; }
}  // namespace

extern "C" int fpf_vvc_gradient_batch(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *z,
                                      int z_rows, int z_cols, int n_scen, const double *pq, double beta0, int ld,
                                      double *g, double *load_nodes, int *n_loads, double *stats,
                                      signed char *gstatus) {
    (void)z_cols;
    if (!feeder || !ctrl_dl || !z || n_scen < 0 || (n_scen > 0 && (!pq || !g || !stats || !gstatus)) || !load_nodes ||
        !n_loads || ld < 1 || ncols < 12)
        return FPF_ERR_ARG;
    fpf_feeder_info in;
    if (fpf_feeder_get_info(feeder, &in) != FPF_OK || in.nl != nl)
        return fpf::feeder_fail(feeder, FPF_ERR_ARG, "fpf_vvc_gradient_batch: ctrl_dl rows differ from the feeder's");
    if (n_scen == 0) return 0;
    const int B = n_scen, nn = in.nn;
    const size_t b = (size_t)B;
    // every scenario must give the (int) load tests of ctrl_dl (VoltVarCtrl.cpp:354-398):
    // the load lists, and with them node_f, are the plan's
    for (int x = 0; x < 3; ++x)
        for (int i = 0; i < nl; ++i) {
            const bool c = (int)ctrl_dl[(size_t)(6 + 2 * x) * nl + i] != 0;
            const double *row = pq + ((size_t)(2 * x) * nl + i) * b;
            for (int s = 0; s < B; ++s)
                if (((int)row[s] != 0) != c)
                    return fpf::feeder_fail(feeder, FPF_ERR_ARG,
                                            "fpf_vvc_gradient_batch: scenario " + std::to_string(s) + ", row " +
                                                std::to_string(i) + ", phase " + std::to_string(x) +
                                                ": its (int) load test differs from ctrl_dl's (VoltVarCtrl.cpp:354-398)");
        }
    const double bkva = fpf_feeder_bkva(feeder), bkv = fpf_feeder_bkv(feeder);
    hipStream_t st = nullptr;
#define GCHK(expr)                                                                                      \
    do {                                                                                                \
        const hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                           \
            return fpf::feeder_fail(feeder, FPF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
#define BUF(var, slot, bytes, host)                                         \
    void *var = fpf::feeder_buf(feeder, (slot), (bytes), (host));           \
    if (!var) return FPF_ERR_HIP
    // ---- the base solves (VoltVarCtrl.cpp:1141), scenario fastest
    // results region: iters | status | loss | vmin | vmax (one copy back)
    const size_t o_it = 0, o_st = al256(4 * b), o_loss = o_st + al256(b), o_vmin = o_loss + al256(8 * b),
                 o_vmax = o_vmin + al256(8 * b), res_bytes = o_vmax + al256(8 * b);
    // flags region: gstatus | singular of phase 0 | 1 | 2
    const size_t o_sing = al256(b), flags_bytes = o_sing + 3 * al256(b);
    BUF(d_pq, SB_PQ, sizeof(double) * 6 * nl * b, false);
    BUF(d_vp, SB_VP, sizeof(double) * 6 * nn * b, false);
    BUF(d_res, SB_RES, res_bytes, false);
    BUF(d_fl, SB_FLAGS, flags_bytes, false);
    BUF(h_res, SB_HOST_RES, std::max(res_bytes, flags_bytes), true);
    char *const dr = (char *)d_res, *const hr = (char *)h_res, *const dfl = (char *)d_fl;
    int8_t *const d_gst = (int8_t *)dfl;
    GCHK(hipMemcpy(d_pq, pq, sizeof(double) * 6 * nl * b, hipMemcpyHostToDevice));
    fpf_outputs o;
    std::memset(&o, 0, sizeof(o));
    o.vpolar = (double *)d_vp;
    o.iters = (int *)(dr + o_it);
    o.status = (signed char *)(dr + o_st);
    o.loss = (double *)(dr + o_loss);
    o.vmin = (double *)(dr + o_vmin);
    o.vmax = (double *)(dr + o_vmax);
    int rc = fpf::solve_batch_device_ex(feeder, B, (const double *)d_pq, &o, nullptr, (void *)st, nullptr, nullptr,
                                        FPF_LAYOUT_SCEN_FASTEST);
    if (rc < 0) return rc;
    GCHK(hipMemcpy(hr, dr, res_bytes, hipMemcpyDeviceToHost));
    const int8_t *const h_st = (const int8_t *)(hr + o_st);
    const int32_t *const h_it = (const int32_t *)(hr + o_it);
    const double *const h_loss = (const double *)(hr + o_loss), *const h_vmin = (const double *)(hr + o_vmin),
                        *const h_vmax = (const double *)(hr + o_vmax);
    rc = fpf::take_exchange_fault(feeder);   // (the copy above synchronised the device)
    if (rc) return rc;
    int s0 = -1;
    for (int s = 0; s < B && s0 < 0; ++s)
        if (h_st[s] == FPF_CONVERGED) s0 = s;
    std::vector<int8_t> h_gst(b);
    for (int s = 0; s < B; ++s) h_gst[s] = h_st[s] == FPF_CONVERGED ? fpf::FPF_GRAD_OK : fpf::FPF_GRAD_NONCONV;
    for (int s = 0; s < B; ++s) {
        stats[(size_t)s * 8 + 4] = h_loss[s];   // Ploss_orig (:1152-1161)
        stats[(size_t)s * 8 + 5] = h_vmin[s];   // Vmin_orig / Vmax_orig (:1201-1207)
        stats[(size_t)s * 8 + 6] = h_vmax[s];
        stats[(size_t)s * 8 + 7] = h_it[s];
    }
    std::memset(g, 0, sizeof(double) * b * 3 * ld);
    if (s0 < 0) {
        for (int s = 0; s < B; ++s) gstatus[s] = h_gst[s];
        return B;
    }
    // ---- the plan, from the first converged scenario's Vpolar (nn x 6 column-major)
    std::vector<double> vp0((size_t)6 * nn);
    GCHK(hipMemcpy2D(vp0.data(), sizeof(double), (const double *)d_vp + s0, sizeof(double) * b, sizeof(double),
                     (size_t)6 * nn, hipMemcpyDeviceToHost));
    GradPlan plan;
    std::string err;
    rc = build_plan(Table{ctrl_dl, nl}, ncols, z, z_rows, vp0.data(), nn, bkva, bkv, plan, &err);
    if (rc != FPF_OK) return fpf::feeder_fail(feeder, rc, "fpf_vvc_gradient_batch: " + err);
    for (int x = 0; x < 3; ++x)   // the device LU keeps two rows of the matrix in LDS
        if (!fpf::gradb_lu_fits(2 * plan.ph[x].lnum))
            return fpf::feeder_fail(feeder, FPF_ERR_UNSUPPORTED,
                                    "fpf_vvc_gradient_batch: phase " + std::to_string(x) + " has " +
                                        std::to_string(plan.ph[x].lnum) +
                                        " load nodes; the device LU holds at most 3200 (fpf_vvc_gradient runs it)");
    GCHK(hipMemcpy(d_gst, h_gst.data(), b, hipMemcpyHostToDevice));
    GCHK(hipMemset(dfl + o_sing, 0, 3 * al256(b)));
    BUF(d_g, SB_G, sizeof(double) * b * 3 * ld, false);
    GCHK(hipMemset(d_g, 0, sizeof(double) * b * 3 * ld));
    // the three phases' set-up / LU / g on three streams: independent matrices (one
    // workgroup each), so their launches overlap; their buffers live until the end.
    // The streams are the device's, created once (creating three per call cost
    // more than the overlap saves on small feeders)
    struct {
        hipStream_t s[3];
    } ps;
    {
        static std::mutex mu;
        static std::map<int, std::array<hipStream_t, 3>> cache;
        int dev = 0;
        GCHK(hipGetDevice(&dev));
        std::lock_guard<std::mutex> lk(mu);
        auto it = cache.find(dev);
        if (it == cache.end()) {
            std::array<hipStream_t, 3> a{};
            for (int x = 0; x < 3; ++x) GCHK(hipStreamCreateWithFlags(&a[x], hipStreamNonBlocking));
            it = cache.emplace(dev, a).first;
        }
        for (int x = 0; x < 3; ++x) ps.s[x] = it->second[x];
    }
    for (int x = 0; x < 3; ++x) {
        const PhaseNet &P = plan.ph[x];
        const int L = P.lnum, n = L + 1, m1 = n - 1, nf = 2 * m1;
        // the plan's arrays for the device
        std::vector<int8_t> vmask((size_t)std::max(P.scan_end, 1), 0);
        for (int j = 0; j < n; ++j)
            if (P.vrow[j] >= 0) vmask[P.vrow[j]] = 1;
        // (a branch end rename_brn did not find keeps its bus number, which can lie
        // outside the V list: the reference would index past its vectors; refused here)
        for (int j = 0; j < L; ++j)
            if (P.s[j] < 0 || P.s[j] >= n || P.r[j] < 0 || P.r[j] >= n) return FPF_ERR_TOPOLOGY;
        std::vector<double> yre_sr(L);
        for (int j = 0; j < L; ++j) yre_sr[j] = P.y(P.s[j], P.r[j]).real();
        std::vector<int32_t> inc_ptr(1, 0), inc_br;
        std::vector<int8_t> inc_role;
        for (int i = 0; i < m1; ++i) {
            for (int j = 0; j < L; ++j) {
                if (P.s[j] == i + 1) { inc_br.push_back(j); inc_role.push_back(0); }
                if (P.r[j] == i + 1) { inc_br.push_back(j); inc_role.push_back(1); }
            }
            inc_ptr.push_back((int32_t)inc_br.size());
        }
        std::vector<int32_t> y_ptr(1, 0), y_col;
        std::vector<double> y_re, y_im, yd_re(n), yd_im(n);
        for (int a = 0; a < n; ++a) {
            for (int m = 0; m < n; ++m) {
                const cplx y = P.y(a, m);
                if (m == a || (y.real() == 0 && y.imag() == 0)) continue;
                y_col.push_back(m);
                y_re.push_back(y.real());
                y_im.push_back(y.imag());
            }
            y_ptr.push_back((int32_t)y_col.size());
            yd_re[a] = P.y(a, a).real();
            yd_im[a] = P.y(a, a).imag();
        }
        const int nld = std::min(plan.lload[x], ld);
        n_loads[x] = nld;
        std::vector<int32_t> ld_ptr(1, 0), ld_ia;
        for (int j = 0; j < nld; ++j) {
            load_nodes[(size_t)x * ld + j] = plan.loads[x][j];
            for (int ia = 0; ia < L; ++ia)
                if (P.node[ia + 1] == plan.loads[x][j]) ld_ia.push_back(ia);
            ld_ptr.push_back((int32_t)ld_ia.size());
        }
        // the sixteen arrays packed into the phase's pinned slot, one copy up
        struct Arr {
            const void *p;
            size_t bytes;
            size_t off;
        };
        Arr arrs[16] = {{P.vrow.data(), 4 * P.vrow.size(), 0},  {vmask.data(), vmask.size(), 0},
                        {P.s.data(), 4 * P.s.size(), 0},        {P.r.data(), 4 * P.r.size(), 0},
                        {yre_sr.data(), 8 * yre_sr.size(), 0},  {inc_ptr.data(), 4 * inc_ptr.size(), 0},
                        {inc_br.data(), 4 * inc_br.size(), 0},  {inc_role.data(), inc_role.size(), 0},
                        {y_ptr.data(), 4 * y_ptr.size(), 0},    {y_col.data(), 4 * y_col.size(), 0},
                        {y_re.data(), 8 * y_re.size(), 0},      {y_im.data(), 8 * y_im.size(), 0},
                        {yd_re.data(), 8 * yd_re.size(), 0},    {yd_im.data(), 8 * yd_im.size(), 0},
                        {ld_ptr.data(), 4 * ld_ptr.size(), 0},  {ld_ia.data(), 4 * ld_ia.size(), 0}};
        static_assert(sizeof(P.vrow[0]) == 4 && sizeof(P.s[0]) == 4 && sizeof(P.r[0]) == 4, "int32 plan arrays");
        size_t tot = 0;
        for (Arr &a : arrs) {
            a.off = tot;
            tot += al256(std::max<size_t>(a.bytes, 1));
        }
        BUF(h_plan, SB_HOST_PLAN0 + x, tot, true);
        BUF(d_plan, SB_PLAN0 + x, tot, false);
        for (const Arr &a : arrs)
            if (a.bytes) std::memcpy((char *)h_plan + a.off, a.p, a.bytes);
        const hipStream_t sx = ps.s[x];
        GCHK(hipMemcpyAsync(d_plan, h_plan, tot, hipMemcpyHostToDevice, sx));
        auto dp = [&](int i) { return (void *)((char *)d_plan + arrs[i].off); };
        fpf::GradPhaseDev D;
        D.x = x;
        D.L = L;
        D.n = n;
        D.nn = nn;
        D.scan_end = P.scan_end;
        D.n_loads = nld;
        D.vrow = (int32_t *)dp(0);
        D.vmask = (int8_t *)dp(1);
        D.bs = (int32_t *)dp(2);
        D.br = (int32_t *)dp(3);
        D.yre_sr = (double *)dp(4);
        D.inc_ptr = (int32_t *)dp(5);
        D.inc_br = (int32_t *)dp(6);
        D.inc_role = (int8_t *)dp(7);
        D.y_ptr = (int32_t *)dp(8);
        D.y_col = (int32_t *)dp(9);
        D.y_re = (double *)dp(10);
        D.y_im = (double *)dp(11);
        D.ydiag_re = (double *)dp(12);
        D.ydiag_im = (double *)dp(13);
        D.ld_ptr = (int32_t *)dp(14);
        D.ld_ia = (int32_t *)dp(15);
        // the dense J^T of a chunk of scenarios at a time (nf^2 doubles each, within ~2 GB)
        const size_t per = (size_t)nf * nf * sizeof(double);
        const int chunk = (int)std::max<size_t>(1, std::min<size_t>(b, ((size_t)2 << 30) / per));
        BUF(d_A, SB_A0 + x, per * chunk, false);
        BUF(d_rhs, SB_RHS0 + x, sizeof(double) * nf * chunk, false);
        int8_t *const d_sing = (int8_t *)(dfl + o_sing + x * al256(b));
        for (int c0 = 0; c0 < B; c0 += chunk) {
            const int nb = std::min(chunk, B - c0);
            double *A = (double *)d_A, *rhs = (double *)d_rhs;
            GCHK(fpf::launch_gradb_setup(D, B, c0, nb, (const double *)d_vp, A, rhs, d_gst, sx));
            // lambda = -inv(J^T) Fx: one LU with partial pivoting and one solve per matrix
            GCHK(fpf::launch_gradb_lu(nf, nb, A, rhs, d_sing + c0, sx));
            GCHK(fpf::launch_gradb_g(D, c0, nb, rhs, ld, (double *)d_g, sx));
        }
    }
    for (int x = 0; x < 3; ++x) GCHK(hipStreamSynchronize(ps.s[x]));
    // per-scenario results: the device's pattern flags and the singular matrices
    // merged with the host's, one copy back
    GCHK(hipMemcpy(hr, dfl, flags_bytes, hipMemcpyDeviceToHost));
    const int8_t *const d_flags = (const int8_t *)hr;
    for (int x = 0; x < 3; ++x) {
        const int8_t *sing = (const int8_t *)(hr + o_sing + x * al256(b));
        for (int s = 0; s < B; ++s)
            if (sing[s] != 0 && h_gst[s] == fpf::FPF_GRAD_OK) h_gst[s] = fpf::FPF_GRAD_SINGULAR;
    }
    GCHK(hipMemcpy(g, d_g, sizeof(double) * b * 3 * ld, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int s = 0; s < B; ++s) {
        int8_t gs = h_gst[s];
        if (gs == fpf::FPF_GRAD_OK && d_flags[s] != fpf::FPF_GRAD_OK) gs = d_flags[s];
        gstatus[s] = gs;
        double *st8 = stats + (size_t)s * 8;
        if (gs != fpf::FPF_GRAD_OK) {
            ++bad;
            std::memset(g + (size_t)s * 3 * ld, 0, sizeof(double) * 3 * ld);
            st8[0] = st8[1] = st8[2] = st8[3] = 0.0;
            continue;
        }
        // gmin / gmax / gabs_min / c0 (:1319-1323) as the host path forms them
        double gmin = INFINITY, gmax = -INFINITY;
        for (int x = 0; x < 3; ++x) {
            double gx_min = INFINITY, gx_max = 0.0;
            for (int j = 0; j < n_loads[x]; ++j) {
                const double a = g[((size_t)s * 3 + x) * ld + j];
                gx_min = std::min(gx_min, std::fabs(a));
                gx_max = std::max(gx_max, std::fabs(a));
            }
            gmin = std::min(gmin, gx_min);
            gmax = std::max(gmax, gx_max);
        }
        st8[0] = gmin;
        st8[1] = gmax;
        st8[2] = gmin;
        st8[3] = beta0 / (bkva / 3) / gmin;
    }
    return bad;
#undef GCHK
#undef BUF
}

// ---------------------------------------------------------------------------
// A whole VVC round per load scenario (VoltVarCtrl.cpp:1141-1762 for B scenarios
// of one control table): the batched gradient, then every scenario's step sizes
// as device batches (the first VVC_LAZY_FIRST of every search as one, the rest of
// the searches without a stop as a second), the reference's stop rule per
// scenario, and the same for the scenarios whose search reverses.

namespace {
// the reference's stop rule over one search (VoltVarCtrl.cpp:1330-1540, as
// fpf_vvc_line_search): keep c_m while c_{m+1} lowers the loss; the direction flag
// drops when a kept loss exceeds Ploss_orig; the first candidate that does not
// converge (the reference throws there)
void stop_rule(const double *loss, const signed char *status, int m_max, double ploss_orig, int *stop, int *reverse,
               int *first_nonconv) {
    *first_nonconv = -1;
    for (int m = 0; m <= m_max; ++m)
        if (status[m] != FPF_CONVERGED) {
            *first_nonconv = m;
            break;
        }
    *stop = -1;
    *reverse = 0;
    for (int m = 0; m < m_max; ++m) {
        if (loss[m + 1] > loss[m]) {
            *stop = m;
            break;
        }
        if (loss[m] > ploss_orig) *reverse = 1;
    }
}
}  // namespace

extern "C" int fpf_vvc_round_batch(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *z,
                                   int z_rows, int z_cols, int n_scen, const double *pq, double beta0, double alpha,
                                   int m_max, int ld, double *g, double *load_nodes, int *n_loads, double *loss_fwd,
                                   double *loss_rev, double *pq_out, double *res, signed char *rstatus) {
    if (!feeder || !ctrl_dl || n_scen < 0 || m_max < 1 || (n_scen > 0 && (!pq || !g || !pq_out || !res || !rstatus)))
        return fpf::feeder_fail(feeder, FPF_ERR_ARG, "fpf_vvc_round_batch: bad arguments");
    if (n_scen == 0) return 0;
    const int B = n_scen, M = m_max + 1;
    const size_t b = (size_t)B, nlz = (size_t)nl;
    std::vector<double> stats(b * 8);
    int rc = fpf_vvc_gradient_batch(feeder, ctrl_dl, nl, ncols, z, z_rows, z_cols, B, pq, beta0, ld, g, load_nodes,
                                    n_loads, stats.data(), rstatus);
    if (rc < 0) return rc;
    const double bkva = fpf_feeder_bkva(feeder);
    std::memcpy(pq_out, pq, sizeof(double) * 6 * nlz * b);
    // the rows each load's Q update touches (rbus == load node, :1334-1372)
    std::vector<std::vector<int>> rows[3];
    for (int x = 0; x < 3; ++x) {
        rows[x].resize(n_loads[x]);
        for (int i = 0; i < n_loads[x]; ++i)
            for (int r = 0; r < nl; ++r)
                if (ctrl_dl[r + 2 * nlz] == load_nodes[(size_t)x * ld + i]) rows[x][i].push_back(r);
    }
    struct Sc {
        int stop[2] = {-1, -1}, reversed = 0, sent = 0, nonconv = 0;
        double after = 0.0;
    };
    std::vector<Sc> sc(b);
    std::vector<int> todo;
    for (int s = 0; s < B; ++s)
        if (rstatus[s] == 0) todo.push_back(s);
#define RCHK(expr)                                                                                      \
    do {                                                                                                \
        const hipError_t e_ = (expr);                                                                   \
        if (e_ != hipSuccess)                                                                           \
            return fpf::feeder_fail(feeder, FPF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
    // the candidate batches are formed on the device (launch_vvc_candidates): the
    // scenarios' loads, g and the (phase, load, row) triples of the Q updates go
    // up once; per pass only the scenario list and the first step sizes
    const double scale = bkva / 3;
    std::vector<int32_t> tri;
    for (int x = 0; x < 3; ++x)
        for (int i = 0; i < n_loads[x]; ++i)
            for (int r : rows[x][i]) tri.insert(tri.end(), {x, i, r});
    const int T = (int)(tri.size() / 3);
    const size_t Bmax = (size_t)todo.size() * M;
    // the cached scratch (fpf::feeder_buf); the loads are still in SB_PQ, where
    // fpf_vvc_gradient_batch put them above
    void *d_pq = nullptr, *d_g = nullptr, *d_tri = nullptr, *d_todo = nullptr, *d_cand = nullptr, *d_out = nullptr;
    const size_t o_cst = al256(sizeof(int32_t) * b), o_stat = al256(sizeof(double) * Bmax);
    if (!todo.empty()) {
        d_pq = fpf::feeder_buf(feeder, SB_PQ, sizeof(double) * 6 * nlz * b);
        d_g = fpf::feeder_buf(feeder, SB_RB_G, sizeof(double) * b * 3 * ld);
        d_tri = fpf::feeder_buf(feeder, SB_RB_TRI, sizeof(int32_t) * std::max<size_t>(tri.size(), 1));
        d_todo = fpf::feeder_buf(feeder, SB_RB_TODO, o_cst + sizeof(double) * b);   // todo | cstart
        d_cand = fpf::feeder_buf(feeder, SB_RB_CAND, sizeof(double) * 6 * nlz * Bmax);
        d_out = fpf::feeder_buf(feeder, SB_RB_OUT, o_stat + Bmax);                  // loss | status
        if (!d_pq || !d_g || !d_tri || !d_todo || !d_cand || !d_out) return FPF_ERR_HIP;
        RCHK(hipMemcpy(d_g, g, sizeof(double) * b * 3 * ld, hipMemcpyHostToDevice));
        if (!tri.empty()) RCHK(hipMemcpy(d_tri, tri.data(), sizeof(int32_t) * tri.size(), hipMemcpyHostToDevice));
    }
    std::vector<char> h_out;
    std::vector<double> lossv;
    std::vector<signed char> statv;
    for (int pass = 0; pass < 2 && !todo.empty(); ++pass) {
        const int K = (int)todo.size();
        // candidate (k, m): scenario todo[k]'s loads with its Q set-points moved by
        // -g (bkva/3) c_m, c_0 = c0 (:1323) or the reversed start
        // -beta0/(bkva/3)/gabs_min (:1546), c_{m+1} = alpha c_m (:1420-1422)
        std::vector<double> cstart(K);
        for (int k = 0; k < K; ++k) {
            const double *st8 = &stats[(size_t)todo[k] * 8];
            cstart[k] = pass == 0 ? st8[3] : -beta0 / (bkva / 3) / st8[2];
        }
        // the step sizes in two stages, as fpf_vvc_round: the first VVC_LAZY_FIRST of
        // every search, then the rest of the searches whose stop rule has not fired
        // (the reference never solves past stop + 1; the large steps are the slow
        // ones).  Unsolved candidates: NaN loss, status "converged" (not looked at)
        lossv.assign((size_t)K * M, NAN);
        statv.assign((size_t)K * M, (signed char)FPF_CONVERGED);
        std::vector<int> ks(K);
        for (int k = 0; k < K; ++k) ks[k] = k;
        std::vector<double> cst = cstart;   // c_{m0} of each search, by the same products
        int m0 = 0;
        while (m0 < M && !ks.empty()) {
            const int m1 = m0 == 0 ? std::min(M, VVC_LAZY_FIRST) : M, Mk = m1 - m0, Ks = (int)ks.size();
            const size_t Bc = (size_t)Ks * Mk;
            // this stage's scenario list and first step sizes, one copy up
            std::vector<char> up(o_cst + sizeof(double) * Ks);
            for (int j = 0; j < Ks; ++j) {
                const int32_t sid = todo[ks[j]];
                std::memcpy(up.data() + sizeof(int32_t) * j, &sid, sizeof(int32_t));
                std::memcpy(up.data() + o_cst + sizeof(double) * j, &cst[ks[j]], sizeof(double));
            }
            RCHK(hipMemcpy(d_todo, up.data(), up.size(), hipMemcpyHostToDevice));
            RCHK(fpf::launch_vvc_candidates((const double *)d_pq, nl, B, (const int32_t *)d_todo, Ks, Mk,
                                            (const int32_t *)d_tri, T, (const double *)d_g, ld, scale, alpha,
                                            (const double *)((char *)d_todo + o_cst), (double *)d_cand, nullptr));
            fpf_outputs out;
            std::memset(&out, 0, sizeof(out));
            out.loss = (double *)d_out;
            out.status = (signed char *)((char *)d_out + o_stat);
            rc = fpf::solve_batch_device_ex(feeder, (int)Bc, (const double *)d_cand, &out, nullptr, nullptr, nullptr,
                                            nullptr, FPF_LAYOUT_SCEN_FASTEST);
            if (rc < 0) return rc;
            // loss | status back in one copy
            h_out.resize(o_stat + Bc);
            RCHK(hipMemcpy(h_out.data(), d_out, o_stat + Bc, hipMemcpyDeviceToHost));
            rc = fpf::take_exchange_fault(feeder);   // (the copy above synchronised the device)
            if (rc) return rc;
            const double *const ls = (const double *)h_out.data();
            const signed char *const ss = (const signed char *)(h_out.data() + o_stat);
            std::vector<int> open;
            for (int j = 0; j < Ks; ++j) {
                const int k = ks[j];
                std::memcpy(&lossv[(size_t)k * M + m0], ls + (size_t)j * Mk, sizeof(double) * Mk);
                std::memcpy(&statv[(size_t)k * M + m0], ss + (size_t)j * Mk, Mk);
                for (int m = 0; m < Mk; ++m) cst[k] = alpha * cst[k];   // c_{m1}
                int stop, reverse, first_nonconv;
                stop_rule(&lossv[(size_t)k * M], &statv[(size_t)k * M], m_max, stats[(size_t)todo[k] * 8 + 4], &stop,
                          &reverse, &first_nonconv);
                if (stop < 0) open.push_back(k);
            }
            ks.swap(open);
            m0 = m1;
        }
        const double *const loss = lossv.data();
        const signed char *const status = statv.data();
        std::vector<int> next;
        for (int k = 0; k < K; ++k) {
            const int s = todo[k];
            Sc &q = sc[s];
            const double *lk = &loss[(size_t)k * M];
            double *lout = pass == 0 ? loss_fwd : loss_rev;
            if (lout) std::memcpy(lout + (size_t)s * M, lk, sizeof(double) * M);
            int stop, reverse, first_nonconv;
            stop_rule(lk, &status[(size_t)k * M], m_max, stats[(size_t)s * 8 + 4], &stop, &reverse, &first_nonconv);
            // the reference solves candidates 0 .. stop + 1 (two per step) and throws
            // at the first that does not converge
            const int last = stop >= 0 ? stop + 1 : m_max;
            if (first_nonconv >= 0 && first_nonconv <= last) q.nonconv = 1;
            q.stop[pass] = stop;
            if (pass == 0) {
                q.reversed = reverse;
                if (reverse) next.push_back(s);
            }
            if (stop >= 0) {
                q.after = lk[stop];
                // Dl = Dl_osize (:1486/:1707): the kept candidate's Q set-points, formed
                // as the device formed them
                double cvq = cstart[k];
                for (int j = 0; j < stop; ++j) cvq = alpha * cvq;
                for (int x = 0; x < 3; ++x) {
                    const size_t fq = (size_t)(1 + 2 * x);
                    for (int i = 0; i < n_loads[x]; ++i) {
                        const double gupdate = g[((size_t)s * 3 + x) * ld + i] * scale * cvq;
                        for (int r : rows[x][i]) pq_out[(fq * nlz + r) * b + s] = pq[(fq * nlz + r) * b + s] - gupdate;
                    }
                }
                if (lk[stop] < stats[(size_t)s * 8 + 4]) q.sent = 1;   // :1495
            } else {
                q.after = lk[m_max - 1];
            }
        }
        todo.swap(next);
    }
#undef RCHK
    int bad = 0;
    for (int s = 0; s < B; ++s) {
        const double *st8 = &stats[(size_t)s * 8];
        const Sc &q = sc[s];
        const double v[13] = {st8[4], st8[5], st8[6], st8[3], (double)q.stop[0], (double)q.stop[1], (double)q.reversed,
                              (double)q.sent, q.after, st8[0], st8[1], st8[2], (double)q.nonconv};
        std::memcpy(res + (size_t)s * 13, v, sizeof(v));
        if (rstatus[s] != 0 || q.nonconv) ++bad;
    }
    return bad;
}
