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

#include <algorithm>
#include <cmath>
#include <complex>
#include <cstring>
#include <string>
#include <vector>

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

// The gradient at the DPF result vpolar (nn x 6) of table t.
int gradient(const Table &t, int ncols, const double *z, int z_rows, const double *vpolar, int nn, double bkva,
             double bkv, double beta0, int ld, double *g, double *load_nodes, int *n_loads, double *stats,
             std::string *err) {
    const int nl = t.nl;
    if (ncols < 12) return FPF_ERR_ARG;
    // ---- Node_f and Load_a/b/c (VoltVarCtrl.cpp:354-398): (int) tests, and the scan
    // stops at the first full counter
    int cnt_nodes = 1;
    int lload[3] = {0, 0, 0};
    for (int i = 0; i < nl; ++i) {
        if ((int)t(i, 0) != 0) ++cnt_nodes;
        for (int x = 0; x < 3; ++x)
            if ((int)t(i, 6 + 2 * x) != 0) ++lload[x];
    }
    std::vector<double> node_f(cnt_nodes, 0.0), loads[3];
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
    PhaseNet ph[3];
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
    double gmin = INFINITY, gmax = -INFINITY;
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
        for (int i = 0, j = 0; i < nn && j < n; ++i) {
            const double mag = vpolar[i + (size_t)(2 * x) * nn];
            if (mag != 0) {
                P.V[j] = mag;
                P.theta[j] = vpolar[i + (size_t)(2 * x + 1) * nn];
                P.node[j] = i < cnt_nodes ? node_f[i] : 0.0;
                ++j;
            }
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
        // Fx = [dF/dtheta; dF/dV] over the n-1 non-reference buses
        const int m1 = n - 1, nf = 2 * m1;
        std::vector<double> Fx(nf, 0.0);
        for (int i = 0; i < m1; ++i) {
            long double Rt = 0, Rv = 0;
            for (int j = 0; j < L; ++j) {
                const int s = P.s[j], r = P.r[j];
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
            for (int m = 0; m < n; ++m) {
                if (m == a) continue;
                const double d = (P.theta[a] - P.theta[m]) * kPi / 180;
                const cplx yam = P.y(a, m);
                Rs = Rs + P.V[m] * (yam.real() * std::sin(d) - yam.imag() * std::cos(d));
                Rc = Rc + P.V[m] * (yam.real() * std::cos(d) + yam.imag() * std::sin(d));
            }
            for (int b = 1; b < n; ++b) {
                const cplx yab = P.y(a, b);
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
    const int rc = fpf_solve_batch(feeder, 1, ctrl_dl + (size_t)6 * nl, &o, nullptr);
    if (rc < 0) return rc;
    if (status != FPF_CONVERGED) return FPF_ERR_UNSUPPORTED;   // the reference throws (DPF_return7.cpp:242)
    std::string err;
    double st[4] = {0, 0, 0, 0};
    const int gr = gradient(Table{ctrl_dl, nl}, ncols, z, z_rows, vpolar.data(), nn, fpf_feeder_bkva(feeder),
                            fpf_feeder_bkv(feeder), beta0, ld, g, load_nodes, n_loads, st, &err);
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
        rc = fpf_vvc_line_search(feeder, ctrl_dl, nl, ncols, g, load_nodes, n_loads, ld, c0, alpha, m_max, ploss_orig,
                                 &ls);
        if (rc < 0) return rc;
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
