/*
 * ref_vvc.c -- TEST INFRASTRUCTURE ONLY (the parity oracle of the VVC round).
 *
 * A scalar C restatement of the Volt-VAR control numerics around the solve:
 *   Node_f / Load_a,b,c          Broker/src/vvc/VoltVarCtrl.cpp:349-398
 *   form_Y_abc                   Broker/src/vvc/form_Yabc.cpp:8-260
 *   per-phase branch lists       VoltVarCtrl.cpp:408-433
 *   V_abc_list                   Broker/src/vvc/V_abc_list.cpp:7-81
 *   rename_brn                   Broker/src/vvc/rename_brn.cpp:7-83
 *   form_Ftheta / form_Fv        form_Ftheta.cpp:8-41, form_Fv.cpp:8-32
 *   form_J                       form_J.cpp:8-127
 *   lambda = -inv(J^T) Fx, Gqq, g_vq = -gu^T lambda, step size
 *                                VoltVarCtrl.cpp:1218-1325
 *   the sequential step-size search and its reversal, S2
 *                                VoltVarCtrl.cpp:1327-1762
 * with the reference's quirks: the (int) casts of the load test, the loop
 * guards that stop at the first full counter (:375, :416, form_Yabc.cpp:66),
 * rename_brn's last-match-wins, and the long double accumulators of the
 * F / J sums (x87 80-bit with gcc on x86-64, as the reference's build).
 * inv() is LAPACK in the reference (dgetrf/dgetri, version unpinned): here an
 * LU with partial pivoting, so lambda agrees to rounding, not bit for bit.
 *
 * Only tests/ load this code.  Parity status: unpinned, like ref_dpf.c.
 */
#include <complex.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "ref_dpf.h"

typedef double complex dc;

#define DL(i, j) dl[(size_t)(i) + (size_t)(j) * (size_t)nl]
static const double PI = 3.14159265358979323846;   /* form_Ftheta.cpp:11 */

typedef struct {
    int lnum;          /* Lnum_x */
    dc *brn;           /* [lnum][5] rows of brnches for this phase (VoltVarCtrl.cpp:408-433) */
    dc *Y;             /* (lnum+1)^2 column-major (form_Yabc.cpp:118-220) */
    double *V, *th, *node;   /* V_abc_list: lnum+1 each */
    int ln;            /* Lna = lnum + 1 */
} phase_t;

static void phase_free(phase_t *p) {
    free(p->brn);
    free(p->Y);
    free(p->V);
    free(p->th);
    free(p->node);
}

/* inverse of the n x n column-major A by LU with partial pivoting (Doolittle,
 * row swaps), then A^-1 = U^-1 L^-1 P column by column */
static int lu_inverse(const double *A, int n, double *Ainv) {
    double *a = (double *)malloc(sizeof(double) * (size_t)n * n);
    int *piv = (int *)malloc(sizeof(int) * (size_t)n);
    int i, j, k, rc = 0;
    memcpy(a, A, sizeof(double) * (size_t)n * n);
#define Aij(r, c) a[(size_t)(r) + (size_t)(c) * (size_t)n]
    for (k = 0; k < n; ++k) {
        int p = k;
        double mx = fabs(Aij(k, k));
        for (i = k + 1; i < n; ++i)
            if (fabs(Aij(i, k)) > mx) { mx = fabs(Aij(i, k)); p = i; }
        piv[k] = p;
        if (mx == 0) { rc = -1; break; }
        if (p != k)
            for (j = 0; j < n; ++j) { double t = Aij(k, j); Aij(k, j) = Aij(p, j); Aij(p, j) = t; }
        for (i = k + 1; i < n; ++i) {
            double l = Aij(i, k) / Aij(k, k);
            Aij(i, k) = l;
            for (j = k + 1; j < n; ++j) Aij(i, j) -= l * Aij(k, j);
        }
    }
    if (rc == 0) {
        double *x = (double *)malloc(sizeof(double) * (size_t)n);
        for (j = 0; j < n; ++j) {
            /* e_j permuted by the row swaps, then forward (unit L) and back (U) */
            for (i = 0; i < n; ++i) x[i] = i == j ? 1.0 : 0.0;
            for (k = 0; k < n; ++k)
                if (piv[k] != k) { double t = x[k]; x[k] = x[piv[k]]; x[piv[k]] = t; }
            for (i = 0; i < n; ++i)
                for (k = 0; k < i; ++k) x[i] -= Aij(i, k) * x[k];
            for (i = n - 1; i >= 0; --i) {
                for (k = i + 1; k < n; ++k) x[i] -= Aij(i, k) * x[k];
                x[i] /= Aij(i, i);
            }
            for (i = 0; i < n; ++i) Ainv[(size_t)i + (size_t)j * n] = x[i];
        }
        free(x);
    }
#undef Aij
    free(a);
    free(piv);
    return rc;
}

int ref_vvc_gradient(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
                     const double *vpolar, int nn, double bkva, double bkv, double beta0, int ld,
                     double *g, double *load_nodes, int *n_loads, double *stats)
{
    int i, j, x, cnt_nodes = 0, lload[3] = {0, 0, 0}, lbr = 0, rc = 0;
    double *node_f, *load[3];
    dc *brnches;
    phase_t ph[3];
    const double Zb = pow(bkv, 2) / bkva * 1000;   /* form_Yabc.cpp:11 */
    (void)z_cols;
    if (ncols < 12) return REF_BAD_INPUT;
    memset(ph, 0, sizeof(ph));
    /* ---- Node_f, Load_a/b/c (VoltVarCtrl.cpp:354-398) */
    for (i = 0; i < nl; ++i) {
        if ((int)DL(i, 0) != 0) cnt_nodes++;
        for (x = 0; x < 3; ++x)
            if ((int)DL(i, 6 + 2 * x) != 0) lload[x]++;
    }
    cnt_nodes++;
    node_f = (double *)calloc((size_t)cnt_nodes, sizeof(double));
    for (x = 0; x < 3; ++x) load[x] = (double *)calloc((size_t)(lload[x] > 0 ? lload[x] : 1), sizeof(double));
    {
        int jn = 1, jl[3] = {0, 0, 0};
        for (i = 0; i < nl && jn < cnt_nodes && jl[0] < lload[0] && jl[1] < lload[1] && jl[2] < lload[2]; ++i) {
            if ((int)DL(i, 2) != 0) node_f[jn++] = DL(i, 2);
            for (x = 0; x < 3; ++x)
                if ((int)DL(i, 6 + 2 * x) != 0) load[x][jl[x]++] = DL(i, 2);
        }
    }
    /* ---- form_Y_abc: branches with the per-phase self impedances (form_Yabc.cpp:13-45) */
    for (i = 0; i < nl; ++i)
        if (DL(i, 0) > 0) lbr++;
    brnches = (dc *)calloc((size_t)(lbr > 0 ? lbr : 1) * 5, sizeof(dc));
    for (i = 0, j = 0; i < nl && j < lbr; ++i) {
        const int code = (int)DL(i, 3), idx = 3 * (code - 1);
        if ((int)DL(i, 0) != 0) {
            if (idx < 0 || idx + 2 >= z_rows) { rc = REF_BAD_INPUT; goto done; }
            brnches[j * 5 + 0] = DL(i, 1);
            brnches[j * 5 + 1] = DL(i, 2);
            for (x = 0; x < 3; ++x) {
                const size_t zi = (size_t)(idx + x) + (size_t)x * (size_t)z_rows;
                const dc zz = z[2 * zi] + I * z[2 * zi + 1];
                if (code == 7) brnches[j * 5 + 2 + x] = zz;
                else brnches[j * 5 + 2 + x] = (DL(i, 4) * zz) / Zb;
            }
            ++j;
        }
    }
    for (x = 0; x < 3; ++x) {
        int c = 0;
        for (i = 0; i < lbr; ++i) if (cabs(brnches[i * 5 + 2 + x]) > 0) c++;
        ph[x].lnum = c;
        ph[x].ln = c + 1;
        ph[x].brn = (dc *)calloc((size_t)(c > 0 ? c : 1) * 5, sizeof(dc));
    }
    /* per-phase rows; the guard stops at the first full list (form_Yabc.cpp:66,
     * VoltVarCtrl.cpp:416) */
    {
        int jj[3] = {0, 0, 0};
        for (i = 0; i < lbr && jj[0] < ph[0].lnum && jj[1] < ph[1].lnum && jj[2] < ph[2].lnum; ++i)
            for (x = 0; x < 3; ++x)
                if (cabs(brnches[i * 5 + 2 + x]) != 0) {
                    memcpy(&ph[x].brn[jj[x] * 5], &brnches[i * 5], 5 * sizeof(dc));
                    jj[x]++;
                }
    }
    for (x = 0; x < 3; ++x) {
        phase_t *P = &ph[x];
        const int L = P->lnum, n = L + 1;
        dc *yy = (dc *)calloc((size_t)(L > 0 ? L : 1), sizeof(dc));
        double *ka = (double *)calloc((size_t)n, sizeof(double));
        int m, q;
        if (L == 0) { free(yy); free(ka); rc = REF_BAD_INPUT; goto done; }
        for (i = 0; i < L; ++i) yy[i] = 1.0 / P->brn[i * 5 + 2 + x];   /* cx_unity / z (form_Yabc.cpp:104-117) */
        ka[0] = creal(P->brn[0]);
        for (i = 0; i < L; ++i) ka[i + 1] = creal(P->brn[i * 5 + 1]);
        P->Y = (dc *)calloc((size_t)n * n, sizeof(dc));
        for (m = 0; m < n; ++m)
            for (q = 0; q < n; ++q) {
                dc *y = &P->Y[(size_t)m + (size_t)q * n];
                if (m == q) {
                    for (i = 0; i < L; ++i)
                        if ((int)creal(P->brn[i * 5]) == (int)ka[m] || (int)creal(P->brn[i * 5 + 1]) == (int)ka[m])
                            *y = *y + yy[i];
                } else {
                    for (i = 0; i < L; ++i)
                        if ((int)creal(P->brn[i * 5]) == (int)ka[m] && (int)creal(P->brn[i * 5 + 1]) == (int)ka[q])
                            *y = *y - yy[i];
                    for (i = 0; i < L; ++i)
                        if ((int)creal(P->brn[i * 5 + 1]) == (int)ka[m] && (int)creal(P->brn[i * 5]) == (int)ka[q])
                            *y = *y - yy[i];
                }
            }
        free(yy);
        free(ka);
        /* ---- V_abc_list (V_abc_list.cpp:12-60): the first L+1 nonzero |V| */
        P->V = (double *)calloc((size_t)n, sizeof(double));
        P->th = (double *)calloc((size_t)n, sizeof(double));
        P->node = (double *)calloc((size_t)n, sizeof(double));
        for (i = 0, j = 0; i < nn && j < n; ++i)
            if (vpolar[i + (size_t)(2 * x) * nn] != 0) {
                P->V[j] = vpolar[i + (size_t)(2 * x) * nn];
                P->th[j] = vpolar[i + (size_t)(2 * x + 1) * nn];
                P->node[j] = i < cnt_nodes ? node_f[i] : 0.0;
                ++j;
            }
        /* ---- rename_brn (rename_brn.cpp:16-35): last match wins */
        for (i = 0; i < L; ++i)
            for (j = 0; j < n; ++j) {
                if (round(creal(ph[x].brn[i * 5])) == round(P->node[j])) P->brn[i * 5] = j;
                else if (round(creal(ph[x].brn[i * 5 + 1])) == round(P->node[j])) P->brn[i * 5 + 1] = j;
            }
    }
    /* ---- gradient per phase */
    {
        double gabs_min = INFINITY, gmin = INFINITY, gmax = -INFINITY;
        for (x = 0; x < 3; ++x) {
            phase_t *P = &ph[x];
            const int Ln = P->ln, Lnm = P->lnum, n = Ln;   /* form_J's Lnm is Lna (VoltVarCtrl.cpp:1238) */
            const int nf = 2 * (Ln - 1);
            double *Fx = (double *)calloc((size_t)nf, sizeof(double));
            double *J = (double *)calloc((size_t)nf * nf, sizeof(double));
            double *Jt = (double *)calloc((size_t)nf * nf, sizeof(double));
            double *Ji = (double *)calloc((size_t)nf * nf, sizeof(double));
            double *lam = (double *)calloc((size_t)nf, sizeof(double));
#define Y(r, c) P->Y[(size_t)(r) + (size_t)(c) * (size_t)n]
            int a, b, m;
            double gx_min = INFINITY, gx_max = 0;
            /* form_Ftheta.cpp:14-40 */
            for (i = 0; i < Ln - 1; ++i) {
                long double R = 0;
                for (j = 0; j < Lnm; ++j) {
                    const int s = (int)creal(P->brn[j * 5]), r = (int)creal(P->brn[j * 5 + 1]);
                    if (s == i + 1) R = R - 2 * (-creal(Y(s, r))) * P->V[s] * P->V[r] * (-sin((P->th[s] - P->th[r]) * PI / 180));
                    if (r == i + 1) R = R - 2 * (-creal(Y(s, r))) * P->V[s] * P->V[r] * sin((P->th[s] - P->th[r]) * PI / 180);
                }
                Fx[i] = (double)R;
            }
            /* form_Fv.cpp:14-31 */
            for (i = 0; i < Ln - 1; ++i) {
                long double R = 0;
                for (j = 0; j < Lnm; ++j) {
                    const int s = (int)creal(P->brn[j * 5]), r = (int)creal(P->brn[j * 5 + 1]);
                    if (s == i + 1) R = R + 2 * (-creal(Y(s, r))) * (P->V[s] - P->V[r] * cos((P->th[s] - P->th[r]) * PI / 180));
                    if (r == i + 1) R = R + 2 * (-creal(Y(s, r))) * (P->V[r] - P->V[s] * cos((P->th[s] - P->th[r]) * PI / 180));
                }
                Fx[Ln - 1 + i] = (double)R;
            }
            /* form_J.cpp: J = [H N; K L], each (Ln-1)^2, i, j = 1..Ln-1, m over every bus */
#define JM(r, c) J[(size_t)(r) + (size_t)(c) * (size_t)nf]
            for (a = 1; a < Ln; ++a) {
                long double RH = 0, RN = 0, RK = 0, RL = 0;
                for (m = 0; m < Ln; ++m) {
                    if (m == a) continue;
                    const double d = (P->th[a] - P->th[m]) * PI / 180;
                    RH = RH + P->V[m] * (creal(Y(a, m)) * sin(d) - cimag(Y(a, m)) * cos(d));
                    RN = RN + P->V[m] * (creal(Y(a, m)) * cos(d) + cimag(Y(a, m)) * sin(d));
                }
                RK = RN;
                RL = RH;
                for (b = 1; b < Ln; ++b) {
                    const double d = (P->th[a] - P->th[b]) * PI / 180;
                    const double re = creal(Y(a, b)), im = cimag(Y(a, b));
                    if (a != b) {
                        JM(a - 1, b - 1) = P->V[a] * P->V[b] * (re * sin(d) - im * cos(d));
                        JM(a - 1, Ln - 1 + b - 1) = P->V[a] * (re * cos(d) + im * sin(d));
                        JM(Ln - 1 + a - 1, b - 1) = -P->V[a] * P->V[b] * (re * cos(d) + im * sin(d));
                        JM(Ln - 1 + a - 1, Ln - 1 + b - 1) = P->V[a] * (re * sin(d) - im * cos(d));
                    } else {
                        JM(a - 1, b - 1) = (double)(-P->V[a] * RH);
                        JM(a - 1, Ln - 1 + b - 1) = (double)(RN + 2 * P->V[a] * creal(Y(a, a)));
                        JM(Ln - 1 + a - 1, b - 1) = (double)(P->V[a] * RK);
                        JM(Ln - 1 + a - 1, Ln - 1 + b - 1) = (double)(-2 * P->V[a] * cimag(Y(a, b)) + RL);
                    }
                }
            }
            /* lambda = -inv(J^T) Fx (VoltVarCtrl.cpp:1243-1245) */
            for (a = 0; a < nf; ++a)
                for (b = 0; b < nf; ++b) Jt[(size_t)a + (size_t)b * nf] = JM(b, a);
            if (lu_inverse(Jt, nf, Ji)) rc = REF_BAD_INPUT;
            for (a = 0; a < nf; ++a) {
                double s = 0;
                for (b = 0; b < nf; ++b) s += (-Ji[(size_t)a + (size_t)b * nf]) * Fx[b];
                lam[a] = s;
            }
            /* Gqq (:1261-1297): -1 where the V-list bus ia+1 is load ja; g = -gu^T lambda (:1307-1309) */
            n_loads[x] = lload[x] < ld ? lload[x] : ld;
            for (j = 0; j < lload[x] && j < ld; ++j) {
                double s = 0;
                for (a = 0; a < Lnm; ++a) s += 0.0 * lam[a];   /* the Gpq block (zeros) */
                for (a = 0; a < Lnm; ++a)
                    if (P->node[a + 1] == load[x][j]) s += 1.0 * lam[Lnm + a];   /* (-Gqq) * lambda */
                g[(size_t)x * ld + j] = s;
                load_nodes[(size_t)x * ld + j] = load[x][j];
                if (fabs(s) < gx_min) gx_min = fabs(s);
                if (fabs(s) > gx_max) gx_max = fabs(s);
            }
            if (gx_min < gmin) gmin = gx_min;
            if (gx_max > gmax) gmax = gx_max;
            if (gx_min < gabs_min) gabs_min = gx_min;
#undef JM
#undef Y
            free(Fx);
            free(J);
            free(Jt);
            free(Ji);
            free(lam);
        }
        if (stats) {
            stats[0] = gmin;
            stats[1] = gmax;
            stats[2] = gabs_min;
            stats[3] = beta0 / (bkva / 3) / gabs_min;   /* cvq (:1323) */
        }
    }
done:
    for (x = 0; x < 3; ++x) { phase_free(&ph[x]); free(load[x]); }
    free(node_f);
    free(brnches);
    return rc;
}

/* the candidate control of one step size (:1334-1371) */
static void candidate(const double *ctrl, double *out, int nl, int ncols, const double *g, const double *ln,
                      const int *nload, int ld, double bkva, double c) {
    int x, i, r;
    memcpy(out, ctrl, sizeof(double) * (size_t)nl * ncols);
    for (x = 0; x < 3; ++x)
        for (i = 0; i < nload[x]; ++i) {
            const double gup = g[(size_t)x * ld + i] * (bkva / 3) * c;
            for (r = 0; r < nl; ++r)
                if (ctrl[r + 2 * (size_t)nl] == ln[(size_t)x * ld + i])
                    out[r + (size_t)(7 + 2 * x) * nl] = ctrl[r + (size_t)(7 + 2 * x) * nl] - gup;
        }
}

static int loss_of(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols, const ref_opts *o,
                   double *loss, double *vmin, double *vmax) {
    const int nn = ref_count_nodes(dl, nl, ncols);
    int lnum[3], rc;
    double *vp = (double *)calloc((size_t)nn * 6, sizeof(double));
    double *pb = (double *)calloc((size_t)nn * 6, sizeof(double));
    double *pl = (double *)calloc((size_t)nn * 6, sizeof(double));
    ref_out out;
    memset(&out, 0, sizeof(out));
    out.vpolar = vp;
    out.pqb = pb;
    out.pql = pl;
    rc = ref_dpf_solve(dl, nl, ncols, z, z_rows, z_cols, o, &out);
    if (rc == REF_CONVERGED && ref_lnum(dl, nl, ncols, z, z_rows, z_cols, o->bkva, o->bkv, lnum) == 0)
        ref_vvc_reduce(vp, pb, pl, nn, lnum, loss, vmin, vmax);
    free(vp);
    free(pb);
    free(pl);
    return rc;
}

/* The whole numerics of vvc_main (VoltVarCtrl.cpp:1141-1762), sequentially, one
 * DPF per call as the reference: base solve, gradient, the step-size search,
 * its reversal.  res (13 doubles): [ploss_orig, vmin_orig, vmax_orig, c0,
 * stop_fwd, stop_rev, reversed, sent, ploss_after, gmin, gmax, gabs_min, calls];
 * loss_fwd / loss_rev [m_max]: Ploss_osize of every step evaluated;
 * dl_out: the control after the round (Dl).  Returns 0, REF_NONCONVERGED (a
 * solve did not converge: the reference throws) or REF_BAD_INPUT. */
int ref_vvc_main(const double *dl_in, int nl, int ncols, const double *z, int z_rows, int z_cols, const ref_opts *o,
                 double beta0, double alpha, int m_max, int ld, double *g, double *load_nodes, int *n_loads,
                 double *loss_fwd, double *loss_rev, double *dl_out, double *res)
{
    const double *dl = dl_in;
    const int nn = ref_count_nodes(dl, nl, ncols);
    double *vp = (double *)calloc((size_t)nn * 6, sizeof(double));
    double *cand = (double *)malloc(sizeof(double) * (size_t)nl * ncols);
    double stats[4], ploss_orig = 0, vmin0 = 0, vmax0 = 0, after = 0;
    int rc, m, pass, calls = 1, stop[2] = {-1, -1}, flag = 1, sent = 0;
    ref_out out;
    memset(&out, 0, sizeof(out));
    out.vpolar = vp;
    memcpy(dl_out, dl, sizeof(double) * (size_t)nl * ncols);
    rc = ref_dpf_solve(dl, nl, ncols, z, z_rows, z_cols, o, &out);
    if (rc == REF_CONVERGED) rc = loss_of(dl, nl, ncols, z, z_rows, z_cols, o, &ploss_orig, &vmin0, &vmax0);
    if (rc == REF_CONVERGED)
        rc = ref_vvc_gradient(dl, nl, ncols, z, z_rows, z_cols, vp, nn, o->bkva, o->bkv, beta0, ld, g, load_nodes,
                              n_loads, stats);
    for (pass = 0; pass < 2 && rc == REF_CONVERGED; ++pass) {
        double *lossv = pass == 0 ? loss_fwd : loss_rev;
        double c;
        if (pass == 1 && flag) break;
        c = pass == 0 ? stats[3] : -beta0 / (o->bkva / 3) / stats[2];   /* :1323, :1546 */
        for (m = 0; m < m_max; ++m) {
            double lo = 0, ln = 0, vmn, vmx;
            candidate(dl, cand, nl, ncols, g, load_nodes, n_loads, ld, o->bkva, c);
            rc = loss_of(cand, nl, ncols, z, z_rows, z_cols, o, &lo, &vmn, &vmx);
            ++calls;
            if (rc) break;
            lossv[m] = lo;
            c = alpha * c;
            {
                double *c2 = (double *)malloc(sizeof(double) * (size_t)nl * ncols);
                candidate(dl, c2, nl, ncols, g, load_nodes, n_loads, ld, o->bkva, c);
                rc = loss_of(c2, nl, ncols, z, z_rows, z_cols, o, &ln, &vmn, &vmx);
                ++calls;
                if (ln > lo && rc == 0) {
                    memcpy(dl_out, cand, sizeof(double) * (size_t)nl * ncols);   /* Dl = Dl_osize */
                    after = lo;
                    stop[pass] = m;
                    if (lo < ploss_orig) sent = 1;
                }
                free(c2);
            }
            if (rc || stop[pass] >= 0) break;
            after = lo;
            if (after > ploss_orig && pass == 0) flag = 0;
        }
    }
    if (res) {
        res[0] = ploss_orig;
        res[1] = vmin0;
        res[2] = vmax0;
        res[3] = stats[3];
        res[4] = stop[0];
        res[5] = stop[1];
        res[6] = !flag;
        res[7] = sent;
        res[8] = after;
        res[9] = stats[0];
        res[10] = stats[1];
        res[11] = stats[2];
        res[12] = calls;
    }
    free(vp);
    free(cand);
    return rc;
}
