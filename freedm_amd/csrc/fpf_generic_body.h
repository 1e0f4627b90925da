// fpf_generic_body.h -- the exact sweep of one scenario on three lanes (one per
// phase) with its state streamed through global memory: the body of
// dpf_generic3_kernel (fpf_generic.hip) and of the exact re-solve
// of scenarios the fast kernels flag in their convergence guard
// (dpf_fixup_kernel, and the tail of the wave / wave-block kernels).  Every
// operation is the reference's, on the same operands, in the same order
// (Broker/src/vvc/DPF_return7.cpp:8-263; bit-identical to the parity oracle).
#pragma once
#include "fpf_internal.h"
#include "fpf_math.hpp"

namespace fpf {

namespace g3 {
struct Slots3 {
    double *base;
    size_t ld3;
    int i;   // 3 s + p
    __device__ __forceinline__ cx ld_(int k) const {
        return mk(base[(size_t)(2 * k) * ld3 + i], base[(size_t)(2 * k + 1) * ld3 + i]);
    }
    __device__ __forceinline__ void st(int k, cx v) const {
        base[(size_t)(2 * k) * ld3 + i] = v.re;
        base[(size_t)(2 * k + 1) * ld3 + i] = v.im;
    }
};
__device__ __forceinline__ cx shfl_cx(cx v, int src) { return mk(__shfl(v.re, src, 64), __shfl(v.im, src, 64)); }

constexpr int G3_SPW = 21;   // scenarios per wavefront (three lanes each; lane 63 idles)

// Deterministic reduction of one workgroup of NT threads over scenarios
// [lo, hi): [loss_sum, vmin, vmax, n_conv, n_nonconv, n_over, n_under, 0] over
// converged scenarios, thread t taking t, t + NT, ... and a fixed tree; the
// result in sh[q][0] (sh: [8][NT] shared)
template <int NT>
__device__ void block_aggregate(int lo, int hi, const int8_t *status, const double *loss, const double *vmin,
                                const double *vmax, double lb_v, double ub_v, double (*sh)[NT]) {
    const int t = threadIdx.x;
    double ls = 0, mn = INFINITY, mx = -INFINITY, nc = 0, nnc = 0, no = 0, nu = 0;
    for (int s = lo + t; s < hi; s += NT) {
        if (status[s] == 0) {
            ls += loss[s];
            mn = fmin(mn, vmin[s]);
            mx = fmax(mx, vmax[s]);
            nc += 1;
            if (vmax[s] > ub_v) no += 1;
            if (vmin[s] < lb_v) nu += 1;
        } else if (status[s] == FPF_NONCONVERGED) {   // (not FPF_EXCHANGE_FAILED)
            nnc += 1;
        }
    }
    sh[0][t] = ls; sh[1][t] = mn; sh[2][t] = mx; sh[3][t] = nc;
    sh[4][t] = nnc; sh[5][t] = no; sh[6][t] = nu; sh[7][t] = 0;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
        if (t < w) {
            sh[0][t] += sh[0][t + w];
            sh[1][t] = fmin(sh[1][t], sh[1][t + w]);
            sh[2][t] = fmax(sh[2][t], sh[2][t + w]);
            for (int q = 3; q < 8; ++q) sh[q][t] += sh[q][t + w];
        }
        __syncthreads();
    }
}

// FIX = false: scenario s = the thread group's index in the batch (layout
// [field][row][B]; the host transposes scenario-major batches around it).
// FIX = true (dpf_fixup_kernel): the exact re-solve of the scenarios a fast
// kernel flagged in its guard band (fpf_wave.hip) -- group g takes flag_ids[j]
// for j = g, g + groups, ... < *flag_count, its scratch column is g, the loads
// and results are addressed at the flagged id in the batch's own layout
// (o.smaj); then, if any was flagged, the batch aggregate again and the count
// back to 0 for the next launch.
template <bool FIX>
__device__ __forceinline__ void g3_solve(const FeederDev &f, int B, const double *__restrict__ pq,
                                         double *__restrict__ scr, size_t ld, const OutDev &o, int grp,
                                         int n_groups, int n_work, const int *local_ids = nullptr) {
    const int lane = threadIdx.x & 63;
    const int sw = lane / 3, p = lane - 3 * sw, g0 = 3 * sw;   // scenario in the wave, phase, group's first lane
    const bool lane_ok = lane < 3 * G3_SPW;
    const int nl = f.nl, nn = f.nn;
    const size_t ld3 = 3 * ld;
    if (!FIX && (!lane_ok || grp >= B)) return;   // no lane reads an idle lane: shuffles stay inside a group
    const int smaj = FIX ? o.smaj : 0;
    // (field, row) of scenario s's loads, (column, row) of its Nn-row outputs
    auto pq_at = [&](int s, int fld, int r) -> double {
        return smaj ? pq[(size_t)s * 6 * nl + (size_t)fld * nl + r] : pq[((size_t)fld * nl + r) * B + s];
    };
    auto o6 = [&](int s, int col, int k) -> size_t {
        return smaj ? (size_t)s * 6 * nn + (size_t)col * nn + k : ((size_t)col * nn + k) * B + s;
    };
    auto o3 = [&](int s, int col, int k) -> size_t {
        return smaj ? (size_t)s * 3 * nn + (size_t)col * nn + k : ((size_t)col * nn + k) * B + s;
    };
    for (int j = grp; j < n_work; j += n_groups) {
        if (FIX && !lane_ok) break;   // (the whole loop is wave-uniform apart from idle lane 63)
        // (the flagged ids were published with agent-scope stores by other workgroups,
        // or by the calling workgroup in LDS: local_ids)
        const int s = !FIX ? j
                           : (local_ids ? local_ids[j]
                                        : __hip_atomic_load(o.flag_ids + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        const int i3 = 3 * (FIX ? grp : s) + p;
        const Slots3 V{scr + (size_t)nl * 2 * ld3, ld3, i3};
        const Slots3 IL{scr + (size_t)nl * 4 * ld3, ld3, i3};
        const Slots3 Ib{scr + (size_t)(2 * nl + nn) * 2 * ld3, ld3, i3};
        const cx v0 = mk(f.V0[2 * p], f.V0[2 * p + 1]);
        // Sld(row) = (P + jQ) / (bkva/3) (:46-50), read from the caller's loads at every
        // use (the same division, the same bits) instead of a scratch copy
        auto Sld = [&](int row) { return cdiv(mk(pq_at(s, 2 * p, row), pq_at(s, 2 * p + 1, row)), mk(f.s3, 0.0)); };

        // V(0..Nl-1) = V0 (:92-96): only where a read could see it (FeederDev.v_init)
        if (f.v_init) {
            for (int r = 0; r < nl; ++r) V.st(r, v0);
        } else {
            V.st(0, v0);
        }
        // IL and Ib slots no op writes stay 0 (the ops rewrite all the others)
        for (int q = 0; q < f.n_il_zero; ++q) IL.st(f.il_zero[q], mk(0, 0));
        for (int q = 0; q < f.n_ib_zero; ++q) Ib.st(f.ib_zero[q], mk(0, 0));
        cx ibo = mk(0, 0);
        int iters = 0, status = 1;
        double errmx_last = 0.0;
        // the load currents of sweep it (IL of the final sweep, the post-processing's
        // Ild); sweep 0 of a feeder without the V0 fill reads V0 (not a stale slot)
        auto store_il = [&](int it) {
            const bool vconst = it == 0 && !f.v_init;
            int q = 0;
            for (; q + 4 <= f.n_il; q += 4) {
                IlOp op[4];
                cx sl[4], vv[4];
                for (int u = 0; u < 4; ++u) {
                    op[u] = f.il_ops[q + u];
                    sl[u] = Sld(op[u].row);
                    vv[u] = vconst ? v0 : V.ld_(op[u].ndr);
                }
                for (int u = 0; u < 4; ++u) IL.st(op[u].ndr - 1, load_current(sl[u], vv[u]));
            }
            for (; q < f.n_il; ++q) {
                const IlOp op = f.il_ops[q];
                IL.st(op.ndr - 1, load_current(Sld(op.row), vconst ? v0 : V.ld_(op.ndr)));
            }
        };
        for (int it = 0; it < f.mxitr; ++it) {
            // backward sweep :134-160 (as dpf_generic_kernel, one phase per lane)
            cx ibl = mk(0, 0);
            // sweep 0 of a feeder without the V0 fill: every load current sees V0
            const bool vconst = it == 0 && !f.v_init;
            auto vload = [&](int ndr) { return vconst ? v0 : V.ld_(ndr); };
            if (f.n_bw > 0) {
                BwOp op = f.bw_ops[0];
                IlOp w = f.bw_il[0];
                cx sl = w.row < 0 ? mk(0, 0) : Sld(w.row), vv = w.row < 0 ? mk(0, 0) : vload(w.ndr);
                for (int q = 0; q < f.n_bw; ++q) {
                    const bool more = q + 1 < f.n_bw;
                    BwOp nx = op;
                    cx nsl = mk(0, 0), nvv = mk(0, 0);
                    if (more) {
                        nx = f.bw_ops[q + 1];
                        const IlOp wn = f.bw_il[q + 1];
                        if (wn.row >= 0) {
                            nsl = Sld(wn.row);
                            nvv = vload(wn.ndr);
                        }
                    }
                    const bool has_il = f.bw_il[q].row >= 0;
                    const cx il = has_il ? load_current(sl, vv) : mk(0, 0);
                    const bool first = op.kind & 2;
                    const cx ib = first ? mk(0, 0) : Ib.ld_(op.idx);
                    if (op.kind & 1) {
                        Ib.st(op.idx, cadd(ib, ibl));
                        ibl = mk(0, 0);
                    } else {
                        const cx x = cadd(cadd(ib, ibl), il);
                        Ib.st(op.idx, x);
                        ibl = x;
                    }
                    sl = nsl;
                    vv = nvv;
                    op = nx;
                }
            }
            // convergence :199-210, the reference's max over the phases in phase order
            const cx d = csub(Ib.ld_(0), ibo);
            const double df = hypot(d.re, d.im);
            const double d0 = __shfl(df, g0, 64), d1 = __shfl(df, g0 + 1, 64), d2 = __shfl(df, g0 + 2, 64);
            double errmx = d0;
            if (d1 > errmx) errmx = d1;
            if (d2 > errmx) errmx = d2;
            errmx_last = errmx;
            ibo = Ib.ld_(0);
            const bool conv = errmx < f.eps;
            if (conv || it + 1 == f.mxitr) store_il(it);
            // forward sweep :163-195, software-pipelined as dpf_generic_kernel
            if (f.n_fw > 0) {
                FwOp op = f.fw_ops[0];
                cx b = Ib.ld_(op.ib);
                cx sv = op.src < 0 ? v0 : V.ld_(op.src);
                for (int q = 0; q < f.n_fw; ++q) {
                    const bool more = q + 1 < f.n_fw;
                    FwOp nx = op;
                    cx nb = mk(0, 0), nsv = mk(0, 0);
                    if (more) {
                        nx = f.fw_ops[q + 1];
                        nb = Ib.ld_(nx.ib);
                        if (!(nx.pad & 1)) nsv = nx.src < 0 ? v0 : V.ld_(nx.src);
                    }
                    const cx b0 = shfl_cx(b, g0), b1 = shfl_cx(b, g0 + 1), b2 = shfl_cx(b, g0 + 2);
                    cx rv = csub(sv, drop_col(f.tz + 18 * (size_t)q, b0, b1, b2, p));
                    if (op.mask & (1 << p)) rv = mk(0, 0);
                    V.st(op.dst, rv);
                    if (more && (nx.pad & 1)) nsv = rv;
                    b = nb;
                    sv = nsv;
                    op = nx;
                }
            }
            iters = it + 1;
            if (conv) { status = 0; break; }
        }

        // post-processing (:222-253) with the VVC reductions, per phase; the
        // scenario's loss / Vmin / Vmax combine the phases in the reference's order
        double acc1 = 0, acc2 = 0, pb0 = 0, mn = INFINITY, mx = -INFINITY;
        int cnt = 0;
        for (int k = 0; k < nn; ++k) {
            const cx v = V.ld_(k);
            const cx ib = Ib.ld_(k == 0 ? 0 : k - 1);
            const cx il = IL.ld_(k == 0 ? nn - 1 : k - 1);
            const cx sv = cmul(v, mk(f.s3, 0.0));
            const cx sb = cmul(sv, cconj(ib));
            const cx sl = cmul(sv, cconj(il));
            const double mag = hypot(v.re, v.im);
            if (o.vpolar) { o.vpolar[o6(s, 2 * p, k)] = mag; o.vpolar[o6(s, 2 * p + 1, k)] = polar_angle(v, p); }
            if (o.pqb) { o.pqb[o6(s, 2 * p, k)] = sb.re; o.pqb[o6(s, 2 * p + 1, k)] = sb.im; }
            if (o.pql) { o.pql[o6(s, 2 * p, k)] = sl.re; o.pql[o6(s, 2 * p + 1, k)] = sl.im; }
            if (o.v_re) o.v_re[o3(s, p, k)] = v.re;
            if (o.v_im) o.v_im[o3(s, p, k)] = v.im;
            if (k & 1) acc2 += sl.re; else acc1 += sl.re;
            if (k == 0) pb0 = sb.re;
            if (mag != 0 && cnt < f.K[p]) {
                mn = fmin(mn, mag);
                mx = fmax(mx, mag);
                ++cnt;
            }
        }
        const double x = pb0 - (acc1 + acc2);
        const double pmin = cnt < f.K[p] ? fmin(mn, 0.0) : mn;
        const double pmax = cnt < f.K[p] ? fmax(mx, 0.0) : mx;
        const double x0 = __shfl(x, g0, 64), x1 = __shfl(x, g0 + 1, 64), x2 = __shfl(x, g0 + 2, 64);
        const double n0 = __shfl(pmin, g0, 64), n1 = __shfl(pmin, g0 + 1, 64), n2 = __shfl(pmin, g0 + 2, 64);
        const double m0 = __shfl(pmax, g0, 64), m1 = __shfl(pmax, g0 + 1, 64), m2 = __shfl(pmax, g0 + 2, 64);
        if (p == 0) {
            const double loss = ((0.0 + x0) + x2) + (0.0 + x1);
            double vmin = n0, vmax = m0;
            if (n1 < vmin) vmin = n1;
            if (m1 > vmax) vmax = m1;
            if (n2 < vmin) vmin = n2;
            if (m2 > vmax) vmax = m2;
            if (o.iters) o.iters[s] = iters;
            if (o.status) o.status[s] = (int8_t)status;
            if (o.loss) o.loss[s] = loss;
            if (o.vmin) o.vmin[s] = vmin;
            if (o.vmax) o.vmax[s] = vmax;
            if (o.errmx) o.errmx[s] = errmx_last;
            if (o.guard) o.guard[s] = FIX ? 1 : 0;
        }
    }
}

// The exact re-solve of the n scenarios ids[0..n) a fast workgroup flagged
// itself (a solve without an aggregate: fpf_wave.hip), called by its first
// wave: one group of three lanes takes them in turn, its state in the
// workgroup's LDS (scr, 96 (Nl + Nn) bytes: fpf_api.cpp checks it fits), the
// results written at the scenarios' batch indices.  Not inlined: the fast
// kernel keeps its registers for the sweep.
__device__ __noinline__ void g3_fixup_local(const FeederDev *f, int B, const double *pq, double *scr,
                                            const OutDev *o, const int *ids, int n) {
    if ((threadIdx.x & 63) >= 3) return;
    g3_solve<true>(*f, B, pq, scr, 1, *o, 0, 1, n, ids);
}

}  // namespace g3
}  // namespace fpf
