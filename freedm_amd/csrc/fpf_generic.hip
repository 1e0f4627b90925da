// fpf_generic.hip -- the generic batched DPF kernel for gfx950.
//
// One lane per scenario; every lane runs the reference's sweep program
// (DPF_return7.cpp:102-218) verbatim from the feeder's op lists, so it is exact
// for ANY feeder that passes the index checks (including the malformed orders
// the tiled kernel refuses).  Per-scenario state (Sld, V, IL, Ib) is streamed
// through HBM in a scenario-fastest SoA layout -- slot k, field f of scenario s
// at base[(2k+f)*ld + s] -- so consecutive lanes touch consecutive doubles.
// The op lists are wave-uniform (scalar loads); lanes diverge only at their own
// convergence break (a converged lane stops updating, like the reference).
#include "fpf_internal.h"
#include "fpf_math.hpp"
#include "fpf_generic_body.h"

#include <cstdlib>

#pragma clang fp contract(off)

namespace fpf {

namespace {

struct Slots {
    double *base;
    size_t ld;
    int s;
    __device__ __forceinline__ cx ld_(int slot) const {
        return mk(base[(size_t)(2 * slot) * ld + s], base[(size_t)(2 * slot + 1) * ld + s]);
    }
    __device__ __forceinline__ void st(int slot, cx v) const {
        base[(size_t)(2 * slot) * ld + s] = v.re;
        base[(size_t)(2 * slot + 1) * ld + s] = v.im;
    }
};

}  // namespace

__global__ __launch_bounds__(256) void dpf_generic_kernel(FeederDev f, int B,
                                                          const double *__restrict__ pq,
                                                          double *__restrict__ scr, size_t ld,
                                                          OutDev o) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    const int nl = f.nl, nn = f.nn;
    const Slots Sld{scr, ld, s};
    const Slots V{scr + (size_t)nl * 6 * ld, ld, s};
    const Slots IL{scr + (size_t)nl * 12 * ld, ld, s};
    const Slots Ib{scr + (size_t)(2 * nl + nn) * 6 * ld, ld, s};
    const cx v0[3] = {mk(f.V0[0], f.V0[1]), mk(f.V0[2], f.V0[3]), mk(f.V0[4], f.V0[5])};

    // Sld = (P + jQ) / (bkva/3)   DPF_return7.cpp:46-50
    for (int j = 0; j < nl; ++j)
        for (int p = 0; p < 3; ++p) {
            const cx sl = mk(pq[((size_t)(2 * p) * nl + j) * B + s], pq[((size_t)(2 * p + 1) * nl + j) * B + s]);
            Sld.st(j * 3 + p, cdiv(sl, mk(f.s3, 0.0)));
            V.st(j * 3 + p, v0[p]);                                  // :92-96
        }

    // IL and Ib are fresh zeros every sweep (:106, :134).  The load-current ops
    // write the same IL slots every sweep (stored once, final sweep) and each Ib
    // slot's first op reads the constant 0 (BwOp kind | 2), so only the slots no
    // op writes need zeroing, and that once: they are never written afterwards
    for (int k = 0; k < nn * 3; ++k) IL.st(k, mk(0, 0));
    for (int k = 0; k < (nn - 1) * 3; ++k) Ib.st(k, mk(0, 0));
    cx ibo[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
    int iters = 0, status = 1;
    // load currents  :106-130.  IL itself is only stored for the final sweep
    // (the post-processing's Ild); during the sweeps the backward pass
    // evaluates each IL it adds from the same Sld and (not yet updated) V.
    // 4 ops' loads are issued before their stores (IL, Sld and V are disjoint
    // slot ranges; the stores keep list order, so a repeated slot's last write wins)
    auto store_il = [&]() {
        int q = 0;
        for (; q + 4 <= f.n_il; q += 4) {
            IlOp op[4];
            cx sl[4][3], vv[4][3];
            for (int u = 0; u < 4; ++u) {
                op[u] = f.il_ops[q + u];
                for (int p = 0; p < 3; ++p) {
                    sl[u][p] = Sld.ld_(op[u].row * 3 + p);
                    vv[u][p] = V.ld_(op[u].ndr * 3 + p);
                }
            }
            for (int u = 0; u < 4; ++u)
                for (int p = 0; p < 3; ++p) IL.st((op[u].ndr - 1) * 3 + p, load_current(sl[u][p], vv[u][p]));
        }
        for (; q < f.n_il; ++q) {
            const IlOp op = f.il_ops[q];
            for (int p = 0; p < 3; ++p)
                IL.st((op.ndr - 1) * 3 + p, load_current(Sld.ld_(op.row * 3 + p), V.ld_(op.ndr * 3 + p)));
        }
    };
    for (int it = 0; it < f.mxitr; ++it) {
        // backward sweep  :134-160
        // IL(idx) of a branch op = load_current of the op that last writes that
        // slot in the load-current pass (FeederDev.bw_il; none: 0).  Op q+1's
        // Sld and V operands are loaded before op q runs (neither is written here)
        cx ibl[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
        auto il_operands = [&](int q, cx sl[3], cx vv[3]) {
            const IlOp w = f.bw_il[q];
            for (int p = 0; p < 3; ++p) {
                sl[p] = w.row < 0 ? mk(0, 0) : Sld.ld_(w.row * 3 + p);
                vv[p] = w.row < 0 ? mk(0, 0) : V.ld_(w.ndr * 3 + p);
            }
        };
        if (f.n_bw > 0) {
            BwOp op = f.bw_ops[0];
            cx sl[3], vv[3];
            il_operands(0, sl, vv);
            for (int q = 0; q < f.n_bw; ++q) {
                const bool more = q + 1 < f.n_bw;
                BwOp nx = op;
                cx nsl[3], nvv[3];
                if (more) {
                    nx = f.bw_ops[q + 1];
                    il_operands(q + 1, nsl, nvv);
                }
                const bool has_il = f.bw_il[q].row >= 0;    // wave-uniform
                cx il[3];
                for (int p = 0; p < 3; ++p) il[p] = has_il ? load_current(sl[p], vv[p]) : mk(0, 0);
                const bool first = op.kind & 2;    // wave-uniform
                auto ib = [&](int p) { return first ? mk(0, 0) : Ib.ld_(op.idx * 3 + p); };
                if (op.kind & 1) {
                    for (int p = 0; p < 3; ++p) Ib.st(op.idx * 3 + p, cadd(ib(p), ibl[p]));
                    for (int p = 0; p < 3; ++p) ibl[p] = mk(0, 0);
                } else {
                    for (int p = 0; p < 3; ++p) {
                        const cx x = cadd(cadd(ib(p), ibl[p]), il[p]);
                        Ib.st(op.idx * 3 + p, x);
                        ibl[p] = x;
                    }
                }
                if (more)
                    for (int p = 0; p < 3; ++p) {
                        sl[p] = nsl[p];
                        vv[p] = nvv[p];
                    }
                op = nx;
            }
        }
        // convergence  :199-210 -- tested here, before the forward sweep, which
        // does not touch Ib; the forward sweep still runs in the final sweep
        double errmx = 0;
        for (int p = 0; p < 3; ++p) {
            const cx d = csub(Ib.ld_(p), ibo[p]);
            const double df = hypot(d.re, d.im);
            if (p == 0 || df > errmx) errmx = df;
        }
        for (int p = 0; p < 3; ++p) ibo[p] = Ib.ld_(p);
        const bool conv = errmx < f.eps;
        if (o.errmx) o.errmx[s] = errmx;
        if (conv || it + 1 == f.mxitr) store_il();   // the final sweep's IL (Ild)
        // forward sweep  :163-195
        // software-pipelined: op q+1's Ib (not written here) and source V are
        // loaded before op q stores; when op q+1 reads the V op q writes
        // (FwOp.pad & 1, the chain case) the value comes from registers
        if (f.n_fw > 0) {
            FwOp op = f.fw_ops[0];
            cx b[3], sv[3];
            for (int p = 0; p < 3; ++p) {
                b[p] = Ib.ld_(op.ib * 3 + p);
                sv[p] = op.src < 0 ? v0[p] : V.ld_(op.src * 3 + p);
            }
            for (int q = 0; q < f.n_fw; ++q) {
                const bool more = q + 1 < f.n_fw;
                FwOp nx = op;
                cx nb[3], nsv[3];
                if (more) {
                    nx = f.fw_ops[q + 1];
                    for (int p = 0; p < 3; ++p) {
                        nb[p] = Ib.ld_(nx.ib * 3 + p);
                        nsv[p] = mk(0, 0);
                        if (!(nx.pad & 1)) nsv[p] = nx.src < 0 ? v0[p] : V.ld_(nx.src * 3 + p);
                    }
                }
                const double *t = f.tz + 18 * (size_t)q;
                for (int p = 0; p < 3; ++p) {
                    cx rv = csub(sv[p], drop_col(t, b[0], b[1], b[2], p));
                    if (op.mask & (1 << p)) rv = mk(0, 0);
                    V.st(op.dst * 3 + p, rv);
                    if (more && (nx.pad & 1)) nsv[p] = rv;
                }
                if (more)
                    for (int p = 0; p < 3; ++p) {
                        b[p] = nb[p];
                        sv[p] = nsv[p];
                    }
                op = nx;
            }
        }
        iters = it + 1;
        if (conv) { status = 0; break; }
    }

    // post-processing (:222-253) fused with the VVC reductions
    // (loss VoltVarCtrl.cpp:1152-1161, V_abc_list.cpp:7-81, Vmin/Vmax :1201-1207)
    double acc1[3] = {0, 0, 0}, acc2[3] = {0, 0, 0}, pb0[3] = {0, 0, 0};
    double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    int cnt[3] = {0, 0, 0};
    for (int k = 0; k < nn; ++k) {
        for (int p = 0; p < 3; ++p) {
            const cx v = V.ld_(k * 3 + p);
            const cx ib = Ib.ld_((k == 0 ? 0 : k - 1) * 3 + p);
            const cx il = IL.ld_((k == 0 ? nn - 1 : k - 1) * 3 + p);
            const cx sv = cmul(v, mk(f.s3, 0.0));
            const cx sb = cmul(sv, cconj(ib));
            const cx sl = cmul(sv, cconj(il));
            const double mag = hypot(v.re, v.im);
            const size_t o6 = ((size_t)(2 * p) * nn + k) * B + s, o6i = o6 + (size_t)nn * B;
            if (o.vpolar) { o.vpolar[o6] = mag; o.vpolar[o6i] = polar_angle(v, p); }
            if (o.pqb) { o.pqb[o6] = sb.re; o.pqb[o6i] = sb.im; }
            if (o.pql) { o.pql[o6] = sl.re; o.pql[o6i] = sl.im; }
            if (o.v_re) o.v_re[((size_t)p * nn + k) * B + s] = v.re;
            if (o.v_im) o.v_im[((size_t)p * nn + k) * B + s] = v.im;
            if (k & 1) acc2[p] += sl.re; else acc1[p] += sl.re;
            if (k == 0) pb0[p] = sb.re;
            if (mag != 0 && cnt[p] < f.K[p]) {
                mn[p] = fmin(mn[p], mag);
                mx[p] = fmax(mx[p], mag);
                ++cnt[p];
            }
        }
    }
    double x[3], pmin[3], pmax[3];
    for (int p = 0; p < 3; ++p) {
        x[p] = pb0[p] - (acc1[p] + acc2[p]);
        pmin[p] = cnt[p] < f.K[p] ? fmin(mn[p], 0.0) : mn[p];
        pmax[p] = cnt[p] < f.K[p] ? fmax(mx[p], 0.0) : mx[p];
    }
    const double loss = ((0.0 + x[0]) + x[2]) + (0.0 + x[1]);
    double vmin = pmin[0], vmax = pmax[0];
    for (int p = 1; p < 3; ++p) {
        if (pmin[p] < vmin) vmin = pmin[p];
        if (pmax[p] > vmax) vmax = pmax[p];
    }
    if (o.iters) o.iters[s] = iters;
    if (o.status) o.status[s] = (int8_t)status;
    if (o.loss) o.loss[s] = loss;
    if (o.vmin) o.vmin[s] = vmin;
    if (o.vmax) o.vmax[s] = vmax;
    if (o.guard) o.guard[s] = 0;
}

// ---------------------------------------------------------------------------
// Three lanes per scenario, one per phase: the same op lists and the same
// per-element operations in the same order as dpf_generic_kernel (bit-identical
// results), three times the wavefronts.  At 65 536 scenarios the one-lane form
// has one wavefront per SIMD and is bound by the memory requests it can keep in
// flight; here a wavefront holds 21 scenarios x 3 phases (lane 63 idles) and the
// state of slot k, field f (re/im) lives at base[(2k + f) * ld3 + 3 s + p], so a
// wavefront's access is still one contiguous 504-byte run.  The phases meet
// only where the reference mixes them: the branch product Ib . TEMP (the three
// Ib of a branch by lane shuffles), the convergence test (max over phases) and
// the per-scenario loss / Vmin / Vmax.
using namespace g3;

// FIX = false: scenario s = the thread group's index in the batch (layout
// [field][row][B]; the host transposes scenario-major batches around it).
// FIX = true (dpf_fixup_kernel): the exact re-solve of the scenarios a fast
// kernel flagged in its guard band (fpf_wave.hip) -- group g takes flag_ids[j]
// for j = g, g + groups, ... < *flag_count, its scratch column is g, the loads
// and results are addressed at the flagged id in the batch's own layout
// (o.smaj); then, if any was flagged, the batch aggregate again and the count
// back to 0 for the next launch.
template <bool FIX>
__global__ __launch_bounds__(256) void dpf_generic3_kernel(FeederDev f, int B, const double *__restrict__ pq,
                                                           double *__restrict__ scr, size_t ld, OutDev o) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int grp = (blockIdx.x * 4 + wv) * G3_SPW + lane / 3;
    const int n_work = FIX ? (int)__hip_atomic_load(o.flag_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : B;
    const int n_groups = FIX ? (int)(gridDim.x * 4 * G3_SPW) : B;
    g3_solve<FIX>(f, B, pq, scr, ld, o, grp, n_groups, n_work);
    if (FIX) {
        if (n_work == 0) return;   // (uniform: the common case, nothing flagged)
        // the batch aggregate over the corrected results (one workgroup: its own
        // stores above are visible to its threads behind the fence and barrier)
        __shared__ double sh[8][256];
        __threadfence();
        __syncthreads();
        if (o.agg) {
            block_aggregate<256>(0, B, o.status, o.loss, o.vmin, o.vmax, f.lb_v, f.ub_v, sh);
            if (threadIdx.x < 7) o.agg[threadIdx.x] = sh[threadIdx.x][0];
            if (threadIdx.x == 0) o.agg[7] = (double)B;
        }
        if (threadIdx.x == 0) __hip_atomic_store(o.flag_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}


hipError_t launch_generic(const FeederDev &f, int n_scen, const double *pq, double *scratch,
                          size_t ld, const OutDev &o, hipStream_t st) {
    static const bool one_lane = getenv("FPF_GENERIC_ONE_LANE") != nullptr;   // experiments
    const int block = 256;
    if (one_lane) {
        const int grid = (n_scen + block - 1) / block;
        hipLaunchKernelGGL(dpf_generic_kernel, dim3(grid), dim3(block), 0, st, f, n_scen, pq, scratch, ld, o);
    } else {
        const int per_block = 4 * G3_SPW;
        const int grid = (n_scen + per_block - 1) / per_block;
        hipLaunchKernelGGL(dpf_generic3_kernel<false>, dim3(grid), dim3(block), 0, st, f, n_scen, pq, scratch, ld, o);
    }
    return hipGetLastError();
}

// scratch columns the fixup kernel uses (its groups)
size_t fixup_scratch_ld() { return (size_t)FIXUP_BLOCKS * 4 * G3_SPW; }

// The exact re-solve of the scenarios the fast kernel flagged (o.flag_count /
// o.flag_ids); exits at once when none was (the common case)
hipError_t launch_fixup(const FeederDev &f, int n_scen, const double *pq, double *scratch, size_t ld, const OutDev &o,
                        hipStream_t st) {
    if (ld < fixup_scratch_ld() || !o.flag_count || !o.flag_ids) return hipErrorInvalidValue;
    hipLaunchKernelGGL(dpf_generic3_kernel<true>, dim3(FIXUP_BLOCKS), dim3(256), 0, st, f, n_scen, pq, scratch, ld, o);
    return hipGetLastError();
}

// Deterministic batch aggregate (fixed thread->scenario map and fixed tree):
// [loss_sum, vmin, vmax, n_conv, n_nonconv, n_over, n_under, n_scen].  Block g
// reduces scenarios [g*chunk, (g+1)*chunk); with several blocks each publishes
// its partial (agent-scope stores), takes a ticket, and the last one folds the
// partials in block order.
__global__ __launch_bounds__(1024) void dpf_aggregate_kernel(int B, int chunk, const int8_t *__restrict__ status,
                                                             const double *__restrict__ loss,
                                                             const double *__restrict__ vmin,
                                                             const double *__restrict__ vmax,
                                                             double lb_v, double ub_v, double *agg, double *partials,
                                                             unsigned *ticket) {
    __shared__ double sh[8][1024];
    __shared__ int last;
    const int t = threadIdx.x;
    const int lo = blockIdx.x * chunk, hi = min(B, lo + chunk);
    double ls = 0, mn = INFINITY, mx = -INFINITY, nc = 0, nnc = 0, no = 0, nu = 0;
    for (int s = lo + t; s < hi; s += blockDim.x) {
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
    auto tree = [&]() {
        __syncthreads();
        for (int w = blockDim.x / 2; w > 0; w >>= 1) {
            if (t < w) {
                sh[0][t] += sh[0][t + w];
                sh[1][t] = fmin(sh[1][t], sh[1][t + w]);
                sh[2][t] = fmax(sh[2][t], sh[2][t + w]);
                for (int q = 3; q < 8; ++q) sh[q][t] += sh[q][t + w];
            }
            __syncthreads();
        }
    };
    sh[0][t] = ls; sh[1][t] = mn; sh[2][t] = mx; sh[3][t] = nc;
    sh[4][t] = nnc; sh[5][t] = no; sh[6][t] = nu; sh[7][t] = 0;
    tree();
    if (gridDim.x == 1) {
        if (t < 7) agg[t] = sh[t][0];
        if (t == 0) agg[7] = (double)B;
        return;
    }
    if (t == 0) {
        for (int q = 0; q < 7; ++q)
            __hip_atomic_store(partials + 8 * (size_t)blockIdx.x + q, sh[q][0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
        last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    }
    __syncthreads();
    if (!last) return;
    double a[8] = {0, INFINITY, -INFINITY, 0, 0, 0, 0, 0};
    for (unsigned g = t; g < gridDim.x; g += blockDim.x) {
        for (int q = 0; q < 7; ++q) {
            const double r = __hip_atomic_load(partials + 8 * (size_t)g + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            a[q] = q == 1 ? fmin(a[q], r) : (q == 2 ? fmax(a[q], r) : a[q] + r);
        }
    }
    for (int q = 0; q < 8; ++q) sh[q][t] = a[q];
    tree();
    if (t < 7) agg[t] = sh[t][0];
    if (t == 0) {
        agg[7] = (double)B;
        __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// partials: [>= 256][8] scratch and ticket (0 between launches) for the
// multi-block form; NULL = one block
hipError_t launch_aggregate(int n_scen, const int8_t *status, const double *loss, const double *vmin,
                            const double *vmax, double lb_v, double ub_v, double *d_agg, double *partials,
                            unsigned *ticket, hipStream_t st) {
    int grid = 1, chunk = n_scen;
    if (partials && ticket && n_scen > 8192) {
        chunk = 4096;
        grid = (n_scen + chunk - 1) / chunk;
        if (grid > 256) {
            grid = 256;
            chunk = (n_scen + grid - 1) / grid;
        }
    }
    hipLaunchKernelGGL(dpf_aggregate_kernel, dim3(grid), dim3(1024), 0, st, n_scen, chunk, status, loss, vmin, vmax,
                       lb_v, ub_v, d_agg, partials, ticket);
    return hipGetLastError();
}

}  // namespace fpf
