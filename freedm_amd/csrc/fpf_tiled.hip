// fpf_tiled.hip -- the tiled batched DPF kernel for gfx950 (well-formed feeders).
//
// One workgroup owns a tile of TILE scenarios for the whole solve; their state
// lives in LDS for all sweeps, so HBM only sees the loads in and the results
// out.  One LDS slot per (node k, phase p, scenario s) -- W[(k*3+p)*TILE+s], a
// complex fp64 -- holds, in turn within a sweep:
//     V(k)  --P1-->  IL(k-1)  --S1-->  Ib(k-1)  --P2-->  drop(k)  --S2-->  V(k)
// Slot 0 keeps the constant V0 (the substation, DPF_return7.cpp:84-96).
//
//   P1 (parallel, one task per (s,k), 3 phases per lane):  IL = conj(Sld/V)   :106-130
//   S1 (sequential, one lane per (s,p)): the backward program in row order     :134-160
//      with tap accumulators in LDS, then the substation convergence test     :199-210
//   P2 (parallel): drop(k) = lng*(Ib(k-1) . Zl)  (TEMP table, ZGEMM order)    :163-178
//   S2 (sequential): V(dst) = V(src) - drop(dst), phase zeroing               :169-195
//   epilogue for scenarios that finish this sweep: Vpolar/PQb/PQL/V to HBM   :222-253
//      and the VVC reductions (loss, Vmin/Vmax) in the reference's order.
// Every arithmetic step is the reference's operation on the same operands, so V
// is bit-identical to the sequential program (and to the oracle).
//
// The parallel stages carry the divisions and the 3x3 products (>85 % of the
// flops); the sequential stages are 1-2 dependent complex adds per row.  A lane
// keeps Sld, IL and Ib of its tasks in VGPRs across the sweep.
#include "fpf_internal.h"
#include "fpf_math.hpp"

#pragma clang fp contract(off)

namespace fpf {

namespace {

constexpr int MAXT = 2;          // tasks per lane
constexpr int MAX_SEQ_TILE = 16; // 4 sequential lanes per scenario in one wave

struct Flags {
    int active[MAX_SEQ_TILE];    // still iterating
    int fin[MAX_SEQ_TILE];       // 1 = converged this sweep, 2 = hit mxitr this sweep
};

__device__ __forceinline__ cx lds_ld(const double2 *w, int i) {
    const double2 v = w[i];
    return mk(v.x, v.y);
}
__device__ __forceinline__ void lds_st(double2 *w, int i, cx v) { w[i] = make_double2(v.re, v.im); }

// Outputs of node k, phase p (DPF_return7.cpp:222-253).  Not inlined: it runs
// once per node per scenario, and inlining its hypot/atan six times per lane
// would cost the sweep loop its occupancy.  Returns (Re SL, |V|) for the
// ordered VVC reductions.
__device__ __noinline__ double2 emit_node(const OutDev &o, double s3, int nn, int B, int k, int p, size_t gs,
                                          cx v, cx ilv, cx ibv) {
    const cx sv = cmul(v, mk(s3, 0.0));
    const cx sb = cmul(sv, cconj(ibv));
    const cx sl = cmul(sv, cconj(ilv));
    const double mag = hypot(v.re, v.im);
    const size_t o6 = ((size_t)(2 * p) * nn + k) * B + gs, o6i = o6 + (size_t)nn * B;
    if (o.vpolar) { o.vpolar[o6] = mag; o.vpolar[o6i] = polar_angle(v, p); }
    if (o.pqb) { o.pqb[o6] = sb.re; o.pqb[o6i] = sb.im; }
    if (o.pql) { o.pql[o6] = sl.re; o.pql[o6i] = sl.im; }
    if (o.v_re) o.v_re[((size_t)p * nn + k) * B + gs] = v.re;
    if (o.v_im) o.v_im[((size_t)p * nn + k) * B + gs] = v.im;
    return make_double2(sl.re, mag);
}

}  // namespace

template <int NT>
__global__ __launch_bounds__(NT, 2) void dpf_tiled_kernel(FeederDev f, int B, const double *__restrict__ pq,
                                                       OutDev o, int TILE) {
    extern __shared__ double2 lds[];
    const int nn = f.nn, nb = nn - 1, nl = f.nl;
    double2 *W = lds;
    double2 *T = W + (size_t)nn * 3 * TILE;
    Flags *fl = (Flags *)(T + (size_t)f.n_taps * 3 * TILE);

    const int tid = threadIdx.x;
    const int s0 = blockIdx.x * TILE;
    const int ns = min(TILE, B - s0);
    const int ntask = TILE * nb;
    const cx v0[3] = {mk(f.V0[0], f.V0[1]), mk(f.V0[2], f.V0[3]), mk(f.V0[4], f.V0[5])};

    // ---- init: every V slot = V0 (:92-96), tap accumulators 0, flags
    for (int i = tid; i < nn * 3 * TILE; i += NT) {
        const int p = (i / TILE) % 3;
        lds_st(W, i, p == 0 ? v0[0] : (p == 1 ? v0[1] : v0[2]));
    }
    for (int i = tid; i < f.n_taps * 3 * TILE; i += NT) lds_st(T, i, mk(0, 0));
    if (tid < MAX_SEQ_TILE) {
        fl->active[tid] = tid < ns ? 1 : 0;
        fl->fin[tid] = 0;
    }

    // ---- per-task loads Sld = (P + jQ)/(bkva/3) (:46-50), kept in VGPRs
    cx sld[MAXT][3], il[MAXT][3], ib[MAXT][3];
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
        const int t = tid + j * NT;
        const int s = t % TILE, k = 1 + t / TILE;
        if (t < ntask && s < ns) {
            const int row = f.node_ops[k].row;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const cx sl = mk(pq[((size_t)(2 * p) * nl + row) * B + s0 + s],
                                 pq[((size_t)(2 * p + 1) * nl + row) * B + s0 + s]);
                sld[j][p] = cdiv(sl, mk(f.s3, 0.0));
            }
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) { il[j][p] = mk(0, 0); ib[j][p] = mk(0, 0); }
    }
    __syncthreads();

    // sequential-lane identity: lane (s, p) = tid (4 lanes per scenario, p=3 shadows p=2)
    const int qs = tid >> 2, qp4 = tid & 3, qp = qp4 < 3 ? qp4 : 2;
    const bool qlane = tid < 4 * TILE && qs < ns;
    const int gbase = (tid & 63) & ~3;
    cx ibo = mk(0, 0);

    int n_active = ns;
    for (int it = 0; it < f.mxitr && n_active > 0; ++it) {
        // ---- P1: load currents
#pragma unroll
        for (int j = 0; j < MAXT; ++j) {
            const int t = tid + j * NT;
            const int s = t % TILE, k = 1 + t / TILE;
            if (t < ntask && s < ns && fl->active[s]) {
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    const int w = (k * 3 + p) * TILE + s;
                    il[j][p] = load_current(sld[j][p], lds_ld(W, w));
                    lds_st(W, w, il[j][p]);
                }
            }
        }
        __syncthreads();

        // ---- S1: backward program + convergence
        if (qlane && fl->active[qs]) {
            cx ibl = mk(0, 0);
            const int n = f.n_seq_bw;
            for (int q = 0; q < n; ++q) {
                const SeqBw e = f.seq_bw[q];
                if (e.node == 0) {
                    const int ti = ((e.tap1 - 1) * 3 + qp) * TILE + qs;
                    const cx x = cadd(lds_ld(T, ti), ibl);
                    if (qp4 < 3) lds_st(T, ti, x);
                    ibl = mk(0, 0);
                } else {
                    const cx acc = e.tap1 ? lds_ld(T, ((e.tap1 - 1) * 3 + qp) * TILE + qs) : mk(0, 0);
                    const int w = (e.node * 3 + qp) * TILE + qs;
                    const cx x = cadd(cadd(acc, ibl), lds_ld(W, w));
                    if (qp4 < 3) lds_st(W, w, x);
                    ibl = x;
                }
            }
            // reset this lane's tap accumulators for the next sweep
            if (qp4 < 3)
                for (int tp = 0; tp < f.n_taps; ++tp) lds_st(T, (tp * 3 + qp) * TILE + qs, mk(0, 0));
            // errmx = max_p |Ib(0,p) - Ibo(p)|  (first element, then strict '>')
            const cx ib0 = lds_ld(W, (1 * 3 + qp) * TILE + qs);
            const cx d = csub(ib0, ibo);
            const double df = hypot(d.re, d.im);
            const double d0 = __shfl(df, gbase + 0, 64), d1 = __shfl(df, gbase + 1, 64),
                         d2 = __shfl(df, gbase + 2, 64);
            double errmx = d0;
            if (d1 > errmx) errmx = d1;
            if (d2 > errmx) errmx = d2;
            ibo = ib0;
            if (qp4 == 0) fl->fin[qs] = errmx < f.eps ? 1 : (it == f.mxitr - 1 ? 2 : 0);
            if (qp4 == 0 && (errmx < f.eps || it == f.mxitr - 1)) {
                if (o.iters) o.iters[s0 + qs] = it + 1;
                if (o.status) o.status[s0 + qs] = errmx < f.eps ? 0 : 1;
            }
        }
        __syncthreads();

        // ---- P2: branch drops
#pragma unroll
        for (int j = 0; j < MAXT; ++j) {
            const int t = tid + j * NT;
            const int s = t % TILE, k = 1 + t / TILE;
            if (t < ntask && s < ns && fl->active[s]) {
                const int wb = k * 3 * TILE + s;
                ib[j][0] = lds_ld(W, wb);
                ib[j][1] = lds_ld(W, wb + TILE);
                ib[j][2] = lds_ld(W, wb + 2 * TILE);
                const double *tz = f.tz + 18 * (size_t)f.node_ops[k].fw;
#pragma unroll
                for (int p = 0; p < 3; ++p) lds_st(W, wb + p * TILE, drop_col(tz, ib[j][0], ib[j][1], ib[j][2], p));
            }
        }
        __syncthreads();

        // ---- S2: forward program
        if (qlane && fl->active[qs]) {
            int prev = -1;
            cx vprev = mk(0, 0);
            const int n = f.n_seq_fw;
            for (int q = 0; q < n; ++q) {
                const SeqFw e = f.seq_fw[q];
                const int dst = e.dst, src = e.src_mask & 0x1FFF, mask = e.src_mask >> 13;
                const cx sv = src == prev ? vprev : lds_ld(W, (src * 3 + qp) * TILE + qs);
                const int w = (dst * 3 + qp) * TILE + qs;
                cx rv = csub(sv, lds_ld(W, w));
                if ((mask >> qp) & 1) rv = mk(0, 0);
                if (qp4 < 3) lds_st(W, w, rv);
                vprev = rv;
                prev = dst;
            }
        }
        __syncthreads();

        // ---- epilogue for scenarios finishing this sweep
        int any_fin = 0;
        for (int s = 0; s < ns; ++s) any_fin |= fl->active[s] && fl->fin[s];
        if (any_fin) {
#pragma unroll
            for (int j = 0; j < MAXT; ++j) {
                const int t = tid + j * NT;
                const int s = t % TILE, k = 1 + t / TILE;
                if (t < ntask && s < ns && fl->active[s] && fl->fin[s]) {
                    const size_t gs = (size_t)s0 + s;
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        const int w = (k * 3 + p) * TILE + s;
                        W[w] = emit_node(o, f.s3, nn, B, k, p, gs, lds_ld(W, w), il[j][p], ib[j][p]);
                    }
                }
            }
            __syncthreads();
            if (qlane && fl->active[qs] && fl->fin[qs]) {
                const int gs = s0 + qs;
                // substation row 0: V0, Ib(0) (= ibo, this sweep's), IL(nn-1) = 0
                const cx v = qp == 0 ? v0[0] : (qp == 1 ? v0[1] : v0[2]);
                OutDev oq = o;
                if (qp4 == 3) oq = OutDev{};   // the shadow lane computes but does not store
                const double2 r0 = emit_node(oq, f.s3, nn, B, 0, qp, (size_t)gs, v, mk(0, 0), ibo);
                const cx sb = cmul(cmul(v, mk(f.s3, 0.0)), cconj(ibo));
                const cx sl = mk(r0.x, 0.0);
                const double mag0 = r0.y;
                // loss: Armadillo accumulate over PQL col 2p (even rows -> acc1, odd -> acc2)
                double acc1 = 0.0 + sl.re, acc2 = 0.0;
                // V_abc_list: first K_p nonzero |V| in row order, zero padded
                double mn = INFINITY, mx = -INFINITY;
                int cnt = 0;
                const int K = qp == 0 ? f.K[0] : (qp == 1 ? f.K[1] : f.K[2]);
                if (mag0 != 0 && cnt < K) { mn = fmin(mn, mag0); mx = fmax(mx, mag0); ++cnt; }
                for (int k = 1; k < nn; ++k) {
                    const cx r = lds_ld(W, (k * 3 + qp) * TILE + qs);
                    if (k & 1) acc2 += r.re; else acc1 += r.re;
                    if (r.im != 0 && cnt < K) { mn = fmin(mn, r.im); mx = fmax(mx, r.im); ++cnt; }
                }
                if (cnt < K) { mn = fmin(mn, 0.0); mx = fmax(mx, 0.0); }
                const double x = sb.re - (acc1 + acc2);
                const double x0 = __shfl(x, gbase + 0, 64), x1 = __shfl(x, gbase + 1, 64), x2 = __shfl(x, gbase + 2, 64);
                const double n0 = __shfl(mn, gbase + 0, 64), n1 = __shfl(mn, gbase + 1, 64), n2 = __shfl(mn, gbase + 2, 64);
                const double m0 = __shfl(mx, gbase + 0, 64), m1 = __shfl(mx, gbase + 1, 64), m2 = __shfl(mx, gbase + 2, 64);
                if (qp4 == 0) {
                    double vmin = n0, vmax = m0;
                    if (n1 < vmin) vmin = n1;
                    if (n2 < vmin) vmin = n2;
                    if (m1 > vmax) vmax = m1;
                    if (m2 > vmax) vmax = m2;
                    if (o.loss) o.loss[gs] = ((0.0 + x0) + x2) + (0.0 + x1);
                    if (o.vmin) o.vmin[gs] = vmin;
                    if (o.vmax) o.vmax[gs] = vmax;
                }
            }
            __syncthreads();
            if (tid < ns && fl->fin[tid]) fl->active[tid] = 0;
            __syncthreads();
        }
        n_active = 0;
        for (int s = 0; s < ns; ++s) n_active += fl->active[s];
    }
}

namespace {
template <int NT>
hipError_t launch_nt(const FeederDev &f, int n_scen, const double *pq, const OutDev &o, int tile, hipStream_t st) {
    const size_t lds = tiled_lds_bytes(f, tile);
    static bool attr_done = false;
    if (!attr_done) {
        hipError_t e = hipFuncSetAttribute((const void *)dpf_tiled_kernel<NT>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_done = true;
    }
    const int grid = (n_scen + tile - 1) / tile;
    hipLaunchKernelGGL(dpf_tiled_kernel<NT>, dim3(grid), dim3(NT), lds, st, f, n_scen, pq, o, tile);
    return hipGetLastError();
}
}  // namespace

size_t tiled_lds_bytes(const FeederDev &f, int tile) {
    return sizeof(double2) * 3 * (size_t)tile * (size_t)(f.nn + f.n_taps) + sizeof(Flags);
}

int tiled_max_tile(const FeederDev &f) {
    const int nb = f.nn - 1;
    // prefer 256-thread workgroups (two per CU fit the VGPR budget), else wider
    int t = std::min(MAX_SEQ_TILE, (256 * MAXT) / nb);
    if (t == 0) t = std::min(MAX_SEQ_TILE, (1024 * MAXT) / nb);
    while (t > 0 && tiled_lds_bytes(f, t) > 160 * 1024) --t;
    return t;
}

hipError_t launch_tiled(const FeederDev &f, int n_scen, const double *pq, const OutDev &o, int tile,
                        hipStream_t st) {
    const int tasks = tile * (f.nn - 1);
    if (tasks <= 256 * MAXT) return launch_nt<256>(f, n_scen, pq, o, tile, st);
    if (tasks <= 512 * MAXT) return launch_nt<512>(f, n_scen, pq, o, tile, st);
    return launch_nt<1024>(f, n_scen, pq, o, tile, st);
}

}  // namespace fpf
