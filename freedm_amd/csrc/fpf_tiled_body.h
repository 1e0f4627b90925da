// fpf_tiled_body.h -- the tiled batched DPF kernel body for gfx950 (well-formed feeders).
//
// One workgroup owns a tile of TILE scenarios for the whole solve; their state
// lives in LDS for all sweeps, so HBM only sees the loads in and the results
// out.  One LDS slot per (node k, phase p, scenario s) -- byte offset
// slot(k)*3*TILE*16 + (p*TILE + s)*16, a complex fp64 -- holds, in turn within a sweep:
//     V(k)  --P1-->  IL(k-1)  --S1-->  Ib(k-1)  --P2-->  drop(k)  --S2-->  V(k)
// The substation's V0 (DPF_return7.cpp:84-96) sits in slot 0 (slots 0..T-1 in
// the multi-track layout), never overwritten.
//
//   P1 (parallel, one task per (s,k), 3 phases per lane):  IL = conj(Sld/V)   :106-130
//   S1 (sequential): the backward program in row order                        :134-160
//      then the substation convergence test                                   :199-210
//   P2 (parallel): drop(k) = lng*(Ib(k-1) . Zl)  (TEMP table, ZGEMM order)    :163-178
//   S2 (sequential): V(dst) = V(src) - drop(dst), phase zeroing               :169-195
//   (a scenario retires after its last sweep; its state stays frozen)
//   epilogue once per tile: Vpolar/PQb/PQL/V to HBM                           :222-253
//      and the VVC reductions (loss, Vmin/Vmax) in the reference's order.
// Every arithmetic step is the reference's operation on the same operands, so V
// is bit-identical to the sequential program (and to the oracle).
//
// The parallel stages carry the divisions and the 3x3 products; the sequential
// stages are 1-2 dependent complex adds per row.  Their lanes are
// (phase p, track t, scenario s), lane = (p*T + t)*NS + s: a Prog with T tracks
// runs T independent chains of the feeder's block tree side by side in one
// instruction stream (fpf_rtc.cpp), NS scenarios per wave, 3*T*NS <= 64.  The
// specialised layout pads the phase and slot strides so those lanes hit
// distinct LDS banks (fpf_api.cpp: bank_layout).  RuntimeProg (T = 1)
// interprets LDS-staged op programs (fpf_internal.h: SeqBw/SeqFw) in chunks of
// SEQ_CHUNK ops, all of a chunk's LDS operands loaded before its dependent adds.
// A lane keeps Sld, IL and Ib of its tasks in VGPRs across the sweep.
#pragma once
#include "fpf_internal.h"
#include "fpf_math.hpp"

#pragma clang fp contract(off)

namespace fpf {

#ifdef FPF_STAMPS
// diagnostic build only: lane 0 of each of the first 64 workgroups records
// s_memtime at every stage boundary (never read by the kernel itself)
__device__ unsigned long long *fpf_stamp_buf = nullptr;
#define STAMP(idx)                                                                                  \
    do {                                                                                            \
        if (fpf_stamp_buf && threadIdx.x == 0 && blockIdx.x < 64 && (idx) < 128)                    \
            fpf_stamp_buf[blockIdx.x * 128 + (idx)] = __builtin_amdgcn_s_memtime();                 \
    } while (0)
#else
#define STAMP(idx) ((void)0)
#endif

namespace {

constexpr int AOT_MAXT = 2;      // tasks per lane of the AOT (interpreted) build
constexpr int MAX_SEQ_TILE = 16; // scenarios per workgroup (flag arrays)
constexpr int U = SEQ_CHUNK;

struct Flags {
    int active[MAX_SEQ_TILE];    // still iterating
    int fin[MAX_SEQ_TILE];       // 1 = converged this sweep, 2 = hit mxitr this sweep
};

__device__ __forceinline__ cx lds_ld(const double2 *w, int i) {
    const double2 v = w[i];
    return mk(v.x, v.y);
}
__device__ __forceinline__ void lds_st(double2 *w, int i, cx v) { w[i] = make_double2(v.re, v.im); }

// Outputs of node k, phase p (DPF_return7.cpp:222-253).  Returns (Re SL, |V|)
// for the ordered VVC reductions.
template <bool EXACT>
__device__ __forceinline__ double2 emit_node(const OutDev &o, double s3, int nn, int B, int k, int p, size_t gs, cx v,
                                             cx ilv, cx ibv) {
    const cx sv = cmul(v, mk(s3, 0.0));
    const cx sb = cmul(sv, cconj(ibv));
    const cx sl = cmul(sv, cconj(ilv));
    // std::abs -> hypot (exact mode); fast mode: sqrt(re^2 + im^2), |V| ~ 1 p.u.
    const double mag = EXACT ? hypot(v.re, v.im) : sqrt(fma(v.re, v.re, v.im * v.im));
    const size_t o6 = ((size_t)(2 * p) * nn + k) * B + gs, o6i = o6 + (size_t)nn * B;
    if (o.vpolar) { o.vpolar[o6] = mag; o.vpolar[o6i] = polar_angle(v, p); }
    if (o.pqb) { o.pqb[o6] = sb.re; o.pqb[o6i] = sb.im; }
    if (o.pql) { o.pql[o6] = sl.re; o.pql[o6i] = sl.im; }
    if (o.v_re) o.v_re[((size_t)p * nn + k) * B + gs] = v.re;
    if (o.v_im) o.v_im[((size_t)p * nn + k) * B + gs] = v.im;
    return make_double2(sl.re, mag);
}

// Sequential stages from the LDS-staged op programs (fpf_internal.h: SeqBw/SeqFw),
// executed in chunks of SEQ_CHUNK ops with all of a chunk's LDS operands
// loaded before its dependent arithmetic.  Layout: slot k = node k, slot nn a
// permanent zero, slot nn+1 a dummy sink, then the tap accumulators.
struct RuntimeProg {
    static constexpr int kTile = 0;
    static constexpr int kNN = 0;
    static constexpr int kTracks = 1;
    static constexpr int kNs = 21;
    static constexpr int kSlots = 0;       // runtime: nn + 2
    static constexpr int kSlotBytes = 0;   // runtime: 3*TILE*16
    static constexpr int kPhaseBytes = 0;  // runtime: TILE*16
    static constexpr bool kKeepIb = true;  // Ib of the last sweep kept for PQb
    static constexpr bool kExact = true;   // the reference's roundings (fpf_opts.exact)
    static constexpr bool kTempLds = false;// TEMP blocks read from global memory
    static constexpr bool kFullK = false;  // general V_abc_list semantics in the epilogue
    static constexpr long kStagger = 0;    // diagnostic: cycles some workgroups wait before starting
    static constexpr int kStaggerShift = 0;
    __device__ static __forceinline__ int node_slot(const FeederDev &, int k) { return k; }
    static constexpr bool kLdsProgram = true;
    static constexpr bool kLdsTaps = true;

    __device__ static __forceinline__ void s1(char *L, uint32_t lane_off, uint32_t, int, int, const SeqBw *pbw,
                                              int nbw) {
        auto at = [&](uint32_t off) -> double2 * { return (double2 *)(L + off); };
        cx ibl = mk(0, 0);
        for (int q0 = 0; q0 < nbw; q0 += U) {
            SeqBw e[U];
            cx vil[U], va[U], vt[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                e[u] = pbw[q0 + u];
                e[u].r = __builtin_amdgcn_readfirstlane(e[u].r);
                e[u].w = __builtin_amdgcn_readfirstlane(e[u].w);
                e[u].a = __builtin_amdgcn_readfirstlane(e[u].a);
                e[u].p = __builtin_amdgcn_readfirstlane(e[u].p);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double2 a = *at(e[u].r + lane_off), b = *at(e[u].a + lane_off),
                              c = *at((e[u].p & ~BW_SEP) + lane_off);
                vil[u] = mk(a.x, a.y);
                va[u] = mk(b.x, b.y);
                vt[u] = mk(c.x, c.y);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const cx x = cadd(cadd(va[u], ibl), vil[u]);
                *at(e[u].w + lane_off) = make_double2(x.re, x.im);
                const cx t = cadd(vt[u], x);
                *at((e[u].p & ~BW_SEP) + lane_off) = make_double2(t.re, t.im);
                ibl = (e[u].p & BW_SEP) ? mk(0, 0) : x;
            }
        }
    }

    __device__ static __forceinline__ void s2(char *L, uint32_t lane_off, uint32_t, int, int qp, const SeqFw *pfw,
                                              int nfw) {
        auto at = [&](uint32_t off) -> double2 * { return (double2 *)(L + off); };
        cx vprev = mk(0, 0);
        for (int q0 = 0; q0 < nfw; q0 += U) {
            SeqFw e[U];
            cx vd[U], vs[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                e[u] = pfw[q0 + u];
                e[u].dst = __builtin_amdgcn_readfirstlane(e[u].dst);
                e[u].src = __builtin_amdgcn_readfirstlane(e[u].src);
                e[u].flags = __builtin_amdgcn_readfirstlane(e[u].flags);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const double2 a = *at(e[u].dst + lane_off), b = *at(e[u].src + lane_off);
                vd[u] = mk(a.x, a.y);
                vs[u] = mk(b.x, b.y);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const cx sv = (e[u].flags & FW_PREV) ? vprev : vs[u];
                cx rv = csub(sv, vd[u]);
                if ((e[u].flags >> qp) & 1) rv = mk(0, 0);
                *at(e[u].dst + lane_off) = make_double2(rv.re, rv.im);
                vprev = rv;
            }
        }
    }
};

}  // namespace

// The kernel body.  Prog supplies the two sequential stages and the LDS layout:
// RuntimeProg runs the LDS-staged op programs (any well-formed feeder); the
// hipRTC path (fpf_rtc.cpp) generates a Prog whose stages are the feeder's
// multi-track schedule as straight-line code with constant LDS offsets and a
// compile-time tile.
template <int NT, int MAXT, class Prog>
__device__ __forceinline__ void tiled_body(const FeederDev &f, int B, const double *__restrict__ pq,
                                           const OutDev &o) {
    extern __shared__ double2 lds[];
    constexpr int NW = NT / 64;
    constexpr int T = Prog::kTracks, NS = Prog::kNs;
    static_assert(3 * T * NS <= 64, "sequential lanes exceed a wave");
    const int TILE = Prog::kTile > 0 ? Prog::kTile : f.tile;
    const int nn = Prog::kNN > 0 ? Prog::kNN : f.nn, nb = nn - 1, nl = f.nl;
    const int nbw = f.n_seq_bw, nfw = f.n_seq_fw;
    const uint32_t slot = Prog::kSlotBytes > 0 ? (uint32_t)Prog::kSlotBytes : 3u * (uint32_t)TILE * 16u;
    const uint32_t psb = Prog::kPhaseBytes > 0 ? (uint32_t)Prog::kPhaseBytes : (uint32_t)TILE * 16u;
    char *const L = (char *)lds;
    const int n_w = Prog::kSlots > 0 ? Prog::kSlots : nn + 2;   // state slots
    const int zero_from = Prog::kSlots > 0 ? Prog::kSlots : nn; // slots >= this start at zero
    const uint32_t w_bytes = (uint32_t)n_w * slot;
    const uint32_t t_bytes = Prog::kLdsTaps ? (uint32_t)(f.n_taps + 2) * slot : 0u;
    Flags *fl = (Flags *)(L + w_bytes + t_bytes);
    // specialised layout: the TEMP blocks (9 complex per branch) staged in LDS after the flags
    const uint32_t temp_base = (w_bytes + t_bytes + (uint32_t)sizeof(Flags) + 15u) & ~15u;
    const bool plds = Prog::kLdsProgram && f.prog_lds;
    SeqBw *pbw = plds ? (SeqBw *)(fl + 1) : (SeqBw *)f.seq_bw;
    SeqFw *pfw = plds ? (SeqFw *)((SeqBw *)(fl + 1) + nbw) : (SeqFw *)f.seq_fw;
    auto at = [&](uint32_t off) -> double2 * { return (double2 *)(L + off); };

    const int tid = threadIdx.x;
    const int s0 = blockIdx.x * TILE;
    const int ns = min(TILE, B - s0);
    const int ntask = TILE * nb;
    const cx v0[3] = {mk(f.V0[0], f.V0[1]), mk(f.V0[2], f.V0[3]), mk(f.V0[4], f.V0[5])};
    STAMP(0);
    if (Prog::kStagger > 0 && ((blockIdx.x >> Prog::kStaggerShift) & 1)) {
        // two resident tiles per CU out of phase: one's sequential stage beside the other's parallel stage
        const long t_go = (long)clock64() + Prog::kStagger;
        while ((long)clock64() < t_go) __builtin_amdgcn_s_sleep(4);
    }

    // ---- init: state slots = V0 (:92-96), zero/dummy slots 0, taps 0, flags, programs
    for (int i = tid; i < n_w * 3 * TILE; i += NT) {
        const int j = i / (3 * TILE), p = (i / TILE) % 3, s = i % TILE;
        const cx v = j >= zero_from ? mk(0, 0) : (p == 0 ? v0[0] : (p == 1 ? v0[1] : v0[2]));
        const double2 w = make_double2(v.re, v.im);
        *(double2 *)(L + (uint32_t)j * slot + (uint32_t)p * psb + (uint32_t)s * 16u) = w;
    }
    if (Prog::kLdsTaps)
        for (int i = tid; i < (f.n_taps + 2) * 3 * TILE; i += NT) lds_st((double2 *)(L + w_bytes), i, mk(0, 0));
    if (plds) {
        for (int i = tid; i < nbw; i += NT) pbw[i] = f.seq_bw[i];
        for (int i = tid; i < nfw; i += NT) pfw[i] = f.seq_fw[i];
    }
    if (tid < MAX_SEQ_TILE) {
        fl->active[tid] = tid < ns ? 1 : 0;
        fl->fin[tid] = 0;
    }
    if (Prog::kTempLds)
        for (int i = tid; i < f.n_fw * 9; i += NT) *(double2 *)(L + temp_base + 16u * (uint32_t)i) = ld_global2(f.tz, i);

    // ---- per-task constants: LDS offset, TEMP block, Sld = (P + jQ)/(bkva/3) (:46-50)
    cx sld[MAXT][3], il[MAXT][3], ib[MAXT][3];
    const double *tz[MAXT];
    uint32_t toff[MAXT];                             // LDS offset of the task's TEMP block (kTempLds)
    uint32_t woff[MAXT];
    int tsc[MAXT];                                   // scenario of the task, -1 = none
    unsigned rr_ok = 0;                              // bit j: task j's Sld in dv_in_range
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
        const int t = tid + j * NT;
        const int s = t % TILE, k = 1 + t / TILE;
        tz[j] = f.tz;
        toff[j] = temp_base;
        woff[j] = 0;
        tsc[j] = -1;
        if (t < ntask && s < ns) {
            const NodeOp nd = f.node_ops[k];
            tz[j] = f.tz + 18 * (size_t)nd.fw;
            toff[j] = temp_base + 144u * (uint32_t)nd.fw;
            woff[j] = (uint32_t)nd.slot * slot + (uint32_t)s * 16u;
            tsc[j] = s;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const cx sl = mk(pq[((size_t)(2 * p) * nl + nd.row) * B + s0 + s],
                                 pq[((size_t)(2 * p + 1) * nl + nd.row) * B + s0 + s]);
                sld[j][p] = cdiv(sl, mk(f.s3, 0.0));
            }
            bool ok = true;
#pragma unroll
            for (int p = 0; p < 3; ++p) ok = ok && dv_in_range(sld[j][p].re) && dv_in_range(sld[j][p].im);
            rr_ok |= (ok ? 1u : 0u) << j;
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) { il[j][p] = mk(0, 0); ib[j][p] = mk(0, 0); }
    }

    // sequential lanes (track qt, phase qp, scenario qs): NS scenarios per wave,
    // scenario s on wave s / NS; the stages are latency-bound chains, so a tile
    // uses as few waves as hold it
    const int NWS = (TILE + NS - 1) / NS < NW ? (TILE + NS - 1) / NS : NW;
    const int wv = tid >> 6, ln = tid & 63;
    const int qp = ln / (T * NS), qt = (ln / NS) % T, qsl = ln % NS;
    const int qs = wv * NS + qsl;
    const bool qlane = wv < NWS && ln < 3 * T * NS && qs < ns;
    const bool qlead = qlane && qt == 0;               // one chain per (scenario, phase) does the tests
    const int gbase = qt * NS + qsl;                   // lane of phase 0 of this (track, scenario)
    const uint32_t lane_off = qlane ? (uint32_t)qp * psb + (uint32_t)qs * 16u : 0u;
    const uint32_t vbase = lane_off + (uint32_t)qt * slot;
    const uint32_t n1_off = (uint32_t)f.node_ops[1].slot * slot;   // Ib(0) lives in node 1's slot
    cx ibo = mk(0, 0);
    __syncthreads();
    STAMP(1);

    int n_active = ns;
    for (int it = 0; it < f.mxitr && n_active > 0; ++it) {
        // ---- P1: load currents
#pragma unroll
        for (int j = 0; j < MAXT; ++j) {
            if (tsc[j] >= 0 && fl->active[tsc[j]]) {
                double2 *w[3];
                cx v[3];
                bool rr = (rr_ok >> j) & 1;
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    w[p] = at(woff[j] + p * psb);
                    v[p] = mk(w[p]->x, w[p]->y);
                    if (Prog::kExact) rr = rr && dv_in_range(v[p].re) && dv_in_range(v[p].im);
                }
                if (!Prog::kExact) {
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        il[j][p] = load_current_fast(sld[j][p], v[p]);
                        __builtin_amdgcn_sched_barrier(0);   // phase by phase: registers
                    }
                } else if (rr) {   // the shared-reciprocal division (same bits as the reference's)
#pragma unroll
                    for (int p = 0; p < 3; ++p) il[j][p] = load_current_rr(sld[j][p], v[p]);
                } else {
#pragma unroll
                    for (int p = 0; p < 3; ++p) il[j][p] = load_current(sld[j][p], v[p]);
                }
#pragma unroll
                for (int p = 0; p < 3; ++p) *w[p] = make_double2(il[j][p].re, il[j][p].im);
            }
            // one task at a time: interleaving both tasks' divisions costs more
            // registers than the 128 a 1024-thread workgroup has
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        STAMP(2 + it * 5);

        // ---- S1: backward program + convergence
        if (qlane && fl->active[qs]) {
            Prog::s1(L, lane_off, vbase, qt, qp, pbw, nbw);
            // reset this lane's tap accumulators for the next sweep
            if (Prog::kLdsTaps)
                for (int tp = 0; tp < f.n_taps; ++tp) *at(w_bytes + tp * slot + lane_off) = make_double2(0, 0);
            // errmx = max_p |Ib(0,p) - Ibo(p)|  (first element, then strict '>')
            const double2 b0 = *at(n1_off + lane_off);
            const cx ib0 = mk(b0.x, b0.y);
            const cx d = csub(ib0, ibo);
            const double df = hypot(d.re, d.im);
            const double d0 = __shfl(df, gbase + 0 * T * NS, 64), d1 = __shfl(df, gbase + 1 * T * NS, 64),
                         d2 = __shfl(df, gbase + 2 * T * NS, 64);
            double errmx = d0;
            if (d1 > errmx) errmx = d1;
            if (d2 > errmx) errmx = d2;
            ibo = ib0;
            if (qlead && qp == 0) {
                fl->fin[qs] = errmx < f.eps ? 1 : (it == f.mxitr - 1 ? 2 : 0);
                if (errmx < f.eps || it == f.mxitr - 1) {
                    if (o.iters) o.iters[s0 + qs] = it + 1;
                    if (o.status) o.status[s0 + qs] = errmx < f.eps ? 0 : 1;
                    if (o.errmx) o.errmx[s0 + qs] = errmx;
                    if (o.guard) o.guard[s0 + qs] = 0;   // exact kernel: no guard band
                }
            }
        }
        __syncthreads();
        STAMP(3 + it * 5);

        // ---- P2: branch drops
#pragma unroll
        for (int j = 0; j < MAXT; ++j) {
            if (tsc[j] >= 0 && fl->active[tsc[j]]) {
                double2 *w0 = at(woff[j]), *w1 = at(woff[j] + psb), *w2 = at(woff[j] + 2 * psb);
                const cx b0 = mk(w0->x, w0->y), b1 = mk(w1->x, w1->y), b2 = mk(w2->x, w2->y);
                if (Prog::kKeepIb) {
                    ib[j][0] = b0;
                    ib[j][1] = b1;
                    ib[j][2] = b2;
                }
                if (Prog::kTempLds) {
                    // column by column from the LDS TEMP table: 3 TEMP values live at a time
                    const double2 *tl = (const double2 *)(L + toff[j]);
                    double2 *wa[3] = {w0, w1, w2};
#pragma unroll
                    for (int a = 0; a < 3; ++a) {
                        cx tc[9];
#pragma unroll
                        for (int l = 0; l < 3; ++l) tc[l * 3 + a] = lds_ld(tl, l * 3 + a);
                        const cx d = Prog::kExact ? drop_col_r(tc, b0, b1, b2, a) : drop_col_fma(tc, b0, b1, b2, a);
                        *wa[a] = make_double2(d.re, d.im);
                    }
                } else {
                    cx tm[9];
                    load_temp(tz[j], tm);
                    const cx d0 = Prog::kExact ? drop_col_r(tm, b0, b1, b2, 0) : drop_col_fma(tm, b0, b1, b2, 0);
                    const cx d1 = Prog::kExact ? drop_col_r(tm, b0, b1, b2, 1) : drop_col_fma(tm, b0, b1, b2, 1);
                    const cx d2 = Prog::kExact ? drop_col_r(tm, b0, b1, b2, 2) : drop_col_fma(tm, b0, b1, b2, 2);
                    *w0 = make_double2(d0.re, d0.im);
                    *w1 = make_double2(d1.re, d1.im);
                    *w2 = make_double2(d2.re, d2.im);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();
        STAMP(4 + it * 5);

        // ---- S2: forward program; a scenario whose last sweep this was retires
        // (its state -- V in LDS, IL/Ib in the task registers, Ib(0) in ibo -- is
        // then frozen until the epilogue)
        if (qlane && fl->active[qs]) {
            Prog::s2(L, lane_off, vbase, qt, qp, pfw, nfw);
            // every lane of the scenario is on this wave and past s2 here
            if (qlead && qp == 0 && fl->fin[qs]) fl->active[qs] = 0;
        }
        __syncthreads();
        STAMP(5 + it * 5);
        n_active = 0;
        for (int s = 0; s < ns; ++s) n_active += fl->active[s];
    }
    STAMP(126);

    // ---- epilogue, once per tile: outputs of every (scenario, node, phase)
#pragma unroll
    for (int j = 0; j < MAXT; ++j) {
        const int s = tsc[j];
        if (s >= 0) {
            const int k = 1 + (tid + j * NT) / TILE;
            const size_t gs = (size_t)s0 + s;
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                double2 *w = at(woff[j] + p * psb);
                *w = emit_node<Prog::kExact>(o, f.s3, nn, B, k, p, gs, mk(w->x, w->y), il[j][p],
                                             Prog::kKeepIb ? ib[j][p] : mk(0, 0));   // !kKeepIb: no PQb requested
            }
        }
    }
    __syncthreads();
    STAMP(125);
    // ---- per-scenario reductions: loss (VoltVarCtrl.cpp:1152-1161), Vmin/Vmax
    // (V_abc_list.cpp:7-81, VoltVarCtrl.cpp:1201-1207).  Row k's (Re SL, |V|) sits
    // in node k's slot; lane (phase, track, scenario) of the sequential layout.
    if (qlane) {
        const int gs = s0 + qs;
        const cx v = qp == 0 ? v0[0] : (qp == 1 ? v0[1] : v0[2]);
        const cx sb = cmul(cmul(v, mk(f.s3, 0.0)), cconj(ibo));
        // substation row 0: V0, Ib(0) (= ibo, the last sweep's), IL(nn-1) = 0
        double2 r0 = make_double2(0.0, 0.0);
        if (qt == 0) r0 = emit_node<Prog::kExact>(o, f.s3, nn, B, 0, qp, (size_t)gs, v, mk(0, 0), ibo);
        auto row = [&](int k) -> double2 { return *at((uint32_t)Prog::node_slot(f, k) * slot + lane_off); };
        double acc1 = 0.0, acc2 = 0.0, mn = INFINITY, mx = -INFINITY;
        if (Prog::kFullK) {
            // every K_p = nn: V_abc_list keeps every row, so the extremes are plain
            // min/max over all rows (exact in any order): rows k = t (mod T) per track.
            // The loss keeps Armadillo's accumulate order: acc1 = even rows, acc2 = odd
            // rows, each one sequential chain (tracks 0 and 1 when T > 1).
            constexpr int TL2 = T > 1 ? 1 : 0;
            if (qt == 0) {
                acc1 = 0.0 + r0.x;
#pragma unroll
                for (int k = 2; k < (Prog::kNN > 0 ? Prog::kNN : 1 << 30) && k < nn; k += 2) acc1 += row(k).x;
            }
            if (qt == TL2) {
#pragma unroll
                for (int k = 1; k < (Prog::kNN > 0 ? Prog::kNN : 1 << 30) && k < nn; k += 2) acc2 += row(k).x;
            }
            if (qt == 0) { mn = r0.y; mx = r0.y; }
#pragma unroll
            for (int k0 = T; k0 < (Prog::kNN > 0 ? Prog::kNN : 1 << 30) + T && k0 < nn + T; k0 += T) {
                const int k = k0 - T + qt;
                if (k >= 1 && k < nn) {
                    const double m = row(k).y;
                    mn = fmin(mn, m);
                    mx = fmax(mx, m);
                }
            }
#pragma unroll
            for (int t = 1; t < T; ++t) {
                const double a = __shfl(mn, (qp * T + t) * NS + qsl, 64), b = __shfl(mx, (qp * T + t) * NS + qsl, 64);
                mn = fmin(mn, a);
                mx = fmax(mx, b);
            }
            if (T > 1) acc2 = __shfl(acc2, (qp * T + TL2) * NS + qsl, 64);
        } else if (qt == 0) {
            // general V_abc_list: the first K_p nonzero |V| in row order, zero padded
            acc1 = 0.0 + r0.x;
            int cnt = 0;
            const int K = qp == 0 ? f.K[0] : (qp == 1 ? f.K[1] : f.K[2]);
            if (r0.y != 0 && cnt < K) { mn = fmin(mn, r0.y); mx = fmax(mx, r0.y); ++cnt; }
            // rows 1..nn-1 in order; operands loaded 8 at a time ahead of the ordered adds
            for (int k0 = 1; k0 < nn; k0 += 8) {
                double2 r[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) r[u] = k0 + u < nn ? row(k0 + u) : make_double2(0, 0);
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    if (k0 + u < nn) {
                        if ((k0 + u) & 1) acc2 += r[u].x; else acc1 += r[u].x;
                        if (r[u].y != 0 && cnt < K) { mn = fmin(mn, r[u].y); mx = fmax(mx, r[u].y); ++cnt; }
                    }
                }
            }
            if (cnt < K) { mn = fmin(mn, 0.0); mx = fmax(mx, 0.0); }
        }
        const double x = sb.re - (acc1 + acc2);
        const double x0 = __shfl(x, gbase + 0 * T * NS, 64), x1 = __shfl(x, gbase + 1 * T * NS, 64),
                     x2 = __shfl(x, gbase + 2 * T * NS, 64);
        const double n0 = __shfl(mn, gbase + 0 * T * NS, 64), n1 = __shfl(mn, gbase + 1 * T * NS, 64),
                     n2 = __shfl(mn, gbase + 2 * T * NS, 64);
        const double m0 = __shfl(mx, gbase + 0 * T * NS, 64), m1 = __shfl(mx, gbase + 1 * T * NS, 64),
                     m2 = __shfl(mx, gbase + 2 * T * NS, 64);
        if (qlead && qp == 0) {
            double vmin = n0, vmax = m0;
            if (n1 < vmin) vmin = n1;
            if (n2 < vmin) vmin = n2;
            if (m1 > vmax) vmax = m1;
            if (m2 > vmax) vmax = m2;
            const double loss = ((0.0 + x0) + x2) + (0.0 + x1);
            if (o.loss) o.loss[gs] = loss;
            if (o.vmin) o.vmin[gs] = vmin;
            if (o.vmax) o.vmax[gs] = vmax;
            if (o.agg) {   // this scenario's row of the tile aggregate
                double *ra = (double *)(L + temp_base) + 8 * qs;   // TEMP blocks are dead now
                ra[0] = loss;
                ra[1] = vmin;
                ra[2] = vmax;
                ra[3] = o.status ? (double)o.status[gs] : 0.0;
            }
        }
    }
    if (o.agg) {
        // ---- fused batch aggregate [loss_sum, vmin, vmax, n_conv, n_nonconv, n_over,
        // n_under, n_scen] over converged scenarios.  The tile's partials (scenario
        // order) are published with write-through (sc1) stores; one agent-scope
        // ticket per tile; the tile that arrives last sums the partials in tile
        // order (a fixed tree: deterministic) -- the hand-off form of
        // MI355X_MICROARCH.md "Valid forms", row 1 of the sc1 table.
        __syncthreads();
        if (tid == 0) {
            double ls = 0, mn = INFINITY, mx = -INFINITY, nc = 0, nnc = 0, no = 0, nu = 0;
            const double *ra = (const double *)(L + temp_base);
            for (int s = 0; s < ns; ++s) {
                const double *r = ra + 8 * s;
                if (r[3] == 0.0) {
                    ls += r[0];
                    mn = fmin(mn, r[1]);
                    mx = fmax(mx, r[2]);
                    nc += 1;
                    if (r[2] > f.ub_v) no += 1;
                    if (r[1] < f.lb_v) nu += 1;
                } else {
                    nnc += 1;
                }
            }
            const double part[8] = {ls, mn, mx, nc, nnc, no, nu, (double)ns};
            double *dst = o.partials + 8 * (size_t)blockIdx.x;
            for (int q = 0; q < 8; ++q) __hip_atomic_store(dst + q, part[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned t = __hip_atomic_fetch_add(o.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            fl->active[0] = t == gridDim.x - 1;   // flags are dead: tell the workgroup
        }
        __syncthreads();
        if (fl->active[0]) {
            // the last tile: thread i folds tiles i, i + NT, ... in order, then a fixed
            // tree over the threads in the (dead) state region of LDS
            // R threads (power of two) whose 8 x R doubles fit below the flags
            int R = NT;
            while (R > 1 && (uint32_t)R * 64u > w_bytes) R >>= 1;
            double a[8] = {0, INFINITY, -INFINITY, 0, 0, 0, 0, 0};
            for (unsigned b = tid; tid < R && b < gridDim.x; b += R) {
                double r[8];
#pragma unroll
                for (int q = 0; q < 8; ++q)
                    r[q] = __hip_atomic_load(o.partials + 8 * (size_t)b + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                a[0] += r[0];
                a[1] = fmin(a[1], r[1]);
                a[2] = fmax(a[2], r[2]);
#pragma unroll
                for (int q = 3; q < 8; ++q) a[q] += r[q];
            }
            double *sh = (double *)L;   // [8][R]
            if (tid < R) {
#pragma unroll
                for (int q = 0; q < 8; ++q) sh[q * R + tid] = a[q];
            }
            __syncthreads();
            for (int w = R / 2; w > 0; w >>= 1) {
                if (tid < w) {
                    sh[0 * R + tid] += sh[0 * R + tid + w];
                    sh[1 * R + tid] = fmin(sh[1 * R + tid], sh[1 * R + tid + w]);
                    sh[2 * R + tid] = fmax(sh[2 * R + tid], sh[2 * R + tid + w]);
#pragma unroll
                    for (int q = 3; q < 8; ++q) sh[q * R + tid] += sh[q * R + tid + w];
                }
                __syncthreads();
            }
            if (tid < 8) o.agg[tid] = sh[tid * R];
            if (tid == 0) __hip_atomic_store(o.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    STAMP(127);
}


}  // namespace fpf
