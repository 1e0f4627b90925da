// fpf_wblk_body.h -- the wave-block kernel's device code (dpf_wblk_kernel),
// included by fpf_wblk.hip and embedded for hipRTC (fpf_rtc.cpp: the per-plan
// specialised build, FPF_WSPEC).  See fpf_wblk.hip for the design.
#pragma once
#include "fpf_internal.h"
#include "fpf_math.hpp"
#include "fpf_wave_common.h"

namespace fpf {

// diagnostic ablation builds (tools/build_ablations.sh wblk <bits>): results are
// wrong when set.  1: every workgroup stages column s & 15 (L2-resident loads);
// 2: no V write-out; 4: stop after staging; 8: no barrier after the X stores (2 of 5 per sweep).  Compiled out of the product.
#ifdef FPF_WBLK_ABL
#define WABL(bit) (FPF_WBLK_ABL & (bit))
#else
#define WABL(bit) 0
#endif
// diagnostic build without the convergence guard's code (FPF_WBLK_NO_GUARD_CODE)
#ifdef FPF_WBLK_NO_GUARD_CODE
constexpr bool GUARD_CODE = false;
#else
constexpr bool GUARD_CODE = true;
#endif

#if defined(FPF_STAMPS) && !defined(FPF_WSPEC)
// diagnostic build only (tools/wblk_stamps.py): thread 0 of each of 64 workgroups
// from fpf_wblk_stamp_base on records s_memtime at stage boundaries, [64][128]:
// 0 entry, 1 staged (after the barrier), 4 + 8 it + k in sweep it < 14 (k = 0 top,
// 1 backward scan + wave totals, 2 Ib gathered, 3 drops, 4 forward scan + wave
// totals, 5 block offsets, 6 V), 120 after the loop, 121 extremes, 122 results,
// 123 V written
__device__ unsigned long long *fpf_wblk_stamp_buf = nullptr;
__device__ unsigned fpf_wblk_stamp_base = 0;
#define BSTAMP(idx)                                                                                    \
    do {                                                                                               \
        const unsigned w_ = blockIdx.x - fpf_wblk_stamp_base;                                          \
        if (fpf_wblk_stamp_buf && threadIdx.x == 0 && w_ < 64u && (idx) < 128)                         \
            fpf_wblk_stamp_buf[w_ * 128 + (idx)] = __builtin_amdgcn_s_memtime();                        \
    } while (0)
extern "C" int fpf_debug_set_wblk_stamp_buffer(void *dptr, unsigned base) {
    unsigned long long *p = (unsigned long long *)dptr;
    if (hipMemcpyToSymbol(HIP_SYMBOL(fpf_wblk_stamp_base), &base, sizeof(base)) != hipSuccess) return -3;
    return hipMemcpyToSymbol(HIP_SYMBOL(fpf_wblk_stamp_buf), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#define BSTAMP_IT(k) BSTAMP(it < 14 ? 4 + 8 * it + (k) : 999)
#else
#define BSTAMP(idx) ((void)0)
#define BSTAMP_IT(k) ((void)0)
#endif

namespace {
constexpr int WB_C = 4;   // slots per lane
constexpr int WB_BD = 6;  // block-chain depth resolved from registers (deeper: the LDS loop)

}  // namespace

// GX (the full variant's general paths, as the wave kernel's): bit 0 zeroed
// phases (has_mask / has_rel, SEG), bit 1 the sequential-order plan (has_lag)
template <int W, bool FULL, int C, bool SEG, int GX = FULL ? 1 : 0>
__global__ __launch_bounds__(W * 64, C >= 8 ? 1 : (C <= 2 ? 4 : 2)) void dpf_wblk_kernel(WaveDev f, int B, const double *__restrict__ pq,
                                                             OutDev o) {
    constexpr bool FM = FULL && (GX & 1), FLG = FULL && (GX & 2), FG = FM || FLG;
    // the full outputs of the lean variant (GX 0) formed after the sweep loop from
    // IL / Ib stashed in the last sweep (no VGPR spills); the general variants emit
    // in the last sweep as before (stashing measured slower there: 1.63 -> 1.93 ms,
    // and faulted in the segmented one)
    constexpr bool STASH = FULL && GX == 0 && !SEG;
#ifdef FPF_WSPEC
    // the per-plan hipRTC build (fpf_rtc.cpp: wblk_rtc_source): the plan's
    // uniform values as constants; the host checks they match
    f.nn = FPF_WSPEC_NN;
    f.nl = FPF_WSPEC_NL;
    f.nblk = FPF_WSPEC_NBLK;
    f.bdepth = FPF_WSPEC_BDEPTH;
    f.ncomp = FPF_WSPEC_NCOMP;
    f.temp_sym = FPF_WSPEC_TEMP_SYM;
    f.has_mask = FPF_WSPEC_HAS_MASK;
    f.has_rel = FPF_WSPEC_HAS_REL;
    f.mxitr = FPF_WSPEC_MXITR;
    f.ncode = FPF_WSPEC_NCODE;
#endif
    constexpr int L = 64 * W, NT = 64 * W;
    extern __shared__ double2 lds[];
    if (o.skip && *o.skip) return;   // (the multi-area solve's device-side stop)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    BSTAMP(0);
    const int s = xcd_tile(blockIdx.x, gridDim.x);   // this workgroup's scenario
    const int nblk = f.nblk, nn = f.nn, nl = f.nl, bdepth = f.bdepth, XC = f.ncomp + 1;
    const int ntz = f.temp_sym ? 4 : 9, PS = nl + 1;
    // LDS: Zl per code | Sld [3][Nl + 1] (row Nl = 0 for empty slots; node k's V
    // over row k - 1 in the last sweep) | X [3][XC] gathered scan values (entry
    // XC - 1 = 0) | block offsets [3][nblk] | V0 [3] (+1 pad) | wave totals
    // [2][W][8] (backward, forward; entries 6, 7: loss, Vmin, Vmax) | block chains
    double2 *const zc = lds;
    double2 *const stg = zc + f.ncode * ntz;
    double2 *const X = stg + 3 * PS;
    double2 *const OFF = X + 3 * XC;
    double2 *const OFFA = OFF + 3 * nblk;   // [3][nblk] off(b) itself (has_rel only)
    double2 *const V0S = OFF + 3 * nblk * (f.has_rel ? 2 : 1);
    const int NLAG = FLG ? f.nlag : 0;              // (the sequential-order plan: V_prev entries)
    double2 *const LAGV = V0S + 4;                   // [3][nlag]
    double *const wtb = (double *)(V0S + 4 + 3 * NLAG);
    double *const wtf = wtb + 8 * W;
    double *const vx = wtf + 8 * W;             // [3][2] per-phase Vmin / Vmax (zeroed phases)
    int *const pairs = (int *)(vx + 8);         // [bdepth][2][nblk]

    // ---- the scenario's loads P/Q [6][Nl] (column s of pq, or its contiguous
    // block in the scenario-major layout) into Sld scaled by 1/(bkva/3)
    // (DPF_return7.cpp:46-50), all of a thread's loads in flight
    {
        const double inv_s3 = 1.0 / f.s3;
        double *const sd = (double *)stg;
        const int total = 6 * nl;
        constexpr int U = 8, U2 = 16;   // U2: every 16-byte load of a thread in flight (2048 buses: 13 per thread)
        if (o.smaj) {
            // one contiguous block of 6 Nl doubles (16-byte aligned: 6 Nl is even)
            typedef double d2v __attribute__((ext_vector_type(2)));
            const d2v *src = (const d2v *)(pq + (WABL(1) ? (size_t)(s & 15) : (size_t)s) * total);
            const int total2 = total / 2;
            // element e = 2 i: (field, row) walked 2 NT elements per load
            RowWalk w;
            w.init(2 * tid, 2 * NT, nl);
            for (int i0 = 0; i0 < total2; i0 += U2 * NT) {
                d2v r[U2];
                int q0[U2], q1[U2];
#pragma unroll
                for (int u = 0; u < U2; ++u) {
                    const int i = i0 + u * NT + tid;
                    r[u] = __builtin_nontemporal_load(src + (i < total2 ? i : 0));
                    q0[u] = 2 * ((w.fq >> 1) * PS + w.rr) + (w.fq & 1);
                    const int f1 = w.rr + 1 < nl ? w.fq : w.fq + 1, r1 = w.rr + 1 < nl ? w.rr + 1 : 0;
                    q1[u] = 2 * ((f1 >> 1) * PS + r1) + (f1 & 1);
                    w.next();
                }
#pragma unroll
                for (int u = 0; u < U2; ++u) {
                    const int i = i0 + u * NT + tid;
                    if (i < total2) {
                        sd[q0[u]] = r[u].x * inv_s3;
                        sd[q1[u]] = r[u].y * inv_s3;
                    }
                }
            }
        } else {
            RowWalk w;   // (field, row) of element i, walked NT per load
            w.init(tid, NT, nl);
            for (int i0 = 0; i0 < total; i0 += U * NT) {
                double r[U];
                int q[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = i0 + u * NT + tid;
                    r[u] = pq[(size_t)(i < total ? i : 0) * B + (WABL(1) ? (s & 15) : s)];
                    q[u] = 2 * ((w.fq >> 1) * PS + w.rr) + (w.fq & 1);
                    w.next();
                }
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int i = i0 + u * NT + tid;
                    if (i < total) sd[q[u]] = r[u] * inv_s3;
                }
            }
        }
        for (int i = tid; i < f.ncode * ntz; i += NT) zc[i] = ld_global2(f.code_z, i);
        for (int i = tid; i < 2 * bdepth * nblk; i += NT) pairs[i] = f.blk_pairs[i];
        if (tid < 3) {
            stg[tid * PS + nl] = make_double2(0.0, 0.0);
            X[tid * XC + XC - 1] = make_double2(0.0, 0.0);
            // the source voltage: V0 (:84-89), or this scenario's (an area of the
            // multi-area solve, fed from its boundary bus)
            double2 v0 = tid == 0 ? make_double2(f.V0[0], f.V0[1])
                                  : (tid == 1 ? make_double2(f.V0[2], f.V0[3]) : make_double2(f.V0[4], f.V0[5]));
            if (o.vsrc) v0 = make_double2(o.vsrc[(size_t)(2 * tid) * B + s], o.vsrc[(size_t)(2 * tid + 1) * B + s]);
            V0S[tid] = v0;
        }
    }
    // this thread's block chain (thread b < nblk resolves block b): the (tap,
    // first - 1) index pairs, packed two per register, so that all of a chain's X
    // reads issue together every sweep instead of one dependent pair per level
    const bool chain_regs = bdepth <= WB_BD && nblk <= NT && XC < 65536;
    // one (block, phase) per thread where the workgroup has 3 nblk threads (thread
    // t: block t % nblk, phase t / nblk): a third of the chain reads and adds per
    // thread, on every wave instead of the first nblk / 64 (round 5: the block
    // offsets were 28 % of a config-3 sweep with one block per thread, 3 phases each)
    // (the per-plan builds only: in the static build, with the plan's values at
    // run time, the second chain form spilled 118 VGPRs of the light variant)
#if defined(FPF_WAVE_WBLK_NO_OFF3)
    const bool off3 = false;   // (experiment: the per-plan build with one block per thread)
#elif defined(FPF_WSPEC) || defined(FPF_WBLK_OFF3_STATIC)
    const bool off3 = chain_regs && 3 * nblk <= NT;
#else
    // (the general full variants keep it -- zeroed phases 1.65 vs 1.78 ms, 2048-bus x
    // 2048 -- but not the segmented one, which faulted with it on the 2048-bus table)
    const bool off3 = FULL && GX != 0 && !SEG && chain_regs && 3 * nblk <= NT;
#endif
    const int op3 = off3 ? tid / nblk : 0, ob3 = off3 ? tid - op3 * nblk : tid;
    int bp[WB_BD];
#pragma unroll
    for (int j = 0; j < WB_BD; ++j) {
        const bool ok = chain_regs && j < bdepth && (off3 ? tid < 3 * nblk : tid < nblk);
        bp[j] = ok ? f.blk_pairs[(2 * j) * nblk + ob3] | (f.blk_pairs[(2 * j + 1) * nblk + ob3] << 16)
                   : (XC - 1) | ((XC - 1) << 16);
    }
    int si[C], sb[C], bk[C], cz[C];
    double lg[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const int r = f.slot_row[c * L + tid];
        sb[c] = r < 0 ? nl : r;
        si[c] = f.slot_info[c * L + tid];
        bk[c] = f.slot_blk[c * L + tid];
        cz[c] = f.slot_code[c * L + tid] * ntz;
        lg[c] = f.slot_lng[c * L + tid];
    }
    __syncthreads();
    BSTAMP(1);
    if (WABL(4)) return;

    // flat start (V = V0 on every node, DPF_return7.cpp:92-96, the feeder's own
    // source): the first sweep's load currents use the uniform 1/|V0_p|^2 and take
    // the guard record's sum from their Sld reads
    const bool flat = !o.vsrc && !o.vinit_re;
    // the guard record: sum_k |S_k|_1 of the scenario (wtb[7], read after the loop;
    // Sld is overwritten by V in the last sweep)
    if (GUARD_CODE && o.flag_count && !flat) {
        double a = 0.0;
#pragma unroll
        for (int c = 0; c < C; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const cx x = ldx(stg, p * PS + sb[c]);
                a += fabs(x.re) + fabs(x.im);
            }
        a = seg_incl<64>(a);
        if (lane == 63) wtb[8 * wv + 7] = a;
    }
    cx v[C][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const cx v0 = ldx(V0S, p);
#pragma unroll
        for (int c = 0; c < C; ++c) v[c][p] = v0;   // V(0..Nl-1) = V0  (:92-96)
    }
    if (o.vinit_re) {
        // the multi-area solve's warm start: node k of each slot from the given V
#pragma unroll
        for (int c = 0; c < C; ++c)
            if (si_valid(si[c])) {
                const int k = f.slot_node[c * L + tid];
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    v[c][p] = mk(o.vinit_re[((size_t)p * nn + k) * B + s], o.vinit_im[((size_t)p * nn + k) * B + s]);
            }
    }
    cx ibo[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
    int it = 0;
    bool conv = false;
    double dmin = INFINITY;  // closest |err2 - eps^2| of a decision in the guard's coarse band
    double err2_last = 0.0;
    for (;; ++it) {
        if (FLG && f.has_lag) {
            // (the sequential-order plan, fpf_api.cpp: analyse_wave_lag) the sources
            // read before their own rows see the previous sweep's V, stored here
            // before this sweep updates it (read after the barriers below)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int lg = (f.slot_lagx[c * L + tid] >> 18) - 1;
                if (lg >= 0) {
#pragma unroll
                    for (int p = 0; p < 3; ++p) stx(LAGV, p * NLAG + lg, v[c][p]);
                }
            }
        }
        BSTAMP_IT(0);
        // ---- load currents (:106-130)
        cx il[C][3], ib[C][3];
        if (flat && it == 0) {
            // IL = conj(S/V0) = conj(S) V0 / |V0|^2 (V0 != 0)
            double a = 0.0;
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    const cx x = ldx(stg, p * PS + sb[c]);
                    const double vr = f.V0[2 * p], vi = f.V0[2 * p + 1], r0 = f.rv0[p];
                    il[c][p] = mk(fma(x.re, vr, x.im * vi) * r0, fma(x.re, vi, -(x.im * vr)) * r0);
                    a += fabs(x.re) + fabs(x.im);
                }
            if (GUARD_CODE && o.flag_count) {
                a = seg_incl<64>(a);
                if (lane == 63) wtb[8 * wv + 7] = a;
            }
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
                for (int p = 0; p < 3; ++p) il[c][p] = il_fast<FM>(ldx(stg, p * PS + sb[c]), v[c][p]);   // 0 on a zeroed phase
        }

        // ---- backward sweep (:134-160): Ib = subtree sums via the prefix scan E of
        // IL: lane-local prefix, wavefront scan, the totals of the waves before
        double sc6[6], pre[6], tot6[6];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            cx acc = il[0][p];
            ib[0][p] = acc;
#pragma unroll
            for (int c = 1; c < C; ++c) { acc = cadd(acc, il[c][p]); ib[c][p] = acc; }
            sc6[2 * p] = acc.re;
            sc6[2 * p + 1] = acc.im;
        }
        seg_incl_n<64>(sc6);
        if (lane == 63) {
#pragma unroll
            for (int q = 0; q < 6; ++q) wtb[8 * wv + q] = sc6[q];
        }
        __syncthreads();
        BSTAMP_IT(1);
        wave_prefix<W, true>(wtb, wv, lane, pre, tot6);
        cx tot[3], exl[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const cx inc = mk(pre[2 * p] + sc6[2 * p], pre[2 * p + 1] + sc6[2 * p + 1]);
            tot[p] = mk(tot6[2 * p], tot6[2 * p + 1]);   // Ib(0): every wave sums the same totals in the same order
            exl[p] = csub(inc, ib[C - 1][p]);              // the lane's exclusive prefix
#pragma unroll
            for (int c = 0; c < C; ++c) ib[c][p] = cadd(exl[p], ib[c][p]);   // Einc at this slot
        }
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const int ci = si_store_b(si[c]);
            if (ci >= 0) {
#pragma unroll
                for (int p = 0; p < 3; ++p) stx(X, p * XC + ci, ib[c][p]);
            }
        }
        if (!WABL(8)) __syncthreads();
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            // Ib = Einc[last] - Eexc; Eexc of slot c = Einc of slot c-1, of slot 0 the lane's prefix
            cx eprev = exl[p];
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const cx e = ib[c][p];
                ib[c][p] = csub(ldx(X, p * XC + si_last(si[c])), eprev);
                eprev = e;
            }
        }
        if (FLG && f.has_lag) {
            // (the sequential-order plan) a post-add target also takes its detached
            // trees' totals; node 1's Ib (position 0: thread 0's slot 0) decides
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const int lx = f.slot_lagx[c * L + tid], hi = lx & 511, lo = (lx >> 9) & 511;
                if (hi != lo) {
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        ib[c][p] = cadd(ib[c][p], csub(ldx(X, p * XC + hi), ldx(X, p * XC + lo)));
                }
            }
            double *const ib1 = wtf + 8 * W;   // (the per-phase extremes' slot: free until after the loop)
            if (tid == 0) {
#pragma unroll
                for (int p = 0; p < 3; ++p) {
                    ib1[2 * p] = ib[0][p].re;
                    ib1[2 * p + 1] = ib[0][p].im;
                }
            }
            __syncthreads();
#pragma unroll
            for (int p = 0; p < 3; ++p) tot[p] = mk(ib1[2 * p], ib1[2 * p + 1]);
        }

        BSTAMP_IT(2);
        // ---- convergence on the substation branch (:199-217), compared as squares;
        // the same in every lane of the workgroup
        double err2 = 0.0;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const double dr = tot[p].re - ibo[p].re, di = tot[p].im - ibo[p].im;
            err2 = fmax(err2, fma(dr, dr, di * di));
            ibo[p] = tot[p];
        }
        conv = __builtin_amdgcn_readfirstlane(err2 < f.eps * f.eps ? 1 : 0) != 0;
        const bool fin = conv || it == f.mxitr - 1;
        if (fin) err2_last = err2;
        if (STASH && fin) {
            // (the full variant) IL into the slot's Sld rows (every Sld read of this
            // sweep is behind the barriers above; the loss reads it back below) and,
            // for the outputs formed after the loop, IL / Ib into the PQL / PQB outputs
            // they become: neither stays in registers through the forward sweep
#pragma unroll
            for (int c = 0; c < C; ++c)
                if (si_valid(si[c])) {
                    const int k = f.slot_node[c * L + tid];
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        stx(stg, p * PS + sb[c], il[c][p]);
                        const size_t o6 = out6(o, nn, B, k, p, (size_t)s), o6i = o6 + out6_im(o, nn, B);
                        if (o.pql) { o.pql[o6] = il[c][p].re; o.pql[o6i] = il[c][p].im; }
                        if (o.pqb) { o.pqb[o6] = ib[c][p].re; o.pqb[o6i] = ib[c][p].im; }
                    }
                }
        }
        // the convergence guard (fpf_wave.hip): err2 is the same in every lane of the
        // workgroup; a decision within 2^-9 of eps^2 keeps its distance in a register
        // (evaluated against the band after the loop)
        if (GUARD_CODE && o.flag_count) {
            const double e2 = f.eps * f.eps, dd = fabs(err2 - e2);
            if (dd <= 0x1p-9 * e2) dmin = fmin(dmin, dd);
        }

        // ---- branch drops lng * (Ib . Zl) (:163-178); in the last sweep also
        // Re(drop . conj(Ib)) per phase for the VVC loss (fpf_wave.hip: the loss identity)
        cx g[C][3];
        double lp[3] = {0.0, 0.0, 0.0};
        if (f.temp_sym) {
            // one common off-diagonal zm: (Ib . Zl)_a = (z_aa - zm) Ib_a + zm (Ib_1 + Ib_2 + Ib_3)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                const cx m = ldx(zc, cz[c] + 3);
                const cx sm = cadd(cadd(ib[c][0], ib[c][1]), ib[c][2]);
                const cx ms = mk(fma(m.re, sm.re, -(m.im * sm.im)), fma(m.re, sm.im, m.im * sm.re));
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const cx d = ldx(zc, cz[c] + a);
                    const cx b = ib[c][a];
                    g[c][a] = mk(lg[c] * fma(d.re, b.re, fma(-d.im, b.im, ms.re)),
                                 lg[c] * fma(d.re, b.im, fma(d.im, b.re, ms.im)));
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < C; ++c) {
                cx tm[9];
#pragma unroll
                for (int j = 0; j < 9; ++j) tm[j] = ldx(zc, cz[c] + j);
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const cx t = drop_col_fma(tm, ib[c][0], ib[c][1], ib[c][2], a);
                    g[c][a] = mk(lg[c] * t.re, lg[c] * t.im);
                }
            }
        }

        // (a uniform branch of its own: inside the slot loops the compiler turned the
        // accumulation into selects executed every sweep)
        if (fin) {
#pragma unroll
            for (int c = 0; c < C; ++c)
#pragma unroll
                for (int a = 0; a < 3; ++a)
                    lp[a] = fma(g[c][a].re, ib[c][a].re, fma(g[c][a].im, ib[c][a].im, lp[a]));
        }

        BSTAMP_IT(3);
        if (SEG) {
            // ---- forward sweep (:163-195): V = V0 - A(k), A(k) = off(block) + Gseg(k),
            // Gseg the block-local path sum of the drops (a prefix scan segmented at
            // the block heads: every block is a run of consecutive positions, each the
            // child of the one before), off(b) = the sum over b's block-ancestor chain
            // of Gseg at the taps.  Lane-local part, resetting at heads:
            int hf = 0;   // a block head among this lane's slots
    #pragma unroll
            for (int c = 0; c < C; ++c) hf |= si_head(si[c]) ? 1 : 0;
    #pragma unroll
            for (int p = 0; p < 3; ++p) {
                cx acc = g[0][p];
    #pragma unroll
                for (int c = 1; c < C; ++c) { acc = si_head(si[c]) ? g[c][p] : cadd(acc, g[c][p]); g[c][p] = acc; }
                sc6[2 * p] = acc.re;
                sc6[2 * p + 1] = acc.im;
            }
            // the wave's segmented scan over the lanes' (total, head) pairs; the lane
            // before's inclusive value by wave_shr:1 (lane 0: none)
            int hs = hf;
            segf_incl64(sc6, hs);
            double pv[6];
    #pragma unroll
            for (int q = 0; q < 6; ++q) pv[q] = dpp_d<0x138, 0xf, 0xf>(sc6[q]);
            const int hp = dpp_i<0x138, 0xf, 0xf>(hs);
            if (lane == 63) {
    #pragma unroll
                for (int q = 0; q < 6; ++q) wtf[8 * wv + q] = sc6[q];
                wtf[8 * wv + 6] = hs ? 1.0 : 0.0;
            }
            __syncthreads();
            wave_prefix_seg<W>(wtf, wv, lane, pre);
    #pragma unroll
            for (int p = 0; p < 3; ++p) {
                // the carry into this lane: the segment running in from the lanes and
                // waves before, up to this lane's first head
                const cx lc = hp ? mk(pv[2 * p], pv[2 * p + 1]) : mk(pre[2 * p] + pv[2 * p], pre[2 * p + 1] + pv[2 * p + 1]);
                bool seen = false;
    #pragma unroll
                for (int c = 0; c < C; ++c) {
                    seen = seen || si_head(si[c]);
                    if (!seen) g[c][p] = cadd(lc, g[c][p]);   // Gseg at this slot
                }
            }
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                const int ci = si_store_f(si[c]);
                if (ci >= 0) {
    #pragma unroll
                    for (int p = 0; p < 3; ++p) stx(X, p * XC + ci, g[c][p]);
                }
            }
            if (!WABL(8)) __syncthreads();
            // block offsets, one thread per block, stored as V0 - off(b) (and off(b)
            // itself for the restart below a zeroed phase); one X read per chain level
            if (off3) {
                if (tid < 3 * nblk) {
                    cx of = mk(0, 0);
    #pragma unroll
                    for (int j = 0; j < WB_BD; ++j)
                        if (j < bdepth) of = cadd(of, ldx(X, op3 * XC + (bp[j] & 0xffff)));   // uniform bound
                    stx(OFF, op3 * nblk + ob3, csub(ldx(V0S, op3), of));
                    if (FM && f.has_rel) stx(OFFA, op3 * nblk + ob3, of);   // (has_rel: never with has_lag)
                }
            } else if (chain_regs) {
                if (tid < nblk) {
                    cx of[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
    #pragma unroll
                    for (int j = 0; j < WB_BD; ++j) {
                        if (j < bdepth) {   // uniform; levels past a chain's depth read the zero entry
    #pragma unroll
                            for (int p = 0; p < 3; ++p) of[p] = cadd(of[p], ldx(X, p * XC + (bp[j] & 0xffff)));
                        }
                    }
    #pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        stx(OFF, p * nblk + tid, csub(ldx(V0S, p), of[p]));
                        if (FM && f.has_rel) stx(OFFA, p * nblk + tid, of[p]);
                    }
                }
            } else
            for (int b = tid; b < nblk; b += NT) {
                cx of[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
                for (int j = 0; j < bdepth; ++j) {
                    const int pa = pairs[(2 * j) * nblk + b];
    #pragma unroll
                    for (int p = 0; p < 3; ++p) of[p] = cadd(of[p], ldx(X, p * XC + pa));
                }
    #pragma unroll
                for (int p = 0; p < 3; ++p) {
                    stx(OFF, p * nblk + b, csub(ldx(V0S, p), of[p]));
                    if (FM && f.has_rel) stx(OFFA, p * nblk + b, of[p]);
                }
            }
            __syncthreads();
    #pragma unroll
            for (int c = 0; c < C; ++c)
    #pragma unroll
                for (int p = 0; p < 3; ++p) {
                    const cx vr = csub(ldx(OFF, p * nblk + bk[c]), g[c][p]);   // V0 - A(k)
                    v[c][p] = (FM && ((si_mask(si[c]) >> p) & 1)) ? mk(0.0, 0.0) : vr;   // phase zeroing (:180-192)
                }
            if (FM && f.has_rel) {
                // below a zeroed ancestor m: V(k,p) = A(m) - A(k) (:180-195: the path
                // restarts from 0 at m), both small path sums; the forward entries (the
                // block offsets are read) carry A now
    #pragma unroll
                for (int c = 0; c < C; ++c) {
                    const int ci = si_store_f(si[c]);
                    if (ci >= 0) {
    #pragma unroll
                        for (int p = 0; p < 3; ++p) stx(X, p * XC + ci, cadd(ldx(OFFA, p * nblk + bk[c]), g[c][p]));
                    }
                }
                __syncthreads();
    #pragma unroll
                for (int c = 0; c < C; ++c)
    #pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        const int mr = f.slot_mref[(p * C + c) * L + tid];
                        if (mr >= 0 && !((si_mask(si[c]) >> p) & 1))
                            v[c][p] = csub(ldx(X, p * XC + mr), cadd(ldx(OFFA, p * nblk + bk[c]), g[c][p]));
                    }
            }
        } else {
            // (feeders without a live phase below a zeroed one: one global prefix scan,
            // off(b) from the differences Ginc[tap] - Ginc[first - 1]; 5 % faster than
            // the segmented scan on config 3)
            // ---- forward sweep (:163-195): V = V0 - A, A = Ginc + off(block)
    #pragma unroll
            for (int p = 0; p < 3; ++p) {
                cx acc = g[0][p];
    #pragma unroll
                for (int c = 1; c < C; ++c) { acc = cadd(acc, g[c][p]); g[c][p] = acc; }
                sc6[2 * p] = acc.re;
                sc6[2 * p + 1] = acc.im;
            }
            seg_incl_n<64>(sc6);
            if (lane == 63) {
    #pragma unroll
                for (int q = 0; q < 6; ++q) wtf[8 * wv + q] = sc6[q];
            }
            __syncthreads();
            BSTAMP_IT(4);
            wave_prefix<W, false>(wtf, wv, lane, pre, tot6);
    #pragma unroll
            for (int p = 0; p < 3; ++p) {
                const cx ex = csub(mk(pre[2 * p] + sc6[2 * p], pre[2 * p + 1] + sc6[2 * p + 1]), g[C - 1][p]);
    #pragma unroll
                for (int c = 0; c < C; ++c) g[c][p] = cadd(ex, g[c][p]);   // Ginc at this slot
            }
    #pragma unroll
            for (int c = 0; c < C; ++c) {
                const int ci = si_store_f(si[c]);
                if (ci >= 0) {
    #pragma unroll
                    for (int p = 0; p < 3; ++p) stx(X, p * XC + ci, g[c][p]);
                }
            }
            if (!WABL(8)) __syncthreads();
            // block offsets, one thread per block, stored as V0 - off(b): off(b) = sum over
            // b's block-ancestor chain of Ginc[tap] - Ginc[first - 1] (block 0: 0)
            if (off3) {
                if (tid < 3 * nblk) {
                    cx of = mk(0, 0);
    #pragma unroll
                    for (int j = 0; j < WB_BD; ++j)
                        if (j < bdepth)   // uniform; levels past a chain's depth read the zero entry
                            of = cadd(of, csub(ldx(X, op3 * XC + (bp[j] & 0xffff)), ldx(X, op3 * XC + (bp[j] >> 16))));
                    const int bb = (FLG && f.has_lag) ? f.blk_base[ob3] : -1;   // (sequential-order plan: V_prev base)
                    stx(OFF, op3 * nblk + ob3, csub(bb >= 0 ? ldx(LAGV, op3 * NLAG + bb) : ldx(V0S, op3), of));
                }
            } else if (chain_regs) {
                if (tid < nblk) {
                    cx of[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
    #pragma unroll
                    for (int j = 0; j < WB_BD; ++j) {
                        if (j < bdepth) {   // uniform; levels past a chain's depth read the zero entry
    #pragma unroll
                            for (int p = 0; p < 3; ++p)
                                of[p] = cadd(of[p], csub(ldx(X, p * XC + (bp[j] & 0xffff)), ldx(X, p * XC + (bp[j] >> 16))));
                        }
                        // (two levels' twelve reads in flight at a time: the registers of
                        // all of them at once would spill)
                        if (j & 1) __builtin_amdgcn_sched_barrier(0);
                    }
                    const int bb = (FLG && f.has_lag) ? f.blk_base[tid] : -1;
    #pragma unroll
                    for (int p = 0; p < 3; ++p)
                        stx(OFF, p * nblk + tid, csub(bb >= 0 ? ldx(LAGV, p * NLAG + bb) : ldx(V0S, p), of[p]));
                }
            } else
            for (int b = tid; b < nblk; b += NT) {
                cx of[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
                for (int j = 0; j < bdepth; ++j) {
                    const int pa = pairs[(2 * j) * nblk + b], mi = pairs[(2 * j + 1) * nblk + b];
    #pragma unroll
                    for (int p = 0; p < 3; ++p) of[p] = cadd(of[p], csub(ldx(X, p * XC + pa), ldx(X, p * XC + mi)));
                }
                const int bb = (FLG && f.has_lag) ? f.blk_base[b] : -1;
    #pragma unroll
                for (int p = 0; p < 3; ++p)
                    stx(OFF, p * nblk + b, csub(bb >= 0 ? ldx(LAGV, p * NLAG + bb) : ldx(V0S, p), of[p]));
            }
            __syncthreads();
            BSTAMP_IT(5);
    #pragma unroll
            for (int c = 0; c < C; ++c)
    #pragma unroll
                for (int p = 0; p < 3; ++p) {
                    const cx vr = csub(ldx(OFF, p * nblk + bk[c]), g[c][p]);   // V0 - A(k)
                    v[c][p] = (FM && ((si_mask(si[c]) >> p) & 1)) ? mk(0.0, 0.0) : vr;   // phase zeroing (:180-192)
                }
        }
        BSTAMP_IT(6);

        if (fin) {
            // ---- the last sweep: the wave's part of the VVC loss
            // (VoltVarCtrl.cpp:1152-1161), then V of node k over Sld row k - 1; the
            // full outputs after the loop
            double x;
            if (FG && (f.has_mask || f.has_lag)) {
                // zeroed phases, the sequential-order plan: the reference's sum over PQL
                // (the loss identity needs every phase live and tree paths); the wave's
                // part of sum Re(V conj(IL)), IL from the slot's Sld rows (SEG: still in
                // registers)
                x = 0.0;
#pragma unroll
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        if (si_valid(si[c])) {
                            const cx ils = STASH ? ldx(stg, p * PS + sb[c]) : il[c][p];
                            x = fma(v[c][p].re, ils.re, fma(v[c][p].im, ils.im, x));
                        }
                x = seg_incl<64>(x);
            } else {
                x = seg_incl<64>(lp[0] + lp[1] + lp[2]);
            }
            if (lane == 63) wtb[8 * wv + 6] = x;
            if (STASH) __syncthreads();   // (every stashed IL read before V goes over the rows)
#pragma unroll
            for (int c = 0; c < C; ++c) {
                if (si_valid(si[c])) {
                    const int k = f.slot_node[c * L + tid];
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        stx(stg, p * PS + k - 1, v[c][p]);
                        // (the general variants emit here; see STASH)
                        if (FULL && !STASH) emit_full(o, f.s3, nn, B, k, p, (size_t)s, v[c][p], il[c][p], ib[c][p]);
                    }
                }
            }
            break;
        }
    }
    BSTAMP(120);
    if (STASH && (o.pql || o.pqb)) __threadfence();   // (the stashes, for the other threads' reads below)
    __syncthreads();
    if (STASH) {
        // (the full variant) the outputs of DPF_return7.cpp:222-253, node by node in
        // output order (consecutive threads, consecutive nodes): V from its row, IL / Ib
        // from the stashes (node 0: below, from the last sweep's Ib(0))
        const size_t oim = out6_im(o, nn, B);
        for (int i = tid; i < 3 * nn; i += NT) {
            const int p = i / nn, k = i - p * nn;
            if (k == 0) continue;
            const size_t o6 = out6(o, nn, B, k, p, (size_t)s);
            const cx ils = o.pql ? mk(__hip_atomic_load(o.pql + o6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                      __hip_atomic_load(o.pql + o6 + oim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                                 : mk(0, 0);
            const cx ibs = o.pqb ? mk(__hip_atomic_load(o.pqb + o6, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                                      __hip_atomic_load(o.pqb + o6 + oim, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                                 : mk(0, 0);
            emit_full(o, f.s3, nn, B, k, p, (size_t)s, ldx(stg, p * PS + k - 1), ils, ibs);
        }
    }

    // ---- Vmin/Vmax (V_abc_list.cpp:7-81, VoltVarCtrl.cpp:1201-1207)
    if (FM && f.has_mask) {
        // general V_abc_list: per phase the first K_p nonzero |V| in node order,
        // zero padded; one wave per phase, 64 nodes per step (ballot ranks); also
        // min over every nonzero |V|^2 of the wave's phases (the guard band)
        double mz = INFINITY;
        for (int p = wv; p < 3; p += W) {
            const int K = f.K[p];
            int cnt = 0;
            double mn = INFINITY, mx = -INFINITY;
            for (int k0 = 0; k0 < nn; k0 += 64) {
                const int k = k0 + lane;
                double m = 0.0;
                if (k < nn) {
                    const cx vv = k == 0 ? ldx(V0S, p) : ldx(stg, p * PS + k - 1);
                    m = sqrt(fma(vv.re, vv.re, vv.im * vv.im));
                }
                const bool nz = k < nn && m != 0.0;
                if (nz) mz = fmin(mz, m * m);
                const unsigned long long bal = __ballot(nz);
                const int rank = cnt + __popcll(bal & ((1ull << lane) - 1ull));
                if (nz && rank < K) { mn = fmin(mn, m); mx = fmax(mx, m); }
                cnt += __popcll(bal);
            }
            if (cnt < K) { mn = fmin(mn, 0.0); mx = fmax(mx, 0.0); }
            mn = seg_reduce_min<64>(mn);
            mx = seg_reduce_max<64>(mx);
            if (lane == 63) {
                vx[2 * p] = mn;
                vx[2 * p + 1] = mx;
            }
        }
        mz = seg_reduce_min<64>(mz);
        if (lane == 63) wtf[8 * wv + 5] = mz;   // (the forward totals are dead)
    } else {
        // no zeroed phases: every Lnum_p + 1 = Nn and V_abc_list keeps every row --
        // the plain extremes of |V| (|V|^2 compared, one sqrt each)
        double mn = INFINITY, mx = -INFINITY;
        for (int k = tid; k < nn; k += NT) {
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const cx vv = k == 0 ? ldx(V0S, p) : ldx(stg, p * PS + k - 1);
                const double m2 = fma(vv.re, vv.re, vv.im * vv.im);
                mn = fmin(mn, m2);
                mx = fmax(mx, m2);
            }
        }
        mn = seg_reduce_min<64>(mn);
        mx = seg_reduce_max<64>(mx);
        if (lane == 63) {
            wtf[8 * wv + 6] = mn;
            wtf[8 * wv + 7] = mx;
        }
    }
    __syncthreads();
    BSTAMP(121);

    // ---- per-scenario results and the fused batch aggregate [loss_sum, vmin, vmax,
    // n_conv, n_nonconv, n_over, n_under, n_scen]: the scenario's partial, published
    // with agent-scope stores; one ticket per workgroup; the last to arrive folds
    // the partials in scenario order (deterministic)
    __shared__ int last_wg;
    const bool agg = o.agg != nullptr;
    if (tid == 0) {
        double x = 0.0, mn = INFINITY, mx = -INFINITY;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            x += wtb[8 * w + 6];
            mn = fmin(mn, wtf[8 * w + 6]);
            mx = fmax(mx, wtf[8 * w + 7]);
        }
        if (FG && (f.has_mask || f.has_lag)) {
            // PQb(0).re - sum_k PQL(k).re, V0 conj(Ib(0)) of the last sweep
            double sb0 = 0.0;
#pragma unroll
            for (int p = 0; p < 3; ++p) sb0 += cmul(cmul(ldx(V0S, p), mk(f.s3, 0.0)), cconj(ibo[p])).re;
            x = sb0 - f.s3 * x;
        } else {
            x *= f.s3;
        }
        if (FM && f.has_mask) {
            mn = fmin(fmin(vx[0], vx[2]), vx[4]);
            mx = fmax(fmax(vx[1], vx[3]), vx[5]);
        } else {
            mn = sqrt(mn);
            mx = sqrt(mx);
        }
        if (o.iters) o.iters[s] = it + 1;
        if (o.status) o.status[s] = conv ? 0 : 1;
        if (o.loss) o.loss[s] = x;
        if (o.errmx) o.errmx[s] = sqrt(err2_last);
        if (GUARD_CODE && o.flag_count) {
            // the guard band (fpf_api.cpp: guard_factor) of a decision in the coarse
            // band: errmx within tau = guard_k sum_k |IL_k|_1 of eps, with sum_k
            // |IL_k|_1 <= sqrt2 sum_k |S_k|_1 / min_k |V_k| over the nonzero V (the
            // final V; 1.25 covers its drift from the deciding sweep's); flagged
            // scenarios are re-solved on the exact kernel (dpf_fixup_kernel)
            bool near = false;
            if (dmin < INFINITY) {
                double sabs = 0.0, m2 = INFINITY;
#pragma unroll
                for (int w = 0; w < W; ++w) {
                    sabs += wtb[8 * w + 7];
                    m2 = fmin(m2, (FM && f.has_mask) ? wtf[8 * w + 5] : wtf[8 * w + 6]);
                }
                const double tau = 1.25 * f.guard_k * 1.4142135623730951 * sabs / sqrt(m2);
                near = dmin <= 2.0 * f.eps * (1.0 + 0x1p-9) * tau;
            }
            if (o.guard) o.guard[s] = near ? 1 : 0;
            if (near) guard_flag(o, s, nullptr, nullptr);
        } else if (o.guard) {
            o.guard[s] = 0;
        }
        if (o.vmin) o.vmin[s] = mn;
        if (o.vmax) o.vmax[s] = mx;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const cx v0p = ldx(V0S, p);
            // substation row 0: V0, Ib(0) = the last sweep's total, no load
            if (FULL) emit_full(o, f.s3, nn, B, 0, p, (size_t)s, v0p, mk(0, 0), ibo[p]);
            if (o.s_in) {   // PQb row 0: (bkva/3) V0 conj(Ib(0))  (:242-244)
                const cx sbv = cmul(cmul(v0p, mk(f.s3, 0.0)), cconj(ibo[p]));
                o.s_in[(size_t)(2 * p) * B + s] = sbv.re;
                o.s_in[(size_t)(2 * p + 1) * B + s] = sbv.im;
            }
        }
        if (agg) {
            const double part[8] = {conv ? x : 0.0, conv ? mn : INFINITY, conv ? mx : -INFINITY, conv ? 1.0 : 0.0,
                                    conv ? 0.0 : 1.0, conv && mx > f.ub_v ? 1.0 : 0.0, conv && mn < f.lb_v ? 1.0 : 0.0,
                                    1.0};
            double *dst = o.partials + 8 * (size_t)s;
            for (int q = 0; q < 8; ++q) __hip_atomic_store(dst + q, part[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned t = __hip_atomic_fetch_add(o.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_wg = t == gridDim.x - 1;
        }
    }
    BSTAMP(122);
    // ---- V out: [3][Nn][B] re / im planes, column s (or the scenario's
    // contiguous [3][Nn] block in the scenario-major layout)
    if (!FULL && (o.v_re || o.v_im) && !WABL(2)) {
        const size_t base = o.smaj ? (size_t)s * 3 * nn : (size_t)s, step = o.smaj ? 1 : (size_t)B;
        RowWalk w;   // (phase, node) of element i = p Nn + k, walked NT apart
        w.init(tid, NT, nn);
        for (int i = tid; i < 3 * nn; i += NT, w.next()) {
            const int p = w.fq, k = w.rr;
            const double2 vv = k == 0 ? V0S[p] : stg[p * PS + k - 1];
            double *const re = o.v_re + base + (size_t)i * step, *const im = o.v_im + base + (size_t)i * step;
            if (o.smaj) {   // streaming rows of one block
                if (o.v_re) __builtin_nontemporal_store(vv.x, re);
                if (o.v_im) __builtin_nontemporal_store(vv.y, im);
            } else {        // 8 bytes of lines the neighbouring scenarios' workgroups share (L2)
                if (o.v_re) *re = vv.x;
                if (o.v_im) *im = vv.y;
            }
        }
    }
    BSTAMP(123);
    if (agg) {
        __syncthreads();
        if (last_wg) {
            // thread i folds scenarios i, i + NT, ... in order, then a fixed tree
            double a[8] = {0, INFINITY, -INFINITY, 0, 0, 0, 0, 0};
            for (unsigned b = tid; b < gridDim.x; b += NT) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const double r = __hip_atomic_load(o.partials + 8 * (size_t)b + q, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                    a[q] = q == 1 ? fmin(a[q], r) : (q == 2 ? fmax(a[q], r) : a[q] + r);
                }
            }
            double *sh = (double *)stg;   // [8][NT] (Sld / V and the rest are dead; wblk_lds_bytes covers it)
#pragma unroll
            for (int q = 0; q < 8; ++q) sh[q * NT + tid] = a[q];
            __syncthreads();
            for (int w = NT / 2; w > 0; w >>= 1) {
                if (tid < w) {
                    sh[0 * NT + tid] += sh[0 * NT + tid + w];
                    sh[1 * NT + tid] = fmin(sh[1 * NT + tid], sh[1 * NT + tid + w]);
                    sh[2 * NT + tid] = fmax(sh[2 * NT + tid], sh[2 * NT + tid + w]);
#pragma unroll
                    for (int q = 3; q < 8; ++q) sh[q * NT + tid] += sh[q * NT + tid + w];
                }
                __syncthreads();
            }
            if (tid < 8) o.agg[tid] = sh[tid * NT];
            if (tid == 0) __hip_atomic_store(o.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tid == 0 && o.flag_out)   // (every workgroup's flag was appended before its ticket)
                *o.flag_out = __hip_atomic_load(o.flag_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace fpf
