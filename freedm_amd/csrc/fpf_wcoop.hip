// fpf_wcoop.hip -- the paired wave-block kernel (fast mode, fpf_opts.exact = 0)
// for feeders of 2049..4096 branches: every sweep of DPF_return7
// (Broker/src/vvc/DPF_return7.cpp:104-217) over two workgroups per scenario.
//
// One 2048-branch scenario already fills a CU (fpf_wblk.hip: V and the sweep
// temporaries in 8 wavefronts' registers, the loads in LDS), so a larger one
// takes two CUs.  The depth-first position order of fpf_wblk.hip is cut in two:
// workgroup g holds the positions [g P, g P + P) (P = ceil(n / 2)), 8 wavefronts
// x 64 lanes x C = 4 slots, with its slots' loads in its own LDS and V in
// registers for the whole solve.  Each prefix scan (the backward sweep's subtree
// sums of IL, :134-160; the forward sweep's path sums of the drops, :163-195) is
// computed per workgroup; the two workgroups then exchange, through an L2-backed
// area of their own, the workgroup totals and the scan values at the positions
// they own that either side gathers (subtree ends; block taps and the positions
// before lateral blocks).  Each side rebuilds the whole gathered array X in its
// LDS, adding workgroup 0's total to workgroup 1's values, so every gather and
// block offset is the global prefix -- two exchanges per sweep.  Ib(0) is the sum
// of the two totals in one fixed order on both sides, so the convergence test
// (:199-217) takes the same decision in both workgroups.
//
// Synchronisation: the members of scenario t are workgroups b and b + 8 (one
// XCD), dispatched in order, so a waiting workgroup's partner is resident or
// next in line.  A member publishes with agent-scope stores, waits for its
// stores, then adds one to the area's arrival count; the other polls the count
// (thread 0, with s_sleep between polls) and reads with agent-scope loads.  A wait
// gives up after a bounded number of polls (the error word is set, every
// workgroup of the launch stops at its next wait, the scenario reports status
// FPF_EXCHANGE_FAILED and the feeder's sticky host word is set),
// so a launch always drains.  The areas are reused round robin (COOP_NSLOT of
// them); a scenario waits until the area's previous scenario has released it.
//
// Zeroed phases as in the wave-block kernel (V = 0 on the phase, the loss over
// PQL, the general V_abc_list extremes: both workgroups' |V| of the last sweep
// through a scratch row, ranked in node order by workgroup 0); a live phase below
// a zeroed one is declined on the host (the generic kernel runs it).
#include <array>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>

#include "fpf_internal.h"
#include "fpf_math.hpp"
#include "fpf_wave_common.h"

namespace fpf {

namespace {
constexpr int CW = 8;                  // wavefronts per workgroup
constexpr int CC = 4;                  // slots per lane
constexpr int CL = 64 * CW;            // lanes (= threads) per workgroup
constexpr int CBD = 6;                 // block-chain depth resolved from registers (the host checks)
constexpr int AH = 48;                 // area header: backward totals [2][8], forward [2][8], final [2][8]

__device__ __forceinline__ int ci_store_b(unsigned x) { return (int)((x >> 4) & 16383u) - 1; }
__device__ __forceinline__ int ci_last(unsigned x) { return (int)(x >> 18); }
__device__ __forceinline__ void ast(double *p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ald(double *p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// thread 0 polls *w until pred(*w) (or the error word is set, or the polls run
// out: then it sets the error word); the verdict is broadcast through LDS
template <typename Pred>
__device__ __forceinline__ bool coop_poll(unsigned *w, unsigned *err, int *flag, int spin, Pred pred) {
    if (threadIdx.x == 0) {
        int ok = 0;
        for (int i = 0; i < spin; ++i) {
            if (pred(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                ok = 1;
                break;
            }
            if (__hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
            __builtin_amdgcn_s_sleep(2);
        }
        if (!ok) __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = ok;
    }
    __syncthreads();
    return *flag != 0;
}

// every thread's area stores complete, then one arrival; wait: until both
// members have arrived `target` times in total
__device__ __forceinline__ bool coop_arrive(unsigned *cnt, unsigned target, unsigned *err, int *flag, int spin,
                                            bool wait) {
    __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!wait) return true;
    return coop_poll(cnt, err, flag, spin, [=](unsigned c) { return c >= target; });
}

// The exchange area through a buffer resource: 16-byte sc1 (write-through)
// stores and sc1 loads (MI355X_MICROARCH.md, inter-workgroup visibility: every
// byte stored sc1, each storing wave waits for its stores before the arrival,
// every load of the bytes an sc1 load after the poll and a workgroup barrier)
typedef double d2v __attribute__((ext_vector_type(2)));
typedef unsigned u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void bst(__amdgpu_buffer_rsrc_t r, int off, double re, double im) {
    const d2v v = {re, im};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), r, off, 0, 16);
}
__device__ __forceinline__ d2v bld(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}

// One exchange of a scan (the owned entries are in X as this workgroup's local
// prefix values): the owned range of the index space [0, split) | [split, n) out
// to the area's entries [3][n] complex at byte xoff (one coalesced pass), the
// workgroup total to the totals [2][8] at byte toff; after both arrivals the
// partner's range into X, workgroup 1's entries (on either side) plus workgroup
// 0's total; both totals to tt (T0 re/im per phase, then T1)
__device__ __forceinline__ bool coop_exchange(double2 *X, int XC, __amdgpu_buffer_rsrc_t r, int xoff, int toff, int n,
                                              int split, int g, const double (&tot6)[6], double *tt, unsigned *cnt,
                                              unsigned target, unsigned *err, int *flag, int spin) {
    const int tid = threadIdx.x;
    __syncthreads();   // (the owned entries are in X)
    const int lo = g ? split : 0, own = g ? n - split : split;
    for (int i = tid; i < 3 * own; i += CL) {
        const int p = i / own, e = lo + i - p * own;
        const double2 x = X[p * XC + e];
        bst(r, xoff + 16 * (p * n + e), x.x, x.y);
    }
    if (tid == 0) {
#pragma unroll
        for (int p = 0; p < 3; ++p) bst(r, toff + 64 * g + 16 * p, tot6[2 * p], tot6[2 * p + 1]);
    }
    // (a wait that gave up reads garbage and the caller finishes the sweep with it:
    // no early exit in the sweep loop)
    const bool ok = coop_arrive(cnt, target, err, flag, spin, true);
    // workgroup 0's total (the carry) loaded beside the entries (every load of a
    // thread in flight at once: the hand-off costs one load latency)
    d2v t0[3];
#pragma unroll
    for (int p = 0; p < 3; ++p) t0[p] = bld(r, toff + 16 * p);
    const d2v tmine = bld(r, toff + 64 * (tid < 6 ? tid / 3 : 0) + 16 * (tid < 6 ? tid % 3 : 0));
    const int plo = g ? 0 : split, pn = g ? split : n - split;
    constexpr int U = 4;
    for (int i0 = 0; i0 < 3 * pn; i0 += U * CL) {
        d2v x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * CL + tid, p = i / pn, e = plo + i - p * pn;
            x[u] = bld(r, i < 3 * pn ? xoff + 16 * (p * n + e) : toff);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int i = i0 + u * CL + tid, p = i / pn, e = plo + i - p * pn;
            if (i < 3 * pn) {
                // workgroup 1's entries (the partner's when g = 0) carry workgroup 0's total
                const d2v c = p == 0 ? t0[0] : (p == 1 ? t0[1] : t0[2]);
                X[p * XC + e] = g ? make_double2(x[u].x, x[u].y) : make_double2(x[u].x + c.x, x[u].y + c.y);
            }
        }
    }
    if (g) {
        for (int i = tid; i < 3 * own; i += CL) {
            const int p = i / own, e = lo + i - p * own;
            const double2 x = X[p * XC + e];
            const d2v c = p == 0 ? t0[0] : (p == 1 ? t0[1] : t0[2]);
            X[p * XC + e] = make_double2(x.x + c.x, x.y + c.y);
        }
    }
    if (tid < 6) {
        tt[2 * tid] = tmine.x;
        tt[2 * tid + 1] = tmine.y;
    }
    __syncthreads();
    return ok;
}
}  // namespace

#ifdef FPF_STAMPS
// diagnostic build only (tools/coop_stamps.py): thread 0 of each of the first 64
// workgroups records s_memtime at stage boundaries, [64][128]: 0 entry, 1 staged,
// 2 area acquired, 4 + 8 it + k in sweep it < 14 (k = 0 top, 1 backward scan,
// 2 backward exchange, 3 drops, 4 forward scan, 5 forward exchange, 6 V),
// 120 after the loop, 121 workgroup 0's final wait
__device__ unsigned long long *fpf_coop_stamp_buf = nullptr;
__device__ unsigned fpf_coop_stamp_base = 0;   // the first recorded workgroup
#define CSTAMP(idx)                                                                                    \
    do {                                                                                               \
        const unsigned w_ = blockIdx.x - fpf_coop_stamp_base;                                          \
        if (fpf_coop_stamp_buf && threadIdx.x == 0 && w_ < 64u && (idx) < 128)                         \
            fpf_coop_stamp_buf[w_ * 128 + (idx)] = __builtin_amdgcn_s_memtime();                        \
    } while (0)
extern "C" int fpf_debug_set_coop_stamp_buffer(void *dptr, unsigned base) {
    unsigned long long *p = (unsigned long long *)dptr;
    if (hipMemcpyToSymbol(HIP_SYMBOL(fpf_coop_stamp_base), &base, sizeof(base)) != hipSuccess) return -3;
    return hipMemcpyToSymbol(HIP_SYMBOL(fpf_coop_stamp_buf), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#define CSTAMP_IT(k) CSTAMP(it < 14 ? 4 + 8 * it + (k) : 999)
#else
#define CSTAMP(idx) ((void)0)
#define CSTAMP_IT(k) ((void)0)
#endif

template <bool FULL>
__global__ __launch_bounds__(CL, 2) void dpf_wcoop_kernel(WaveDev f, int B, const double *__restrict__ pq, OutDev o) {
    extern __shared__ double2 lds[];
    if (o.skip && *o.skip) return;   // (the multi-area solve's device-side stop)
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int b = blockIdx.x, g = (b >> 3) & 1;
    const int s = ((b >> 4) << 3) | (b & 7);   // this pair's scenario (members b, b + 8)
    if (s >= B) return;                        // (both members of a padding pair)
    CSTAMP(0);
    const int nblk = f.nblk, nn = f.nn, nl = f.nl, XC = f.ncomp + 1, nbc = f.nb_c, nfc = f.nf_c;
    const int ntz = f.temp_sym ? 4 : 9;
    constexpr int PS = CC * CL + 1;   // Sld rows: slot c L + tid (row C L = 0)
    // LDS: Zl per code | Sld [3][PS] (this workgroup's slots) | X [3][XC] (the whole
    // gathered array; entry XC - 1 = 0) | block offsets [3][nblk] | V0 [3] (+1) |
    // wave totals [2][W][8] | exchanged totals [16] | flag
    double2 *const zc = lds;
    double2 *const stg = zc + f.ncode * ntz;
    double2 *const X = stg + 3 * PS;
    double2 *const OFF = X + 3 * XC;
    double2 *const V0S = OFF + 3 * nblk;
    double *const wtb = (double *)(V0S + 4);
    double *const wtf = wtb + 8 * CW;
    double *const tt = wtf + 8 * CW;            // [24] the exchanged totals (backward 0..11, forward 12..17)
    int *const flag = (int *)(tt + 24);
    __shared__ int last_wg;

    const int slot = s % f.coop_nslot;
    double *const A = f.xch + (size_t)slot * f.coop_area;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(A, 0, 8 * f.coop_area, 0x00020000);
    unsigned *const cnt = f.xsync + slot, *const gen = f.xsync + f.coop_nslot + slot;
    unsigned *const err = f.xsync + 2 * f.coop_nslot;
    const int so = g * CC * CL;   // this workgroup's slot tables

    // ---- this workgroup's slots: their loads P/Q (column s of pq, or its block in
    // the scenario-major layout) into Sld scaled by 1/(bkva/3) (DPF_return7.cpp:46-50)
    unsigned si[CC];
    unsigned sx[CC];   // bits 0-8 block, 9-22 forward index + 1, 23-31 line code (< 512: analyse_coop checks the widths)
    double sabs = 0.0;   // the guard record: sum |S_k|_1 over the slots
    {
        const double inv_s3 = 1.0 / f.s3;
        int r[CC];
        double x[CC][6];
#pragma unroll
        for (int c = 0; c < CC; ++c) r[c] = f.slot_row[so + c * CL + tid];
#pragma unroll
        for (int c = 0; c < CC; ++c)
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                const size_t e = o.smaj ? (size_t)s * 6 * nl + (size_t)q * nl + (r[c] < 0 ? 0 : r[c])
                                        : ((size_t)q * nl + (r[c] < 0 ? 0 : r[c])) * B + s;
                x[c][q] = __builtin_nontemporal_load(pq + e);
            }
#pragma unroll
        for (int c = 0; c < CC; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const cx v = r[c] < 0 ? mk(0.0, 0.0) : mk(x[c][2 * p] * inv_s3, x[c][2 * p + 1] * inv_s3);
                stx(stg, p * PS + c * CL + tid, v);
                sabs += fabs(v.re) + fabs(v.im);
            }
#pragma unroll
        for (int c = 0; c < CC; ++c) {
            si[c] = (unsigned)f.slot_info[so + c * CL + tid];
            sx[c] = (unsigned)f.slot_blk[so + c * CL + tid] | ((unsigned)f.slot_info2[so + c * CL + tid] << 9) |
                    ((unsigned)f.slot_code[so + c * CL + tid] << 23);
        }
    }
    for (int i = tid; i < f.ncode * ntz; i += CL) zc[i] = ld_global2(f.code_z, i);
    if (tid < 3) {
        X[tid * XC + XC - 1] = make_double2(0.0, 0.0);
        double2 v0 = tid == 0 ? make_double2(f.V0[0], f.V0[1])
                              : (tid == 1 ? make_double2(f.V0[2], f.V0[3]) : make_double2(f.V0[4], f.V0[5]));
        if (o.vsrc) v0 = make_double2(o.vsrc[(size_t)(2 * tid) * B + s], o.vsrc[(size_t)(2 * tid + 1) * B + s]);
        V0S[tid] = v0;
    }
    // this thread's block chain (thread b < nblk resolves block b), two indices per register
    int bp[CBD];
#pragma unroll
    for (int j = 0; j < CBD; ++j) {
        const bool ok = j < f.bdepth && tid < nblk;
        bp[j] = ok ? f.blk_pairs[(2 * j) * nblk + tid] | (f.blk_pairs[(2 * j + 1) * nblk + tid] << 16)
                   : (XC - 1) | ((XC - 1) << 16);
    }
    {
        const double a = seg_incl<64>(sabs);
        if (lane == 63) wtb[8 * wv + 7] = a;
    }
    // the exchange area: free once its previous scenario (s - nslot) has released it
    const unsigned want = (unsigned)(s / f.coop_nslot);
    CSTAMP(1);
    bool alive = coop_poll(gen, err, flag, f.coop_spin, [=](unsigned v) { return v == want; });
    CSTAMP(2);

    cx v[CC][3];
#pragma unroll
    for (int p = 0; p < 3; ++p) {
        const cx v0 = ldx(V0S, p);
#pragma unroll
        for (int c = 0; c < CC; ++c) v[c][p] = v0;   // V(0..Nl-1) = V0  (:92-96)
    }
    if (o.vinit_re) {   // the multi-area solve's warm start
#pragma unroll
        for (int c = 0; c < CC; ++c)
            if ((si[c] >> 3) & 1) {
                const int k = f.slot_node[so + c * CL + tid];
#pragma unroll
                for (int p = 0; p < 3; ++p)
                    v[c][p] = mk(o.vinit_re[((size_t)p * nn + k) * B + s], o.vinit_im[((size_t)p * nn + k) * B + s]);
            }
    }
    cx ibo[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
    int it = 0;
    bool conv = false;
    double dmin = INFINITY, err2_last = 0.0;
    unsigned arrivals = 0;   // this member's arrivals (both members: the same sequence)
    for (; alive; ++it) {
        CSTAMP_IT(0);
        // ---- load currents (:106-130)
        cx il[CC][3], ib[CC][3];
#pragma unroll
        for (int c = 0; c < CC; ++c)
#pragma unroll
            for (int p = 0; p < 3; ++p) il[c][p] = il_fast<FULL>(ldx(stg, p * PS + c * CL + tid), v[c][p]);   // 0 on a zeroed phase

        // ---- backward sweep (:134-160): this workgroup's prefix scan of IL
        double sc6[6], pre[6], tot6[6];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            cx acc = il[0][p];
            ib[0][p] = acc;
#pragma unroll
            for (int c = 1; c < CC; ++c) { acc = cadd(acc, il[c][p]); ib[c][p] = acc; }
            sc6[2 * p] = acc.re;
            sc6[2 * p + 1] = acc.im;
        }
        seg_incl_n<64>(sc6);
        if (lane == 63) {
#pragma unroll
            for (int q = 0; q < 6; ++q) wtb[8 * wv + q] = sc6[q];
        }
        __syncthreads();
        wave_prefix<CW, true>(wtb, wv, lane, pre, tot6);
        cx exl[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            exl[p] = csub(mk(pre[2 * p] + sc6[2 * p], pre[2 * p + 1] + sc6[2 * p + 1]), ib[CC - 1][p]);
#pragma unroll
            for (int c = 0; c < CC; ++c) ib[c][p] = cadd(exl[p], ib[c][p]);   // this workgroup's Einc
        }
        // the owned gathered entries (local values), then the exchange: the whole
        // backward array in X, workgroup 1's entries carried by workgroup 0's total
#pragma unroll
        for (int c = 0; c < CC; ++c) {
            const int ci = ci_store_b(si[c]);
            if (ci >= 0) {
#pragma unroll
                for (int p = 0; p < 3; ++p) stx(X, p * XC + ci, ib[c][p]);
            }
        }
        arrivals += 2;
        CSTAMP_IT(1);
        alive = coop_exchange(X, XC, rs, 8 * AH, 0, nbc, f.nb_split, g, tot6, tt, cnt, arrivals, err, flag, f.coop_spin) &&
                alive;
        CSTAMP_IT(2);
        cx tot[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            tot[p] = mk(tt[2 * p] + tt[6 + 2 * p], tt[2 * p + 1] + tt[6 + 2 * p + 1]);   // Ib(0), the same on both sides
            // Ib = Einc[last] - Eexc; Eexc of slot c = Einc of slot c-1, of slot 0 the lane's prefix
            const cx carry = g ? mk(tt[2 * p], tt[2 * p + 1]) : mk(0.0, 0.0);
            cx eprev = cadd(exl[p], carry);
#pragma unroll
            for (int c = 0; c < CC; ++c) {
                const cx e = cadd(ib[c][p], carry);
                ib[c][p] = csub(ldx(X, p * XC + ci_last(si[c])), eprev);
                eprev = e;
            }
        }

        // ---- convergence on the substation branch (:199-217), compared as squares
        double err2 = 0.0;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const double dr = tot[p].re - ibo[p].re, di = tot[p].im - ibo[p].im;
            err2 = fmax(err2, fma(dr, dr, di * di));
            ibo[p] = tot[p];
        }
        conv = __builtin_amdgcn_readfirstlane(err2 < f.eps * f.eps ? 1 : 0) != 0;
        const bool fin = conv || it == f.mxitr - 1 || !alive;   // (!alive: an exchange gave up)
        if (fin) err2_last = err2;
        if (o.flag_count) {   // the convergence guard (fpf_wblk.hip)
            const double e2 = f.eps * f.eps, dd = fabs(err2 - e2);
            if (dd <= 0x1p-9 * e2) dmin = fmin(dmin, dd);
        }

        // ---- branch drops lng * (Ib . Zl) (:163-178)
        cx gd[CC][3];
        double lp[3] = {0.0, 0.0, 0.0};
        if (f.temp_sym) {
#pragma unroll
            for (int c = 0; c < CC; ++c) {
                const int czc = (int)(sx[c] >> 23) * 4;
                const double lgc = f.slot_lng[so + c * CL + tid];
                const cx m = ldx(zc, czc + 3);
                const cx sm = cadd(cadd(ib[c][0], ib[c][1]), ib[c][2]);
                const cx ms = mk(fma(m.re, sm.re, -(m.im * sm.im)), fma(m.re, sm.im, m.im * sm.re));
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const cx d = ldx(zc, czc + a);
                    const cx bb = ib[c][a];
                    gd[c][a] = mk(lgc * fma(d.re, bb.re, fma(-d.im, bb.im, ms.re)),
                                  lgc * fma(d.re, bb.im, fma(d.im, bb.re, ms.im)));
                }
            }
        } else {
#pragma unroll
            for (int c = 0; c < CC; ++c) {
                cx tm[9];
#pragma unroll
                for (int j = 0; j < 9; ++j) tm[j] = ldx(zc, (int)(sx[c] >> 23) * 9 + j);
                const double lgc = f.slot_lng[so + c * CL + tid];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    const cx t = drop_col_fma(tm, ib[c][0], ib[c][1], ib[c][2], a);
                    gd[c][a] = mk(lgc * t.re, lgc * t.im);
                }
            }
        }
        if (fin) {   // Re(drop . conj(Ib)) per phase: the VVC loss (fpf_wave.hip: the loss identity)
#pragma unroll
            for (int c = 0; c < CC; ++c)
#pragma unroll
                for (int a = 0; a < 3; ++a)
                    lp[a] = fma(gd[c][a].re, ib[c][a].re, fma(gd[c][a].im, ib[c][a].im, lp[a]));
        }

        CSTAMP_IT(3);
        // ---- forward sweep (:163-195): V = V0 - A, A = Ginc + off(block)
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            cx acc = gd[0][p];
#pragma unroll
            for (int c = 1; c < CC; ++c) { acc = cadd(acc, gd[c][p]); gd[c][p] = acc; }
            sc6[2 * p] = acc.re;
            sc6[2 * p + 1] = acc.im;
        }
        seg_incl_n<64>(sc6);
        if (lane == 63) {
#pragma unroll
            for (int q = 0; q < 6; ++q) wtf[8 * wv + q] = sc6[q];
        }
        __syncthreads();
        wave_prefix<CW, true>(wtf, wv, lane, pre, tot6);
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const cx ex = csub(mk(pre[2 * p] + sc6[2 * p], pre[2 * p + 1] + sc6[2 * p + 1]), gd[CC - 1][p]);
#pragma unroll
            for (int c = 0; c < CC; ++c) gd[c][p] = cadd(ex, gd[c][p]);   // this workgroup's Ginc
        }
#pragma unroll
        for (int c = 0; c < CC; ++c) {
            const int i2 = (int)((sx[c] >> 9) & 16383u) - 1;
            if (i2 >= 0) {
#pragma unroll
                for (int p = 0; p < 3; ++p) stx(X, p * XC + i2, gd[c][p]);
            }
        }
        arrivals += 2;
        CSTAMP_IT(4);
        alive = coop_exchange(X, XC, rs, 8 * AH + 48 * nbc, 128, nfc, f.nf_split, g, tot6, tt + 12, cnt, arrivals, err,
                              flag, f.coop_spin) && alive;
        CSTAMP_IT(5);
        // block offsets, one thread per block: V0 - off(b), off(b) = sum over b's
        // block-ancestor chain of Ginc[tap] - Ginc[first - 1] (block 0: 0)
        if (tid < nblk) {
            cx of[3] = {mk(0, 0), mk(0, 0), mk(0, 0)};
#pragma unroll
            for (int j = 0; j < CBD; ++j) {
                if (j < f.bdepth) {   // uniform; levels past a chain's depth read the zero entry
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        of[p] = cadd(of[p], csub(ldx(X, p * XC + (bp[j] & 0xffff)), ldx(X, p * XC + (bp[j] >> 16))));
                }
                if (j & 1) __builtin_amdgcn_sched_barrier(0);
            }
#pragma unroll
            for (int p = 0; p < 3; ++p) stx(OFF, p * nblk + tid, csub(ldx(V0S, p), of[p]));
        }
        __syncthreads();
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const cx carry = g ? mk(tt[12 + 2 * p], tt[12 + 2 * p + 1]) : mk(0.0, 0.0);
#pragma unroll
            for (int c = 0; c < CC; ++c) {
                const cx vr = csub(ldx(OFF, p * nblk + (int)(sx[c] & 511u)), cadd(gd[c][p], carry));
                v[c][p] = (FULL && ((si[c] >> p) & 1)) ? mk(0.0, 0.0) : vr;   // phase zeroing (:180-192)
            }
        }

        CSTAMP_IT(6);
        if (fin) {
            // ---- the last sweep: V (and the full outputs) of this workgroup's nodes
            // straight from registers, its part of the loss and of the V extremes
            double mn = INFINITY, mx = -INFINITY;
#pragma unroll
            for (int c = 0; c < CC; ++c) {
                if ((si[c] >> 3) & 1) {
                    const int k = f.slot_node[so + c * CL + tid];
#pragma unroll
                    for (int p = 0; p < 3; ++p) {
                        if (FULL) {
                            emit_full(o, f.s3, nn, B, k, p, (size_t)s, v[c][p], il[c][p], ib[c][p]);
                        } else {
                            const size_t o3 = o.smaj ? (size_t)s * 3 * nn + (size_t)p * nn + k : ((size_t)p * nn + k) * B + s;
                            if (o.v_re) o.v_re[o3] = v[c][p].re;
                            if (o.v_im) o.v_im[o3] = v[c][p].im;
                        }
                        const double m2 = fma(v[c][p].re, v[c][p].re, v[c][p].im * v[c][p].im);
                        mn = fmin(mn, m2);
                        mx = fmax(mx, m2);
                    }
                }
            }
            double xl = lp[0] + lp[1] + lp[2];
            if (FULL && f.has_mask) {
                // zeroed phases: the reference's loss over PQL (the loss identity needs
                // every phase live): this workgroup's part of sum Re(V conj(IL)); |V| of
                // its nodes to the scenario's scratch row for the general V_abc_list
                // extremes (workgroup 0 ranks the whole feeder after the last exchange)
                double *const xv = f.xvm + (size_t)slot * 3 * nn;
                xl = 0.0;
#pragma unroll
                for (int c = 0; c < CC; ++c) {
                    if ((si[c] >> 3) & 1) {
                        const int k = f.slot_node[so + c * CL + tid];
#pragma unroll
                        for (int p = 0; p < 3; ++p) {
                            xl = fma(v[c][p].re, il[c][p].re, fma(v[c][p].im, il[c][p].im, xl));
                            ast(xv + (size_t)p * nn + k, sqrt(fma(v[c][p].re, v[c][p].re, v[c][p].im * v[c][p].im)));
                        }
                    }
                }
            }
            const double x = seg_incl<64>(xl);
            mn = seg_reduce_min<64>(mn);
            mx = seg_reduce_max<64>(mx);
            if (lane == 63) {
                wtb[8 * wv + 6] = x;
                wtf[8 * wv + 6] = mn;
                wtf[8 * wv + 7] = mx;
            }
            break;
        }
    }
    __syncthreads();
    CSTAMP(120);

    // ---- the pair's results: workgroup 1 hands its sums over and leaves;
    // workgroup 0 writes the per-scenario results, releases the area, and joins
    // the fused batch aggregate [loss_sum, vmin, vmax, n_conv, n_nonconv, n_over,
    // n_under, n_scen] (one ticket per scenario, the last folds in scenario order)
    if (g == 1) {
        if (alive && tid == 0) {
            double x = 0.0, mn = INFINITY, mx = -INFINITY, sa = 0.0;
#pragma unroll
            for (int w = 0; w < CW; ++w) {
                x += wtb[8 * w + 6];
                sa += wtb[8 * w + 7];
                mn = fmin(mn, wtf[8 * w + 6]);
                mx = fmax(mx, wtf[8 * w + 7]);
            }
            ast(A + 40, x);
            ast(A + 41, mn);
            ast(A + 42, mx);
            ast(A + 43, sa);
        }
        if (alive) coop_arrive(cnt, 0, err, flag, f.coop_spin, false);
        return;
    }
    if (alive) alive = coop_arrive(cnt, arrivals + 2, err, flag, f.coop_spin, true);
    CSTAMP(121);
    if (FULL && f.has_mask) {
        // ---- zeroed phases, the general V_abc_list (V_abc_list.cpp:7-81,
        // VoltVarCtrl.cpp:1201-1207): per phase the first K_p nonzero |V| in node
        // order, zero padded.  Both workgroups' |V| into this workgroup's LDS (Sld
        // is dead; every load in flight), then one wave per phase ranks 64 nodes a
        // step by ballot; also min over every nonzero |V|^2 (the guard band)
        double *const mag = (double *)stg;   // [3][nn]
        double *const xv = f.xvm + (size_t)slot * 3 * nn;
        for (int i0 = 0; i0 < 3 * nn; i0 += 8 * CL) {
            double r[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * CL + tid;
                r[u] = i < 3 * nn ? ald(xv + i) : 0.0;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = i0 + u * CL + tid;
                if (i < 3 * nn) mag[i] = r[u];
            }
        }
        __syncthreads();
        double mz = INFINITY;
        for (int p = wv; p < 3; p += CW) {
            const int K = f.K[p];
            int cntk = 0;
            double mn = INFINITY, mx = -INFINITY;
            for (int k0 = 0; k0 < nn; k0 += 64) {
                const int k = k0 + lane;
                double m = 0.0;
                if (k < nn) {
                    if (k == 0) {
                        const cx v0p = ldx(V0S, p);
                        m = sqrt(fma(v0p.re, v0p.re, v0p.im * v0p.im));
                    } else {
                        m = mag[p * nn + k];
                    }
                }
                const bool nz = k < nn && m != 0.0;
                if (nz) mz = fmin(mz, m * m);
                const unsigned long long bal = __ballot(nz);
                const int rank = cntk + __popcll(bal & ((1ull << lane) - 1ull));
                if (nz && rank < K) { mn = fmin(mn, m); mx = fmax(mx, m); }
                cntk += __popcll(bal);
            }
            if (cntk < K) { mn = fmin(mn, 0.0); mx = fmax(mx, 0.0); }
            mn = seg_reduce_min<64>(mn);
            mx = seg_reduce_max<64>(mx);
            if (lane == 63) {
                tt[2 * p] = mn;
                tt[2 * p + 1] = mx;
            }
        }
        mz = seg_reduce_min<64>(mz);
        if (lane == 63) tt[8 + wv] = mz;
        __syncthreads();
    }
    const bool agg = o.agg != nullptr;
    if (tid == 0) {
        double x = 0.0, mn = INFINITY, mx = -INFINITY, sa = 0.0;
#pragma unroll
        for (int w = 0; w < CW; ++w) {
            x += wtb[8 * w + 6];
            sa += wtb[8 * w + 7];
            mn = fmin(mn, wtf[8 * w + 6]);
            mx = fmax(mx, wtf[8 * w + 7]);
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {   // the substation row
            const cx v0p = ldx(V0S, p);
            const double m2 = fma(v0p.re, v0p.re, v0p.im * v0p.im);
            mn = fmin(mn, m2);
            mx = fmax(mx, m2);
        }
        if (alive) {
            x += ald(A + 40);
            mn = fmin(mn, ald(A + 41));
            mx = fmax(mx, ald(A + 42));
            sa += ald(A + 43);
            // release the area: the count back to 0, then the generation
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(gen, want + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            // an exchange gave up (the launch's error word is set): the scenario's
            // status is FPF_EXCHANGE_FAILED, never a non-convergence, and the
            // feeder's sticky word (host memory) tells the host API
            conv = false;
            if (f.xerr_host) __hip_atomic_store(f.xerr_host, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        double m2min = mn;
        if (FULL && f.has_mask) {
            // PQb(0).re - sum_k PQL(k).re, V0 conj(Ib(0)) of the last sweep (fpf_wblk.hip)
            double sb0 = 0.0;
#pragma unroll
            for (int p = 0; p < 3; ++p) sb0 += cmul(cmul(ldx(V0S, p), mk(f.s3, 0.0)), cconj(ibo[p])).re;
            x = sb0 - f.s3 * x;
            mn = fmin(fmin(tt[0], tt[2]), tt[4]);
            mx = fmax(fmax(tt[1], tt[3]), tt[5]);
            m2min = INFINITY;
#pragma unroll
            for (int w = 0; w < CW; ++w) m2min = fmin(m2min, tt[8 + w]);
        } else {
            x *= f.s3;
            mn = sqrt(mn);
            mx = sqrt(mx);
        }
        if (o.iters) o.iters[s] = it + 1;
        if (o.status) o.status[s] = conv ? 0 : (alive ? 1 : 3);
        if (o.loss) o.loss[s] = x;
        if (o.errmx) o.errmx[s] = sqrt(err2_last);
        if (o.flag_count) {
            // the guard band (fpf_wblk.hip), over both workgroups' loads
            bool near = false;
            if (dmin < INFINITY) {
                const double tau = 1.25 * f.guard_k * 1.4142135623730951 * sa / sqrt(m2min);
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
            if (FULL) {
                emit_full(o, f.s3, nn, B, 0, p, (size_t)s, v0p, mk(0, 0), ibo[p]);
            } else {
                const size_t o3 = o.smaj ? (size_t)s * 3 * nn + (size_t)p * nn : (size_t)p * nn * B + s;
                if (o.v_re) o.v_re[o3] = v0p.re;
                if (o.v_im) o.v_im[o3] = v0p.im;
            }
            if (o.s_in) {   // PQb row 0: (bkva/3) V0 conj(Ib(0))  (:242-244)
                const cx sbv = cmul(cmul(v0p, mk(f.s3, 0.0)), cconj(ibo[p]));
                o.s_in[(size_t)(2 * p) * B + s] = sbv.re;
                o.s_in[(size_t)(2 * p + 1) * B + s] = sbv.im;
            }
        }
        if (agg) {
            const double part[8] = {conv ? x : 0.0, conv ? mn : INFINITY, conv ? mx : -INFINITY, conv ? 1.0 : 0.0,
                                    conv || !alive ? 0.0 : 1.0, conv && mx > f.ub_v ? 1.0 : 0.0, conv && mn < f.lb_v ? 1.0 : 0.0,
                                    1.0};
            double *dst = o.partials + 8 * (size_t)s;
            for (int q = 0; q < 8; ++q) __hip_atomic_store(dst + q, part[q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __asm__ volatile("s_waitcnt vmcnt(0)" ::: "memory");
            const unsigned t = __hip_atomic_fetch_add(o.ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            last_wg = t == (unsigned)B - 1u;
        }
    }
    if (agg) {
        __syncthreads();
        if (last_wg) {
            // thread i folds scenarios i, i + CL, ... in order, then a fixed tree
            double a[8] = {0, INFINITY, -INFINITY, 0, 0, 0, 0, 0};
            for (int j = tid; j < B; j += CL) {
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const double r = __hip_atomic_load(o.partials + 8 * (size_t)j + q, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT);
                    a[q] = q == 1 ? fmin(a[q], r) : (q == 2 ? fmax(a[q], r) : a[q] + r);
                }
            }
            double *sh = (double *)stg;   // [8][CL] (Sld is dead; wcoop_lds_bytes covers it)
#pragma unroll
            for (int q = 0; q < 8; ++q) sh[q * CL + tid] = a[q];
            __syncthreads();
            for (int w = CL / 2; w > 0; w >>= 1) {
                if (tid < w) {
                    sh[0 * CL + tid] += sh[0 * CL + tid + w];
                    sh[1 * CL + tid] = fmin(sh[1 * CL + tid], sh[1 * CL + tid + w]);
                    sh[2 * CL + tid] = fmax(sh[2 * CL + tid], sh[2 * CL + tid + w]);
#pragma unroll
                    for (int q = 3; q < 8; ++q) sh[q * CL + tid] += sh[q * CL + tid + w];
                }
                __syncthreads();
            }
            if (tid < 8) o.agg[tid] = sh[tid * CL];
            if (tid == 0) __hip_atomic_store(o.ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (tid == 0 && o.flag_out)
                *o.flag_out = __hip_atomic_load(o.flag_count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

size_t wcoop_lds_bytes(const WaveDev &w) {
    const size_t ntz = w.temp_sym ? 4 : 9, xc = (size_t)w.ncomp + 1;
    return 16 * ((size_t)w.ncode * ntz + 3 * ((size_t)CC * CL + 1) + 3 * xc + 3 * (size_t)w.nblk + 4) +
           2 * 8 * CW * 8 + 24 * 8 + 16;
}

hipError_t launch_wcoop(const WaveDev &w, int n_scen, const double *pq, const OutDev &o, hipStream_t st) {
    if (w.coop != 2 || w.wps != CW || w.C != CC || w.nblk > CL || w.bdepth > CBD || !w.xch || !w.xsync ||
        (w.has_mask && !w.xvm) || w.has_rel)
        return hipErrorInvalidValue;
    // the full-output variant keeps IL and Ib of the last sweep, and the zeroed-phase paths
    const bool full = o.vpolar || o.pqb || o.pql || w.has_mask;
    auto k = full ? dpf_wcoop_kernel<true> : dpf_wcoop_kernel<false>;
    static std::mutex mu;
    static std::set<std::array<int, 2>> attr_done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    {
        std::lock_guard<std::mutex> lk(mu);
        const std::array<int, 2> key = {dev, (int)full};
        if (!attr_done.count(key)) {
            hipFuncAttributes fa{};
            hipError_t e = hipFuncGetAttributes(&fa, (const void *)k);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024 - (int)fa.sharedSizeBytes);
            if (e != hipSuccess) return e;
            attr_done.insert(key);
        }
    }
    // arrival counts, generations and the error word start at 0 every launch
    hipError_t e = hipMemsetAsync(w.xsync, 0, sizeof(unsigned) * (2 * (size_t)w.coop_nslot + 16), st);
    if (e != hipSuccess) return e;
    if (n_scen <= 0) return hipSuccess;
    const unsigned grid = 16u * (unsigned)((n_scen + 7) / 8);   // scenario t: workgroups 16 (t / 8) + (t % 8) + {0, 8}
    hipLaunchKernelGGL(k, dim3(grid), dim3(CL), wcoop_lds_bytes(w), st, w, n_scen, pq, o);
    return hipGetLastError();
}

}  // namespace fpf
