// fpf_wave_common.h -- device helpers shared by the wave kernel (fpf_wave.hip)
// and the wave-block kernel (fpf_wblk.hip): fp64 DPP scans within a wavefront,
// LDS complex loads/stores, the fast load current, the full-output emitter,
// the packed per-slot info and the XCD-aware tile order.
#pragma once
#include "fpf_internal.h"
#include "fpf_math.hpp"

namespace fpf {

namespace {

// DPP move of one fp64 value (two 32-bit halves); lanes without a source read 0
template <int CTRL, int RM, int BM>
__device__ __forceinline__ double dpp_d(double x) {
    const int lo = __double2loint(x), hi = __double2hiint(x);
    const int l2 = __builtin_amdgcn_update_dpp(0, lo, CTRL, RM, BM, true);
    const int h2 = __builtin_amdgcn_update_dpp(0, hi, CTRL, RM, BM, true);
    return __hiloint2double(h2, l2);
}

// inclusive scan within segments of L lanes: row_shr 1, 2, 4, 8 within rows of
// 16, then row_bcast:15 (rows 1, 3) for L >= 32 and row_bcast:31 (rows 2, 3) for L = 64
template <int L>
__device__ __forceinline__ double seg_incl(double x) {
    x += dpp_d<0x111, 0xf, 0xf>(x);
    x += dpp_d<0x112, 0xf, 0xf>(x);
    x += dpp_d<0x114, 0xf, 0xf>(x);
    x += dpp_d<0x118, 0xf, 0xf>(x);
    if (L >= 32) x += dpp_d<0x142, 0xa, 0xf>(x);
    if (L >= 64) x += dpp_d<0x143, 0xc, 0xf>(x);
    return x;
}

// N independent scans step by step, so their DPP/add chains interleave
template <int L, int N>
__device__ __forceinline__ void seg_incl_n(double (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_d<0x111, 0xf, 0xf>(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_d<0x112, 0xf, 0xf>(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_d<0x114, 0xf, 0xf>(x[i]);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] += dpp_d<0x118, 0xf, 0xf>(x[i]);
    if (L >= 32) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] += dpp_d<0x142, 0xa, 0xf>(x[i]);
    }
    if (L >= 64) {
#pragma unroll
        for (int i = 0; i < N; ++i) x[i] += dpp_d<0x143, 0xc, 0xf>(x[i]);
    }
}

// DPP move of a 32-bit int; lanes without a source read 0
template <int CTRL, int RM, int BM>
__device__ __forceinline__ int dpp_i(int x) {
    return __builtin_amdgcn_update_dpp(0, x, CTRL, RM, BM, true);
}

// one Hillis-Steele step of a segmented scan: (x, f) <- (s, fs) o (x, f) with
// (a, g) o (b, h) = (h ? b : a + b, g | h), (s, fs) the DPP source
template <int CTRL, int RM, int BM, int N>
__device__ __forceinline__ void segf_step(double (&x)[N], int &f) {
    double sv[N];
#pragma unroll
    for (int i = 0; i < N; ++i) sv[i] = dpp_d<CTRL, RM, BM>(x[i]);
    const int fs = dpp_i<CTRL, RM, BM>(f);
#pragma unroll
    for (int i = 0; i < N; ++i) x[i] = f ? x[i] : x[i] + sv[i];
    f |= fs;
}

// segmented inclusive scan over the 64 lanes of a wavefront (f != 0: a segment
// head lies in this lane's part), the steps of seg_incl_n
template <int N>
__device__ __forceinline__ void segf_incl64(double (&x)[N], int &f) {
    segf_step<0x111, 0xf, 0xf>(x, f);
    segf_step<0x112, 0xf, 0xf>(x, f);
    segf_step<0x114, 0xf, 0xf>(x, f);
    segf_step<0x118, 0xf, 0xf>(x, f);
    segf_step<0x142, 0xa, 0xf>(x, f);
    segf_step<0x143, 0xc, 0xf>(x, f);
}

// the value of the segment's last lane
template <int L>
__device__ __forceinline__ double seg_last(double x, int seg) {
    if (L == 64) {
        const int lo = __builtin_amdgcn_readlane(__double2loint(x), 63);
        const int hi = __builtin_amdgcn_readlane(__double2hiint(x), 63);
        return __hiloint2double(hi, lo);
    }
    return __shfl(x, seg * L + L - 1, 64);
}

template <int L>
__device__ __forceinline__ double seg_sum(double x) {
#pragma unroll
    for (int m = L / 2; m >= 1; m >>= 1) x += __shfl_xor(x, m, 64);
    return x;
}
template <int L>
__device__ __forceinline__ double seg_min(double x) {
#pragma unroll
    for (int m = L / 2; m >= 1; m >>= 1) x = fmin(x, __shfl_xor(x, m, 64));
    return x;
}
template <int L>
__device__ __forceinline__ double seg_max(double x) {
#pragma unroll
    for (int m = L / 2; m >= 1; m >>= 1) x = fmax(x, __shfl_xor(x, m, 64));
    return x;
}

// LDS ordering between the lanes of one wave: a wave's DS operations execute in
// order; the fence keeps the compiler from moving them across
__device__ __forceinline__ void wfence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

__device__ __forceinline__ cx ldx(const double2 *X, int i) {
    const double2 v = X[i];
    return mk(v.x, v.y);
}
__device__ __forceinline__ void stx(double2 *X, int i, cx v) { X[i] = make_double2(v.re, v.im); }

// IL = conj(S/V) = conj(S) V / |V|^2 with one refined reciprocal; 0 when V == 0
// (:117-125) -- a voltage is exactly 0 only on a zeroed phase, so feeders
// without zeroed phases (ZERO = false) skip the test
template <bool ZERO>
__device__ __forceinline__ cx il_fast(cx s, cx v) {
    const double d2 = fma(v.re, v.re, v.im * v.im);
    // v_rcp_f64 and one Newton step (the hardware reciprocal is good to ~2^-26,
    // one step squares the error)
    double r = __builtin_amdgcn_rcp(d2);
    r = fma(r, fma(-d2, r, 1.0), r);
    if (ZERO) r = d2 == 0.0 ? 0.0 : r;
    return mk(fma(s.re, v.re, s.im * v.im) * r, fma(s.re, v.im, -(s.im * v.re)) * r);
}

// the wavefront totals [W][8] (6 used: re/im per phase) summed over the waves
// before wave wv (pre) and over all waves (tot): lane j < W reads wave j's
// totals, a DPP scan over those lanes, the sums read back as wave-uniform
// values.  Every wave computes the same scan, so tot (Ib(0) in the backward
// sweep) is the same in every wave of the workgroup.
__device__ __forceinline__ double readlane_d(double x, int l) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(x), l);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(x), l);
    return __hiloint2double(hi, lo);
}
template <int W, bool TOT>
__device__ __forceinline__ void wave_prefix(const double *wt, int wv, int lane, double (&pre)[6], double (&tot)[6]) {
    const int j = lane < W ? lane : 0;
    const double2 *t2 = (const double2 *)(wt + 8 * j);
    const double2 a = t2[0], b = t2[1], c = t2[2];
    double t[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
#pragma unroll
    for (int q = 0; q < 6; ++q) t[q] = lane < W ? t[q] : 0.0;
    if (W > 1) {
#pragma unroll
        for (int q = 0; q < 6; ++q) t[q] += dpp_d<0x111, 0xf, 0xf>(t[q]);
    }
    if (W > 2) {
#pragma unroll
        for (int q = 0; q < 6; ++q) t[q] += dpp_d<0x112, 0xf, 0xf>(t[q]);
    }
    if (W > 4) {
#pragma unroll
        for (int q = 0; q < 6; ++q) t[q] += dpp_d<0x114, 0xf, 0xf>(t[q]);
    }
    if (W > 8) {
#pragma unroll
        for (int q = 0; q < 6; ++q) t[q] += dpp_d<0x118, 0xf, 0xf>(t[q]);
    }
    const int wu = __builtin_amdgcn_readfirstlane(wv);
#pragma unroll
    for (int q = 0; q < 6; ++q) {
        pre[q] = wu == 0 ? 0.0 : readlane_d(t[q], wu - 1);
        if (TOT) tot[q] = readlane_d(t[q], W - 1);
    }
}
// wave_prefix for a scan segmented at heads: wt[8 j + 6] != 0 marks a wave
// with a head; pre = the segmented combine of waves 0 .. wv-1 (0 for wave 0)
template <int W>
__device__ __forceinline__ void wave_prefix_seg(const double *wt, int wv, int lane, double (&pre)[6]) {
    const int j = lane < W ? lane : 0;
    const double2 *t2 = (const double2 *)(wt + 8 * j);
    const double2 a = t2[0], b = t2[1], c = t2[2], d = t2[3];
    double t[6] = {a.x, a.y, b.x, b.y, c.x, c.y};
    int fl = lane < W && d.x != 0.0 ? 1 : 0;
#pragma unroll
    for (int q = 0; q < 6; ++q) t[q] = lane < W ? t[q] : 0.0;
    if (W > 1) segf_step<0x111, 0xf, 0xf>(t, fl);
    if (W > 2) segf_step<0x112, 0xf, 0xf>(t, fl);
    if (W > 4) segf_step<0x114, 0xf, 0xf>(t, fl);
    if (W > 8) segf_step<0x118, 0xf, 0xf>(t, fl);
    const int wu = __builtin_amdgcn_readfirstlane(wv);
#pragma unroll
    for (int q = 0; q < 6; ++q) pre[q] = wu == 0 ? 0.0 : readlane_d(t[q], wu - 1);
}

// index of the (Re, Im) field pair of node k, phase p in a [6][Nn] output
// (Vpolar / PQb / PQL): [field][row][B], or [B][field][row] (o.smaj)
__device__ __forceinline__ size_t out6(const OutDev &o, int nn, int B, int k, int p, size_t s) {
    return o.smaj ? s * 6 * nn + (size_t)(2 * p) * nn + k : ((size_t)(2 * p) * nn + k) * B + s;
}
__device__ __forceinline__ size_t out6_im(const OutDev &o, int nn, int B) { return o.smaj ? (size_t)nn : (size_t)nn * B; }

// Outputs of node k, phase p (DPF_return7.cpp:222-253); returns (Re SL, |V|)
__device__ __forceinline__ double2 emit_full(const OutDev &o, double s3, int nn, int B, int k, int p, size_t s, cx v,
                                             cx il, cx ib) {
    const cx sv = cmul(v, mk(s3, 0.0));
    const cx sl = cmul(sv, cconj(il));
    const cx sb = cmul(sv, cconj(ib));
    const double mag = sqrt(fma(v.re, v.re, v.im * v.im));
    // [field][row][B], or [B][field][row] (o.smaj)
    const size_t o6 = out6(o, nn, B, k, p, s), o6i = o6 + out6_im(o, nn, B);
    const size_t o3 = o.smaj ? s * 3 * nn + (size_t)p * nn + k : ((size_t)p * nn + k) * B + s;
    if (o.vpolar) { o.vpolar[o6] = mag; o.vpolar[o6i] = polar_angle(v, p); }
    if (o.pqb) { o.pqb[o6] = sb.re; o.pqb[o6i] = sb.im; }
    if (o.pql) { o.pql[o6] = sl.re; o.pql[o6i] = sl.im; }
    if (o.v_re) o.v_re[o3] = v.re;
    if (o.v_im) o.v_im[o3] = v.im;
    return make_double2(sl.re, mag);
}
}  // namespace

// ---- the convergence guard of the fast kernels (fpf_api.cpp: guard_factor)
// Append scenario s to the batch's flag list (agent-scope stores: a later
// kernel reads it) -- or, in the wave kernel's local mode (OutDev::fix_dev, a
// solve without an aggregate), to its workgroup's own list in LDS.
__device__ __forceinline__ void guard_flag(const OutDev &o, int s, int *local_n, int *local_ids) {
    if (o.fix_dev) {
        local_ids[atomicAdd(local_n, 1)] = s;
        return;
    }
    const unsigned q = __hip_atomic_fetch_add(o.flag_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(o.flag_ids + q, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// packed per-slot info (fpf_api.cpp: analyse_wave)
__device__ __forceinline__ int si_mask(int x) { return x & 7; }
__device__ __forceinline__ bool si_valid(int x) { return (x >> 3) & 1; }
__device__ __forceinline__ int si_store_b(int x) { return ((x >> 4) & 511) - 1; }   // -1: not gathered
__device__ __forceinline__ int si_last(int x) { return (x >> 13) & 511; }
__device__ __forceinline__ int si_store_f(int x) { return ((x >> 22) & 511) - 1; }  // -1: not gathered
__device__ __forceinline__ bool si_head(int x) { return x < 0; }   // bit 31: a block head (wave-block kernel)

// segment-wide reductions by the DPP scan pattern; the segment's last lane holds
// the result.  Lanes without a source keep +inf (bound_ctrl off, old = +inf).
template <int CT>
__device__ __forceinline__ double dpp_min_step(double v) {
    constexpr int RM = CT == 0x142 ? 0xa : (CT == 0x143 ? 0xc : 0xf);
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CT, RM, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0x7ff00000, __double2hiint(v), CT, RM, 0xf, false);
    return fmin(v, __hiloint2double(hi, lo));
}
template <int L>
__device__ __forceinline__ double seg_reduce_min(double x) {
    x = dpp_min_step<0x111>(x);
    x = dpp_min_step<0x112>(x);
    x = dpp_min_step<0x114>(x);
    x = dpp_min_step<0x118>(x);
    if (L >= 32) x = dpp_min_step<0x142>(x);
    if (L >= 64) x = dpp_min_step<0x143>(x);
    return x;
}
template <int L>
__device__ __forceinline__ double seg_reduce_max(double x) { return -seg_reduce_min<L>(-x); }

// (field, row) of a flat index f * n + r, advanced by a fixed step without a
// division per step (the step split once as a * n + b): the staging and
// write-out loops visit a thread's elements NT (or 2 NT) indices apart
struct RowWalk {
    int fq, rr, a, b, n;
    __device__ __forceinline__ void init(int fr, int step, int n_) {
        n = n_;
        fq = fr / n;
        rr = fr - fq * n;
        a = step / n;
        b = step - a * n;
    }
    __device__ __forceinline__ void next() {
        rr += b;
        fq += a;
        if (rr >= n) { rr -= n; ++fq; }
    }
};

// tile of block b: the first 8 * (G / 8) blocks are dealt so that blocks on one
// XCD (b, b + 8, ...) take consecutive tiles; the remainder keeps b
__device__ __forceinline__ int xcd_tile(int b, int G) {
    const int per = G >> 3;
    return b < (per << 3) ? (b & 7) * per + (b >> 3) : b;
}

}  // namespace fpf
