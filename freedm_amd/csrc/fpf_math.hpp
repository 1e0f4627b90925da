// fpf_math.hpp -- complex-fp64 arithmetic with the reference's operation order
// (SURVEY.md 8(a) A9), for host precomputation and gfx950 device code alike.
// The library is compiled with -ffp-contract=off: the reference is ISO C++98
// built without FMA contraction, and bit-exact V needs the same roundings.
#pragma once
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#include <math.h>
#endif

#pragma clang fp contract(off)

namespace fpf {

struct cx {
    double re, im;
};

__host__ __device__ __forceinline__ cx mk(double r, double i) { cx z; z.re = r; z.im = i; return z; }
__host__ __device__ __forceinline__ cx cadd(cx a, cx b) { return mk(a.re + b.re, a.im + b.im); }
__host__ __device__ __forceinline__ cx csub(cx a, cx b) { return mk(a.re - b.re, a.im - b.im); }
// GCC's inline expansion of std::complex<double> * std::complex<double>
__host__ __device__ __forceinline__ cx cmul(cx x, cx y) {
    return mk(x.re * y.re - x.im * y.im, x.re * y.im + x.im * y.re);
}
__host__ __device__ __forceinline__ cx cconj(cx a) { return mk(a.re, -a.im); }

// libgcc __divdc3 (Smith's method): what GCC emits for std::complex<double> '/'
__host__ __device__ __forceinline__ cx cdiv(cx x, cx y) {
    const double a = x.re, b = x.im, c = y.re, d = y.im;
    cx r;
    if (fabs(c) < fabs(d)) {
        const double ratio = c / d;
        const double denom = (c * ratio) + d;
        r.re = ((a * ratio) + b) / denom;
        r.im = ((b * ratio) - a) / denom;
    } else {
        const double ratio = d / c;
        const double denom = (d * ratio) + c;
        r.re = ((b * ratio) + a) / denom;
        r.im = (b - (a * ratio)) / denom;
    }
    return r;
}

// ---- correctly rounded fp64 division with a shared reciprocal ----------------
// hipcc lowers a / b to div_scale(b), rcp, two Newton steps, q = a*y,
// r = fma(-b, q, a), div_fmas(r, y, q), div_fixup.  When every operand is zero
// or has an exponent in [-300, 300], div_scale scales nothing, div_fmas is the
// plain fma and div_fixup returns its input except for a zero numerator (the
// signed zero a*y), so dv_div below yields the same bits as a / b -- and one
// reciprocal serves both quotients of Smith's method.  cdiv_rr is __divdc3 on
// that division; callers guard its range with dv_in_range (checked on the GPU
// against a / b bit for bit, tests/test_gpu_parity.py).
__host__ __device__ __forceinline__ bool dv_in_range(double x) {
    const double ax = fabs(x);
    return ax == 0.0 || (ax >= 0x1p-300 && ax <= 0x1p300);
}
__host__ __device__ __forceinline__ double dv_rcp(double b) {
#ifdef __HIP_DEVICE_COMPILE__
    double y = __builtin_amdgcn_rcp(b);
#else
    double y = 1.0 / b;
#endif
    double e = fma(-b, y, 1.0);
    y = fma(y, e, y);
    e = fma(-b, y, 1.0);
    return fma(y, e, y);
}
__host__ __device__ __forceinline__ double dv_div(double a, double b, double y) {
    const double q = a * y;
    const double r = fma(-b, q, a);
    const double d = fma(r, y, q);
    return a == 0.0 ? q : d;
}
__host__ __device__ __forceinline__ cx cdiv_rr(cx x, cx y) {
    const double a = x.re, b = x.im, c = y.re, d = y.im;
    cx r;
    if (fabs(c) < fabs(d)) {
        const double ratio = dv_div(c, d, dv_rcp(d));
        const double denom = (c * ratio) + d;
        const double yr = dv_rcp(denom);
        r.re = dv_div((a * ratio) + b, denom, yr);
        r.im = dv_div((b * ratio) - a, denom, yr);
    } else {
        const double ratio = dv_div(d, c, dv_rcp(c));
        const double denom = (d * ratio) + c;
        const double yr = dv_rcp(denom);
        r.re = dv_div((b * ratio) + a, denom, yr);
        r.im = dv_div(b - (a * ratio), denom, yr);
    }
    return r;
}
// load current with the shared-reciprocal division; valid when Sld and V are in range
__host__ __device__ __forceinline__ cx load_current_rr(cx s, cx v) {
    if (v.re == 0.0 && v.im == 0.0) return mk(0.0, 0.0);
    return cconj(cdiv_rr(s, v));
}

// ---- fast mode (fpf_opts.exact = 0): the same quantities, fewer roundings -----
// IL = conj(S/V) = (S.re V.re + S.im V.im, S.re V.im - S.im V.re) / |V|^2 with
// one refined reciprocal; a few ulp from __divdc3.  |V|^2 outside
// [2^-600, 2^600] takes the exact path.
__host__ __device__ __forceinline__ cx load_current_fast(cx s, cx v) {
    if (v.re == 0.0 && v.im == 0.0) return mk(0.0, 0.0);
    const double d2 = fma(v.re, v.re, v.im * v.im);
    if (!(d2 >= 0x1p-600 && d2 <= 0x1p600)) return cconj(cdiv(s, v));
    const double r = dv_rcp(d2);
    return mk(fma(s.re, v.re, s.im * v.im) * r, fma(s.re, v.im, -(s.im * v.re)) * r);
}
// column a of Ib(1x3) . TEMP(3x3) as fused complex multiply-adds
__host__ __device__ __forceinline__ cx drop_col_fma(const cx tm[9], const cx ib0, const cx ib1, const cx ib2,
                                                    int a) {
    const cx t0 = tm[0 * 3 + a], t1 = tm[1 * 3 + a], t2 = tm[2 * 3 + a];
    double re = fma(-t0.im, ib0.im, t0.re * ib0.re);
    double im = fma(t0.im, ib0.re, t0.re * ib0.im);
    re = fma(t1.re, ib1.re, re);
    re = fma(-t1.im, ib1.im, re);
    im = fma(t1.re, ib1.im, im);
    im = fma(t1.im, ib1.re, im);
    re = fma(t2.re, ib2.re, re);
    re = fma(-t2.im, ib2.im, re);
    im = fma(t2.re, ib2.im, im);
    im = fma(t2.im, ib2.re, im);
    return mk(re, im);
}

// Load current of one phase, DPF_return7.cpp:117-125:
//   abs(v) == 0 ? 0 : conj(S / v)
__host__ __device__ __forceinline__ cx load_current(cx s, cx v) {
    if (v.re == 0.0 && v.im == 0.0) return mk(0.0, 0.0);
    return cconj(cdiv(s, v));
}

// TEMP(L,a) = ALPHA * Zt(L,a) with ALPHA = cx(lng,0)*cx(1,0) (Armadillo folds the
// scalar lng into the gemm alpha).  Feeder-static, so the host precomputes it.
__host__ __device__ __forceinline__ cx zgemm_temp(double lng, cx z) {
    const cx alpha = cmul(mk(lng, 0.0), mk(1.0, 0.0));
    return cmul(alpha, z);
}

// Column a of lng * (Ib(1x3) * Zt(3x3)) in reference-BLAS ZGEMM order:
//   C(1,a) = ((0 + TEMP(0,a)*Ib0) + TEMP(1,a)*Ib1) + TEMP(2,a)*Ib2
// t points at the op's 9 interleaved TEMP values, t[2*(L*3+a)] = Re TEMP(L,a).
__host__ __device__ __forceinline__ cx drop_col(const double *t, const cx ib0, const cx ib1,
                                                const cx ib2, int a) {
    cx c = mk(0.0, 0.0);
    c = cadd(c, cmul(mk(t[2 * (0 * 3 + a)], t[2 * (0 * 3 + a) + 1]), ib0));
    c = cadd(c, cmul(mk(t[2 * (1 * 3 + a)], t[2 * (1 * 3 + a) + 1]), ib1));
    c = cadd(c, cmul(mk(t[2 * (2 * 3 + a)], t[2 * (2 * 3 + a) + 1]), ib2));
    return c;
}

// The 9 TEMP values of one branch (t as in drop_col) from global memory.  The
// table pointer arrives through a struct of generic pointers; the explicit
// global address space turns the loads into global_load_dwordx4 (a flat load
// also waits on the LDS counter), issued together ahead of the products.
__device__ __forceinline__ void load_temp(const double *t, cx tm[9]) {
#ifdef __HIP_DEVICE_COMPILE__
    typedef const __attribute__((address_space(1))) double2 gd2;
    gd2 *g = (gd2 *)t;
#else
    const double2 *g = (const double2 *)t;
#endif
#pragma unroll
    for (int i = 0; i < 9; ++i) {
        const double2 v = g[i];
        tm[i] = mk(v.x, v.y);
    }
}

// element i of a double2 table in global memory (global_load_dwordx4, see load_temp)
__device__ __forceinline__ double2 ld_global2(const double *t, int i) {
#ifdef __HIP_DEVICE_COMPILE__
    typedef const __attribute__((address_space(1))) double2 gd2;
    const gd2 *g = (const gd2 *)t;
    const double x = g[i].x, y = g[i].y;
    return make_double2(x, y);
#else
    return ((const double2 *)t)[i];
#endif
}

// drop_col on TEMP values held in registers, tm[L*3 + a] = TEMP(L, a)
__host__ __device__ __forceinline__ cx drop_col_r(const cx tm[9], const cx ib0, const cx ib1, const cx ib2, int a) {
    cx c = mk(0.0, 0.0);
    c = cadd(c, cmul(tm[0 * 3 + a], ib0));
    c = cadd(c, cmul(tm[1 * 3 + a], ib1));
    c = cadd(c, cmul(tm[2 * 3 + a], ib2));
    return c;
}

// Vpolar angle, DPF_return7.cpp:232-235
[[maybe_unused]] static __host__ __device__ __noinline__ double polar_angle(cx v, int phase) {
    double ang = (180.0 / 3.14159265358979323846) * atan(v.im / v.re);
    if (!isfinite(ang)) ang = 0.0;
    if (phase == 1) ang = ang - 180;
    if (phase == 2) ang = ang + 180;
    return ang;
}

}  // namespace fpf
