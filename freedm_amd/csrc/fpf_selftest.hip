// fpf_selftest.hip -- on-device self-test of the arithmetic the kernels rely on.
//
// The tiled kernel replaces the compiler's a / b sequence by dv_div with a
// reciprocal shared between the two quotients of Smith's method (fpf_math.hpp),
// claiming the same bits whenever dv_in_range holds.  This kernel checks that
// claim on n seeded operand pairs spread over the whole guarded exponent range
// (plus zeros and signs), for the real division and for the complex division
// cdiv_rr against cdiv (libgcc __divdc3), bit for bit.
#include "../../include/freedm_pf.h"

#include <hip/hip_runtime.h>

#include "fpf_internal.h"
#include "fpf_math.hpp"

#pragma clang fp contract(off)

namespace fpf {
namespace {

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// an operand: sign, exponent in [-300, 300) (or near 0 / 1 for the p.u. regime),
// random mantissa; 1 in 64 is zero
__device__ __forceinline__ double operand(unsigned long long h) {
    if ((h & 63) == 0) return (h & 64) ? -0.0 : 0.0;
    const int mode = (h >> 6) & 3;
    int e;
    if (mode == 0) e = (int)((h >> 8) % 600) - 300;
    else e = (int)((h >> 8) % 24) - 12;                // voltages / loads in p.u.
    const double m = 1.0 + (double)((h >> 20) & ((1ull << 44) - 1)) * 0x1p-44;
    const double v = ldexp(m, e);
    return (h >> 7) & 1 ? -v : v;
}

__global__ void selftest_kernel(long n, unsigned long long seed, unsigned long long *bad) {
    unsigned long long nb = 0;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
        const unsigned long long h = mix(seed ^ (unsigned long long)i);
        const double a = operand(mix(h + 1)), b = operand(mix(h + 2)), c = operand(mix(h + 3)),
                     d = operand(mix(h + 4));
        if (b != 0.0) {
            const double q0 = a / b, q1 = dv_div(a, b, dv_rcp(b));
            if (__double_as_longlong(q0) != __double_as_longlong(q1)) ++nb;
        }
        if (c != 0.0 || d != 0.0) {
            const cx r0 = cdiv(mk(a, b), mk(c, d)), r1 = cdiv_rr(mk(a, b), mk(c, d));
            if (__double_as_longlong(r0.re) != __double_as_longlong(r1.re) ||
                __double_as_longlong(r0.im) != __double_as_longlong(r1.im))
                ++nb;
        }
    }
    if (nb) atomicAdd(bad, nb);
}

}  // namespace
}  // namespace fpf

extern "C" long fpf_selftest_division(int device, long n, unsigned long seed) {
    if (n < 0) return FPF_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return FPF_ERR_HIP;
    unsigned long long *d = nullptr, h = 0;
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return FPF_ERR_HIP;
    hipError_t e = hipMemset(d, 0, sizeof(h));
    if (e == hipSuccess) {
        hipLaunchKernelGGL(fpf::selftest_kernel, dim3(1024), dim3(256), 0, nullptr, n, (unsigned long long)seed, d);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(&h, d, sizeof(h), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    return e == hipSuccess ? (long)h : FPF_ERR_HIP;
}
