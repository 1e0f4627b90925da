// fpf_areas_kernels.hip -- the boundary exchange of the multi-area solve
// (fpf_areas.cpp): every kernel is one pass over [field][row][scenario]
// arrays, scenario fastest, one thread per scenario and field -- coalesced,
// HBM-bound, a few KB per scenario per outer iteration.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "fpf_internal.h"

namespace fpf {
namespace {

// dst[f][r][s] = src[f][row[r]][s] (row[r] < 0: a separator row, 0), also into dst2 when given
__global__ void gather_rows_kernel(const double *__restrict__ src, int nl_src, const int32_t *__restrict__ row, int nl,
                                   int B, double *__restrict__ dst, double *__restrict__ dst2) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int fr = blockIdx.y;   // f * nl + r
    if (s >= B) return;
    const int f = fr / nl, r = fr % nl, m = row[r];
    const double x = m < 0 ? 0.0 : src[((size_t)f * nl_src + m) * B + s];
    dst[(size_t)fr * B + s] = x;
    if (dst2) dst2[(size_t)fr * B + s] = x;
}

// The kernels of one outer iteration do nothing once the loop has converged
// (ctl[0] != 0: iterations enqueued before the host looked are no-ops).

// every child row of one area: work[f][lrow_j][s] = base[f][lrow_j][s] + add_j[f][s]
__global__ void add_rows_kernel(double *__restrict__ work, const double *__restrict__ base, int nl, int B, AreaKids k,
                                const int32_t *__restrict__ ctl) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int f = blockIdx.y % 6, j = blockIdx.y / 6;
    if (s >= B || ctl[0]) return;
    const size_t i = ((size_t)f * nl + k.lrow[j]) * B + s;
    work[i] = base[i] + k.ptr[j][(size_t)f * B + s];
}

// every child of one area after its solve: vsrc_j = V(node lb_j) of this area; diff = max move
__global__ void gather_vsrc_all_kernel(const double *__restrict__ v_re, const double *__restrict__ v_im, int nn, int B,
                                       AreaKids k, double *__restrict__ diff, const int32_t *__restrict__ ctl) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B || ctl[0]) return;
    double d = diff[s];
    for (int j = 0; j < k.n; ++j) {
        double *const vsrc = k.ptr[j];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            const double re = v_re[((size_t)p * nn + k.lrow[j]) * B + s], im = v_im[((size_t)p * nn + k.lrow[j]) * B + s];
            d = fmax(d, fmax(fabs(re - vsrc[(size_t)(2 * p) * B + s]), fabs(im - vsrc[(size_t)(2 * p + 1) * B + s])));
            vsrc[(size_t)(2 * p) * B + s] = re;
            vsrc[(size_t)(2 * p + 1) * B + s] = im;
        }
    }
    diff[s] = d;
}

// dst[p][mono[k]][s] = src[p][k][s] for k = k0 .. nn-1
__global__ void scatter_nodes_kernel(const double *__restrict__ src, int nn, int k0, const int32_t *__restrict__ mono,
                                     int nn_dst, int B, double *__restrict__ dst) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int pk = blockIdx.y;   // p * (nn - k0) + (k - k0)
    if (s >= B) return;
    const int p = pk / (nn - k0), k = k0 + pk % (nn - k0), m = mono[k];
    if (m >= 0) dst[((size_t)p * nn_dst + m) * B + s] = src[((size_t)p * nn + k) * B + s];   // m < 0: a pad bus
}

// whole-feeder results from the areas': loss summed, extremes folded, status = worst
__global__ void fold_results_kernel(int B, const double *__restrict__ loss, const double *__restrict__ vmin,
                                    const double *__restrict__ vmax, const int8_t *__restrict__ status, int first,
                                    double *__restrict__ o_loss, double *__restrict__ o_vmin, double *__restrict__ o_vmax,
                                    int8_t *__restrict__ o_status) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    if (first) {
        o_loss[s] = loss[s];
        o_vmin[s] = vmin[s];
        o_vmax[s] = vmax[s];
        o_status[s] = status[s];
    } else {
        o_loss[s] += loss[s];
        o_vmin[s] = fmin(o_vmin[s], vmin[s]);
        o_vmax[s] = fmax(o_vmax[s], vmax[s]);
        o_status[s] = o_status[s] > status[s] ? o_status[s] : status[s];
    }
}

// the end of one outer iteration: the boundary voltages' largest move (the
// first iteration always moves; a single area needs one), then the device-side
// stop -- ctl[0] done, ctl[1] outer iterations run; last = the move
__global__ void check_kernel(double *__restrict__ x, int n, double tol, int single, int32_t *__restrict__ ctl,
                             double *__restrict__ last) {
    if (ctl[0]) return;   // (uniform)
    __shared__ double sh[256];
    double m = 0.0;
    for (int i = threadIdx.x; i < n; i += 256) {
        m = fmax(m, x[i]);
        x[i] = 0.0;   // (the next iteration's diff starts from 0)
    }
    sh[threadIdx.x] = m;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] = fmax(sh[threadIdx.x], sh[threadIdx.x + w]);
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const int outer = ctl[1] + 1;
        ctl[1] = outer;
        *last = sh[0];
        if (single || (outer > 1 && sh[0] <= tol)) ctl[0] = 1;
    }
}

inline dim3 grid(int B, int y) { return dim3((unsigned)((B + 255) / 256), (unsigned)y); }
}  // namespace

hipError_t areas_gather_rows(const double *src, int nl_src, const int32_t *row, int nl, int B, double *dst,
                             double *dst2, hipStream_t st) {
    hipLaunchKernelGGL(gather_rows_kernel, grid(B, 6 * nl), dim3(256), 0, st, src, nl_src, row, nl, B, dst, dst2);
    return hipGetLastError();
}
hipError_t areas_add_rows(double *work, const double *base, int nl, int B, const AreaKids &k, const int32_t *ctl,
                          hipStream_t st) {
    if (k.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(add_rows_kernel, grid(B, 6 * k.n), dim3(256), 0, st, work, base, nl, B, k, ctl);
    return hipGetLastError();
}
hipError_t areas_gather_vsrc_all(const double *v_re, const double *v_im, int nn, int B, const AreaKids &k, double *diff,
                                 const int32_t *ctl, hipStream_t st) {
    if (k.n <= 0) return hipSuccess;
    hipLaunchKernelGGL(gather_vsrc_all_kernel, grid(B, 1), dim3(256), 0, st, v_re, v_im, nn, B, k, diff, ctl);
    return hipGetLastError();
}
hipError_t areas_scatter_nodes(const double *src, int nn, int k0, const int32_t *mono, int nn_dst, int B, double *dst,
                               hipStream_t st) {
    if (nn - k0 <= 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_nodes_kernel, grid(B, 3 * (nn - k0)), dim3(256), 0, st, src, nn, k0, mono, nn_dst, B, dst);
    return hipGetLastError();
}
hipError_t areas_fold_results(int B, const double *loss, const double *vmin, const double *vmax, const int8_t *status,
                              int first, double *o_loss, double *o_vmin, double *o_vmax, int8_t *o_status,
                              hipStream_t st) {
    hipLaunchKernelGGL(fold_results_kernel, grid(B, 1), dim3(256), 0, st, B, loss, vmin, vmax, status, first, o_loss,
                       o_vmin, o_vmax, o_status);
    return hipGetLastError();
}
hipError_t areas_check(double *diff, int n, double tol, int single, int32_t *ctl, double *last, hipStream_t st) {
    hipLaunchKernelGGL(check_kernel, dim3(1), dim3(256), 0, st, diff, n, tol, single, ctl, last);
    return hipGetLastError();
}

}  // namespace fpf
