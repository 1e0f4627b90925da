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

// The set-up of a solve, one launch: rows y < rows gather every area's
// [field][row] lines of the feeder's batch, dst[y][s] = src[map[y]][s] (map[y] <
// 0: a separator row, 0); the rows after them are the first outer iteration's
// source powers of every non-root area: the loads of its whole subtree (rows
// sub_rows[sub_off[a] .. sub_off[a+1]) of the batch) -- short of the subtree's
// losses only, so that the first solve of the parent already sees nearly all of
// its children's demand -- and the loop's state: ctl (done, outer), the last
// move, the first iteration's inner eps, the two move slots
__global__ void setup_kernel(const double *__restrict__ src, int nl, const int32_t *__restrict__ map, int rows, int B,
                             double *__restrict__ dst, const int32_t *__restrict__ sub_off,
                             const int32_t *__restrict__ sub_rows, double *__restrict__ s_in,
                             int32_t *__restrict__ ctl, double *__restrict__ last, unsigned long long *__restrict__ move,
                             double *__restrict__ eps_dev, double eps_first) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    const int y = blockIdx.y;
    if (s == 0 && y == 0) {
        for (int i = 0; i < 4; ++i) ctl[i] = 0;
        *last = 0.0;
        move[0] = move[1] = 0ull;
        if (eps_dev) *eps_dev = eps_first;
    }
    if (s >= B) return;
    if (y < rows) {
        const int m = map[y];
        dst[(size_t)y * B + s] = m < 0 ? 0.0 : src[(size_t)m * B + s];
        return;
    }
    const int a = (y - rows) / 6, f = (y - rows) % 6;
    double x = 0.0;
    for (int i = sub_off[a]; i < sub_off[a + 1]; ++i) x += src[((size_t)f * nl + sub_rows[i]) * B + s];
    s_in[((size_t)a * 6 + f) * B + s] = x;
}

// The kernels of one outer iteration do nothing once the loop has converged
// (ctl[0] != 0: iterations enqueued before the host looked are no-ops).

// One link of the outer iteration's chain of launches (AreaLink, fpf_internal.h),
// one thread per scenario: after an area's solve, its V at every child's boundary
// bus becomes the child's source voltage and the largest move joins the
// iteration's (a wave maximum, then one atomic per wavefront: non-negative
// doubles order as their bit patterns); before the next area's solve, its child
// rows = base + the children's source powers; at the end of an iteration, the
// stop test on the move (block 0, thread 0; the other blocks may or may not see
// its flag -- the rows they write are only read by a solve that then no-ops).
__global__ void link_kernel(AreaLink L, int B, int32_t *__restrict__ ctl) {
    if (ctl[0]) return;   // (uniform)
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    double d = 0.0;
    if (s < B) {
        for (int j = 0; j < L.post.n; ++j) {
            double *const vsrc = L.post.ptr[j];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                const size_t i = ((size_t)p * L.nn + L.post.lrow[j]) * B + s;
                const double re = L.v_re[i], im = L.v_im[i];
                d = fmax(d, fmax(fabs(re - vsrc[(size_t)(2 * p) * B + s]), fabs(im - vsrc[(size_t)(2 * p + 1) * B + s])));
                vsrc[(size_t)(2 * p) * B + s] = re;
                vsrc[(size_t)(2 * p + 1) * B + s] = im;
            }
        }
        for (int j = 0; j < L.pre.n; ++j)
#pragma unroll
            for (int f = 0; f < 6; ++f) {
                const size_t i = ((size_t)f * L.nl + L.pre.lrow[j]) * B + s;
                L.work[i] = L.base[i] + L.pre.ptr[j][(size_t)f * B + s];
            }
    }
    if (L.post.n > 0) {
        for (int o = 32; o > 0; o >>= 1) d = fmax(d, __shfl_xor(d, o));
        if ((threadIdx.x & 63) == 0 && d > 0.0) atomicMax(L.move_acc, (unsigned long long)__double_as_longlong(d));
    }
    if (L.check && blockIdx.x == 0 && threadIdx.x == 0) areas_stop_test(L, ctl);
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

// whole-feeder results from the areas' (in solve order): loss summed, extremes
// folded, status = worst
__global__ void fold_results_kernel(int B, AreaFold F, double *__restrict__ o_loss, double *__restrict__ o_vmin,
                                    double *__restrict__ o_vmax, int8_t *__restrict__ o_status) {
    const int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= B) return;
    double ls = F.first ? 0.0 : o_loss[s], mn = F.first ? INFINITY : o_vmin[s], mx = F.first ? -INFINITY : o_vmax[s];
    int8_t st = F.first ? (int8_t)0 : o_status[s];
    for (int a = 0; a < F.n; ++a) {
        ls += F.loss[a][s];
        mn = fmin(mn, F.vmin[a][s]);
        mx = fmax(mx, F.vmax[a][s]);
        st = st > F.status[a][s] ? st : F.status[a][s];
    }
    o_loss[s] = ls;
    o_vmin[s] = mn;
    o_vmax[s] = mx;
    o_status[s] = st;
}

inline dim3 grid(int B, int y) { return dim3((unsigned)((B + 255) / 256), (unsigned)y); }
}  // namespace

hipError_t areas_setup(const double *src, int nl, const int32_t *map, int rows, int B, double *dst, int n_areas,
                       const int32_t *sub_off, const int32_t *sub_rows, double *s_in, int32_t *ctl, double *last,
                       unsigned long long *move, double *eps_dev, double eps_first, hipStream_t st) {
    hipLaunchKernelGGL(setup_kernel, grid(B, rows + 6 * n_areas), dim3(256), 0, st, src, nl, map, rows, B, dst, sub_off,
                       sub_rows, s_in, ctl, last, move, eps_dev, eps_first);
    return hipGetLastError();
}
hipError_t areas_link(const AreaLink &L, int B, int32_t *ctl, hipStream_t st) {
    hipLaunchKernelGGL(link_kernel, grid(B, 1), dim3(256), 0, st, L, B, ctl);
    return hipGetLastError();
}
hipError_t areas_scatter_nodes(const double *src, int nn, int k0, const int32_t *mono, int nn_dst, int B, double *dst,
                               hipStream_t st) {
    if (nn - k0 <= 0) return hipSuccess;
    hipLaunchKernelGGL(scatter_nodes_kernel, grid(B, 3 * (nn - k0)), dim3(256), 0, st, src, nn, k0, mono, nn_dst, B, dst);
    return hipGetLastError();
}
hipError_t areas_fold_results(int B, const AreaFold &F, double *o_loss, double *o_vmin, double *o_vmax,
                              int8_t *o_status, hipStream_t st) {
    hipLaunchKernelGGL(fold_results_kernel, grid(B, 1), dim3(256), 0, st, B, F, o_loss, o_vmin, o_vmax, o_status);
    return hipGetLastError();
}

}  // namespace fpf
