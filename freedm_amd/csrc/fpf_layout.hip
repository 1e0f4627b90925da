// fpf_layout.hip -- the batch-layout transpose (fpf_opts.layout): out[c][r] =
// in[r][c] for a row-major [rows][cols] matrix of doubles.  The wave kernels
// read and write the scenario-major layout natively; the host wraps the generic
// and tiled kernels (exact mode) in these transposes instead.
#include "fpf_internal.h"

namespace fpf {

namespace {
constexpr int TT = 32;   // tile edge; 32 x 8 threads, 4 rows each

__global__ __launch_bounds__(256) void transpose_kernel(const double *__restrict__ in, double *__restrict__ out,
                                                        size_t rows, size_t cols) {
    __shared__ double tile[TT][TT + 1];
    const size_t c0 = (size_t)blockIdx.x * TT, r0 = (size_t)blockIdx.y * TT;
    const int tx = threadIdx.x & (TT - 1), ty = threadIdx.x / TT;
#pragma unroll
    for (int j = ty; j < TT; j += 8) {
        const size_t r = r0 + j, c = c0 + tx;
        if (r < rows && c < cols) tile[j][tx] = in[r * cols + c];
    }
    __syncthreads();
#pragma unroll
    for (int j = ty; j < TT; j += 8) {
        const size_t c = c0 + j, r = r0 + tx;
        if (r < rows && c < cols) out[c * rows + r] = tile[tx][j];
    }
}
}  // namespace

hipError_t launch_transpose(const double *in, double *out, size_t rows, size_t cols, hipStream_t st) {
    if (rows == 0 || cols == 0) return hipSuccess;
    const size_t gx = (cols + TT - 1) / TT, gy = (rows + TT - 1) / TT;
    if (gy > 65535 || gx > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)gx, (unsigned)gy), dim3(256), 0, st, in, out, rows, cols);
    return hipGetLastError();
}

}  // namespace fpf
