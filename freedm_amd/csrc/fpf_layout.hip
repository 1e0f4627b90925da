// fpf_layout.hip -- the batch-layout transpose (fpf_opts.layout): out[c][r] =
// in[r][c] for a row-major [rows][cols] matrix of doubles.  The wave kernels
// read and write the scenario-major layout natively; the host wraps the generic
// and tiled kernels (exact mode) in these transposes instead.
#include "fpf_internal.h"

namespace fpf {

namespace {
constexpr int TT = 32;   // tile edge; 32 x 8 threads, 4 rows each

__global__ __launch_bounds__(256) void transpose_kernel(const double *__restrict__ in, double *__restrict__ out,
                                                        size_t rows, size_t cols, size_t row_base) {
    __shared__ double tile[TT][TT + 1];
    const size_t c0 = (size_t)blockIdx.x * TT, r0 = row_base + (size_t)blockIdx.y * TT;
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
    if (gx > 0x7fffffff) return hipErrorInvalidValue;
    // grid y is at most 65535 tiles: a long row dimension (a scenario-major batch
    // of more than ~2.1 M scenarios) goes in launches of that many row tiles
    constexpr size_t GY = 65535;
    for (size_t y0 = 0; y0 < gy; y0 += GY) {
        const size_t n = gy - y0 < GY ? gy - y0 : GY;
        hipLaunchKernelGGL(transpose_kernel, dim3((unsigned)gx, (unsigned)n), dim3(256), 0, st, in, out, rows, cols,
                           y0 * TT);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace fpf
