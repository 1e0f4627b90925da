// traffic_cal.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE against known
// byte counts for the access patterns of this repository's kernels
// (MI355X_MICROARCH.md, HBM: "other access widths are uncalibrated").
//
// Every kernel streams a 2 GiB buffer once (far beyond the 256 MiB Infinity
// Cache), grid-strided, with one access width:
//   rd8   8-byte loads per lane, 64 lanes contiguous (the generic kernel's SoA
//         slots; the wave kernel's 8-byte staging path)
//   rd16  16-byte loads per lane (the wave kernel's staging)
//   wr8   8-byte stores per lane
//   wr16  16-byte stores per lane
//   rd8s  8-byte loads, 8 scenarios (64 B) per row of a [rows][B] array, the
//         row-segment pattern of one 8-scenario workgroup tile
// Usage: traffic_cal <kernel> [reps]; prints one JSON line (bytes, ms, GB/s).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void rd8(const double *__restrict__ a, size_t n, double *__restrict__ sink) {
    double acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += a[i];
    if (acc == 1.2345) sink[0] = acc;   // keeps the loads; never true for the fill
}
__global__ __launch_bounds__(256) void rd16(const d2 *__restrict__ a, size_t n, double *__restrict__ sink) {
    double acc = 0;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const d2 v = a[i];
        acc += v.x + v.y;
    }
    if (acc == 1.2345) sink[0] = acc;
}
__global__ __launch_bounds__(256) void wr8(double *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = (double)i;
}
__global__ __launch_bounds__(256) void wr16(d2 *__restrict__ a, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) a[i] = d2{(double)i, 1.0};
}
// [rows][B] doubles; workgroup g reads the 8-scenario column block g of every row
__global__ __launch_bounds__(256) void rd8s(const double *__restrict__ a, int rows, int B, double *__restrict__ sink) {
    double acc = 0;
    for (int tile = blockIdx.x; tile < B / 8; tile += gridDim.x)
        for (int i = threadIdx.x; i < rows * 8; i += 256) acc += a[(size_t)(i / 8) * B + tile * 8 + (i % 8)];
    if (acc == 1.2345) sink[0] = acc;
}

int main(int argc, char **argv) {
    const char *k = argc > 1 ? argv[1] : "rd8";
    const int reps = argc > 2 ? atoi(argv[2]) : 5;
    const size_t bytes = (size_t)2 << 30, n8 = bytes / 8, n16 = bytes / 16;
    double *a, *sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 0, bytes));
    const int grid = 256 * 8;
    const int rows = 738, B = (int)(n8 / rows) & ~63;
    auto launch = [&]() {
        if (!strcmp(k, "rd8")) hipLaunchKernelGGL(rd8, dim3(grid), dim3(256), 0, 0, a, n8, sink);
        else if (!strcmp(k, "rd16")) hipLaunchKernelGGL(rd16, dim3(grid), dim3(256), 0, 0, (const d2 *)a, n16, sink);
        else if (!strcmp(k, "wr8")) hipLaunchKernelGGL(wr8, dim3(grid), dim3(256), 0, 0, a, n8);
        else if (!strcmp(k, "wr16")) hipLaunchKernelGGL(wr16, dim3(grid), dim3(256), 0, 0, (d2 *)a, n16);
        else if (!strcmp(k, "rd8s")) hipLaunchKernelGGL(rd8s, dim3(grid), dim3(256), 0, 0, a, rows, B, sink);
        else { fprintf(stderr, "unknown kernel %s\n", k); exit(2); }
    };
    launch();
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double per = !strcmp(k, "rd8s") ? (double)rows * B * 8 : (double)bytes;
    printf("{\"kernel\": \"%s\", \"bytes_per_launch\": %.0f, \"ms\": %.4f, \"GBps\": %.1f}\n", k, per, ms / reps,
           per / (ms / reps * 1e-3) / 1e9);
    return 0;
}
