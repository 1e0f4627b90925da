// mfma_a0.hip -- SURVEY.md 8(a) row A0 / 7.6e: is fp64 MFMA worth it on this path?
//
// Two experiments, each against its VALU counterpart, timed with HIP events:
//
//  (1) DLF form.  V = V0 - D IL(V), D = BCBV*BIBC (3Nn x 3Nb complex) -- the
//      algebraic equivalent of one backward+forward sweep of DPF_return7.cpp
//      :134-195.  Real form [Dr -Di; Di Dr] x [ILr; ILi]: an M x K times K x N
//      fp64 GEMM per sweep with M = 2*3*Nn, K = 2*3*Nb, N = scenarios.  At the
//      123-bus feeder (Nn = 123, Nb = 122) and config 2 (4096 scenarios):
//      M = 738 -> 768, K = 732 -> 736 padded.  Kernel: v_mfma_f64_16x16x4_f64,
//      64 x 64 workgroup tile, 4 waves of 32 x 32, K staged through LDS 16 at
//      a time.
//  (2) Per-branch product.  drop = Ib (1x3 complex) . TEMP (3x3 complex)
//      (DPF_return7.cpp:168,178) for 16 scenarios of one branch as an MFMA:
//      A = 16 scenarios x K (6 real Ib components padded to 8), B = K x 16
//      (the 6 real TEMP output columns padded to 16): 2 x 16x16x4 per branch
//      and tile, 28 % of the issued flops useful.  Against the VALU form the
//      wave kernel uses (36 FMAs per scenario and branch, drop_col_fma).
//      Compute-only: Ib and TEMP come from registers / LDS, the drops are
//      folded into a checksum, so neither form is bounded by memory.
//
// Prints one JSON line.  Build: make -C tools/ubench mfma_a0 (hipcc, gfx950).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- (1) GEMM
// C[M][N] = A[M][K] * B[K][N], row-major, M % 64 == N % 64 == K % 16 == 0.
constexpr int TM = 64, TN = 64, TK = 16;
__global__ __launch_bounds__(256) void dgemm_mfma(const double *__restrict__ A, const double *__restrict__ B,
                                                  double *__restrict__ Cm, int M, int N, int K) {
    __shared__ double sa[TK][TM + 1];   // A tile transposed: sa[k][m]
    __shared__ double sb[TK][TN + 1];
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
    const int wm = (w >> 1) * 32, wn = (w & 1) * 32;   // this wave's 32 x 32
    d4 acc[2][2];
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) acc[i][j] = d4{0, 0, 0, 0};
    for (int k0 = 0; k0 < K; k0 += TK) {
        // 64 x 16 of A and 16 x 64 of B: 1024 doubles each, 4 per thread
        for (int r = 0; r < 4; ++r) {
            const int i = t + 256 * r;
            const int am = i / TK, ak = i % TK;        // A row-major: consecutive threads along k
            sa[ak][am] = A[(size_t)(m0 + am) * K + k0 + ak];
            const int bk = i / TN, bn = i % TN;
            sb[bk][bn] = B[(size_t)(k0 + bk) * N + n0 + bn];
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < TK; kk += 4) {
            const int ka = kk + (lane >> 4);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const double a = sa[ka][wm + 16 * i + (lane & 15)];
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const double b = sb[ka][wn + 16 * j + (lane & 15)];
                    acc[i][j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i][j], 0, 0, 0);
                }
            }
        }
        __syncthreads();
    }
    // C/D map of the f64 form: col = lane & 15, row = (lane >> 4) + 4 * r
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j)
            for (int r = 0; r < 4; ++r)
                Cm[(size_t)(m0 + wm + 16 * i + (lane >> 4) + 4 * r) * N + n0 + wn + 16 * j + (lane & 15)] = acc[i][j][r];
}

// ---------------------------------------------------------------- (2) per-branch product
// TEMP of branch b: 3 x 3 complex, synthesised from b (values irrelevant to timing)
__device__ __forceinline__ double tval(int b, int e) { return 1e-3 * (double)((b * 7 + e * 3) % 17 + 1); }

// VALU: one lane per scenario, 36 FMAs per branch (the wave kernel's drop_col_fma)
__global__ __launch_bounds__(256) void branch_valu(int nb, double *out) {
    __shared__ double tz[64][18];   // 64 branches' TEMP blocks, reused nb/64 times
    for (int i = threadIdx.x; i < 64 * 18; i += 256) tz[i / 18][i % 18] = tval(i / 18, i % 18);
    __syncthreads();
    const int s = blockIdx.x * 256 + threadIdx.x;
    double ib[6], acc[6] = {0, 0, 0, 0, 0, 0};
    for (int e = 0; e < 6; ++e) ib[e] = 0.01 * ((s + e) % 13 + 1);
    for (int b = 0; b < nb; ++b) {
        const double *T = tz[b & 63];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            double re = acc[2 * a], im = acc[2 * a + 1];
#pragma unroll
            for (int l = 0; l < 3; ++l) {
                const double tr = T[2 * (3 * l + a)], ti = T[2 * (3 * l + a) + 1];
                re = fma(ib[2 * l], tr, re);
                re = fma(-ib[2 * l + 1], ti, re);
                im = fma(ib[2 * l], ti, im);
                im = fma(ib[2 * l + 1], tr, im);
            }
            acc[2 * a] = re;
            acc[2 * a + 1] = im;
        }
        ib[b % 6] += 1e-9;   // a new Ib per branch (keeps the loop honest)
    }
    double x = 0;
    for (int e = 0; e < 6; ++e) x += acc[e];
    out[s] = x;
}

// MFMA: a wave = 4 tiles of 16 scenarios; per branch and tile 2 MFMAs (K = 8)
// A[s][k] = Ib component k of scenario s (k < 6), B[k][j] = real TEMP (j < 6)
__global__ __launch_bounds__(256) void branch_mfma(int nb, double *out) {
    __shared__ double tb[64][8][16];   // per branch: real 8 x 16 B operand (padded)
    for (int i = threadIdx.x; i < 64 * 8 * 16; i += 256) {
        const int b = i / 128, k = (i / 16) % 8, j = i % 16;
        double v = 0.0;
        if (k < 6 && j < 6) {
            // [re, im] of Ib_l times TEMP(l, a): out_re(a) += re*Tr - im*Ti, out_im(a) += re*Ti + im*Tr
            const int l = k / 2, a = j / 2;
            const double tr = tval(b, 2 * (3 * l + a)), ti = tval(b, 2 * (3 * l + a) + 1);
            v = (k & 1) == 0 ? ((j & 1) == 0 ? tr : ti) : ((j & 1) == 0 ? -ti : tr);
        }
        tb[b][k][j] = v;
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int s = blockIdx.x * 256 + threadIdx.x;   // 4 tiles x 16 scenarios per wave, 4 waves
    d4 acc[4];
    for (int q = 0; q < 4; ++q) acc[q] = d4{0, 0, 0, 0};
    // A fragment: lane holds A[row = lane & 15][k = lane >> 4] (+4 for the 2nd MFMA)
    double a0[4], a1[4];
    for (int q = 0; q < 4; ++q) {
        const int k0 = lane >> 4, k1 = 4 + (lane >> 4);
        a0[q] = 0.01 * ((s + q + k0) % 13 + 1);
        a1[q] = k1 < 6 ? 0.01 * ((s + q + k1) % 13 + 1) : 0.0;
    }
    for (int b = 0; b < nb; ++b) {
        const double b0 = tb[b & 63][lane >> 4][lane & 15], b1 = tb[b & 63][4 + (lane >> 4)][lane & 15];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0[q], b0, acc[q], 0, 0, 0);
            acc[q] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1[q], b1, acc[q], 0, 0, 0);
        }
        a0[b & 3] += 1e-9;
    }
    double x = 0;
    for (int q = 0; q < 4; ++q) x += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
    out[s] = x;
}

template <typename F>
static double time_ms(F launch, int reps) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
}

int main(int argc, char **argv) {
    const int which = argc > 1 ? atoi(argv[1]) : 0;   // 0 all, 1 GEMM, 2 branch products (profiling)
    // ---- (1) DLF GEMM at the 123-bus feeder, config 2 batch
    const int M = 768, K = 736, N = 4096;
    std::vector<double> hA((size_t)M * K), hB((size_t)K * N);
    for (size_t i = 0; i < hA.size(); ++i) hA[i] = 1e-3 * (double)((i * 2654435761u) % 1000) - 0.5e-3 * 999;
    for (size_t i = 0; i < hB.size(); ++i) hB[i] = 1e-3 * (double)((i * 40503u) % 997);
    double *A, *B, *Cm;
    CK(hipMalloc(&A, hA.size() * 8));
    CK(hipMalloc(&B, hB.size() * 8));
    CK(hipMalloc(&Cm, (size_t)M * N * 8));
    CK(hipMemcpy(A, hA.data(), hA.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(B, hB.data(), hB.size() * 8, hipMemcpyHostToDevice));
    double gemm_ms = 0, gemm_err = 0;
    if (which == 0 || which == 1) {
        gemm_ms = time_ms([&] { hipLaunchKernelGGL(dgemm_mfma, dim3(N / TN, M / TM), dim3(256), 0, 0, A, B, Cm, M, N, K); },
                          which ? 200 : 20);
        // spot check 64 entries against a host dot product
        std::vector<double> hC((size_t)M * N);
        CK(hipMemcpy(hC.data(), Cm, hC.size() * 8, hipMemcpyDeviceToHost));
        for (int t = 0; t < 64; ++t) {
            const int i = (t * 37) % M, j = (t * 1013) % N;
            double ref = 0;
            for (int k = 0; k < K; ++k) ref = fma(hA[(size_t)i * K + k], hB[(size_t)k * N + j], ref);
            gemm_err = std::max(gemm_err, std::fabs(hC[(size_t)i * N + j] - ref) / std::max(std::fabs(ref), 1e-300));
        }
    }
    const double gemm_flop = 2.0 * M * N * K;
    // ---- (2) per-branch products, compute-only
    const int nb = 2047, S = 65536;
    double *o;
    CK(hipMalloc(&o, (size_t)S * 8));
    double valu_ms = 0, mfma_ms = 0;
    if (which == 0 || which == 2) {
        valu_ms = time_ms([&] { hipLaunchKernelGGL(branch_valu, dim3(S / 256), dim3(256), 0, 0, nb, o); }, which ? 20 : 5);
        // MFMA kernel: 64 scenarios per wave (4 tiles of 16), 256 per workgroup
        mfma_ms = time_ms([&] { hipLaunchKernelGGL(branch_mfma, dim3(S / 256), dim3(256), 0, 0, nb, o); }, which ? 20 : 5);
    }
    const double useful = 2.0 * 36.0 * (double)nb * S;   // 36 real MACs per scenario and branch
    printf("{\"dlf_gemm\": {\"M\": %d, \"K\": %d, \"N\": %d, \"ms\": %.5f, \"tflops\": %.3f, \"peak_tflops\": 78.6, "
           "\"max_rel_err\": %.3e, \"note\": \"one sweep of the DLF form at the 123-bus feeder, 4096 scenarios\"}, "
           "\"branch_product\": {\"branches\": %d, \"scenarios\": %d, \"valu_ms\": %.4f, \"mfma_ms\": %.4f, "
           "\"valu_useful_tflops\": %.3f, \"mfma_useful_tflops\": %.3f, \"mfma_issued_tflops\": %.3f}}\n",
           M, K, N, gemm_ms, gemm_ms > 0 ? gemm_flop / (gemm_ms * 1e-3) / 1e12 : 0.0, gemm_err, nb, S, valu_ms, mfma_ms,
           valu_ms > 0 ? useful / (valu_ms * 1e-3) / 1e12 : 0.0, mfma_ms > 0 ? useful / (mfma_ms * 1e-3) / 1e12 : 0.0,
           mfma_ms > 0 ? (2.0 * 2048.0 * nb * (S / 16)) / (mfma_ms * 1e-3) / 1e12 : 0.0);
    return 0;
}
