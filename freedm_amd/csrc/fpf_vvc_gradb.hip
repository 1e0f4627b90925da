// fpf_vvc_gradb.hip -- the batched VVC gradient's device half
// (fpf_vvc_grad.cpp: fpf_vvc_gradient_batch): per scenario and phase the
// V_abc_list values, Fx = [dF/dtheta; dF/dV] and J^T = [H N; K L]^T
// (Broker/src/vvc/form_Ftheta.cpp, form_Fv.cpp, form_J.cpp, V_abc_list.cpp;
// VoltVarCtrl.cpp:1222-1325), then g = -gu^T lambda from the LU solution.
// The structure (the branch lists, Y, the V_abc_list rows, the renamed branch
// ends, the load map) is the host plan's, shared by every scenario of the batch.
//
// The reference's F and J sums run in x87 long double; here every such sum is
// a double-double (TwoSum) accumulation of the same double terms in the same
// order, rounded once -- at least the long double's precision.  The terms are
// the reference's double expressions, left to right, no FMA contraction
// (-ffp-contract=off).  Terms of a zero admittance (the reference sums them:
// +-0) are skipped: adding a signed zero leaves a nonzero sum unchanged.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <mutex>
#include <set>

#include "fpf_gradb.h"

namespace fpf {
namespace {

constexpr double kPi = 3.14159265358979323846;   // form_Ftheta.cpp:11

struct DD {
    double hi = 0.0, lo = 0.0;
    __device__ void add(double x) {   // TwoSum
        const double s = hi + x, bb = s - hi;
        lo += (hi - (s - bb)) + (x - bb);
        hi = s;
    }
    __device__ double value() const { return hi + lo; }
};
// v * (hi + lo), rounded once (the long double product of the reference)
__device__ double dd_mul(double v, const DD &d) {
    const double p = v * d.hi;
    const double e = fma(v, d.hi, -p) + v * d.lo;
    return p + e;
}

// One workgroup per scenario s of this phase: the V list, Fx into rhs[s], J^T
// into A[s] (column-major, lda = nf; every entry written: zeros first).
// (a launch covers scenarios c0 .. c0 + gridDim.x of the batch: vpolar and gstat
// are the batch's arrays, A and rhs the chunk's)
__global__ __launch_bounds__(256) void gradb_setup_kernel(GradPhaseDev P, int B, int c0,
                                                          const double *__restrict__ vpolar, double *__restrict__ A,
                                                          double *__restrict__ rhs, int8_t *__restrict__ gstat) {
    extern __shared__ double sh[];
    const int k = blockIdx.x, s = c0 + k, t = threadIdx.x, NT = blockDim.x;
    const int n = P.n, m1 = n - 1, nf = 2 * m1, nn = P.nn;
    double *const V = sh, *const TH = sh + n;
    // V_abc_list (V_abc_list.cpp): the first n rows with a nonzero |V|; the rows
    // are the plan's -- a scenario whose nonzero pattern differs is flagged
    for (int j = t; j < n; j += NT) {
        const int i = P.vrow[j];
        V[j] = i < 0 ? 0.0 : vpolar[((size_t)(2 * P.x) * nn + i) * B + s];
        TH[j] = i < 0 ? 0.0 : vpolar[((size_t)(2 * P.x + 1) * nn + i) * B + s];
    }
    for (int i = t; i < P.scan_end; i += NT) {
        const bool nz = vpolar[((size_t)(2 * P.x) * nn + i) * B + s] != 0;
        if (nz != (P.vmask[i] != 0) && gstat[s] == FPF_GRAD_OK) gstat[s] = FPF_GRAD_PATTERN;
    }
    double *const As = A + (size_t)k * nf * nf;
    for (size_t q = t; q < (size_t)nf * nf; q += NT) As[q] = 0.0;
    __syncthreads();
    // Fx (form_Ftheta.cpp, form_Fv.cpp): bus i + 1's terms in branch order
    double *const Fx = rhs + (size_t)k * nf;
    for (int i = t; i < m1; i += NT) {
        DD rt, rv;
        for (int q = P.inc_ptr[i]; q < P.inc_ptr[i + 1]; ++q) {
            const int j = P.inc_br[q];
            const int sb = P.bs[j], rb = P.br[j];
            const double d = (TH[sb] - TH[rb]) * kPi / 180;
            const double gsr = -P.yre_sr[j];   // -Y(s, r).real()
            if (P.inc_role[q] == 0) {          // s == i + 1
                rt.add(-(2 * gsr * V[sb] * V[rb] * (-sin(d))));
                rv.add(2 * gsr * (V[sb] - V[rb] * cos(d)));
            } else {                           // r == i + 1
                rt.add(-(2 * gsr * V[sb] * V[rb] * sin(d)));
                rv.add(2 * gsr * (V[rb] - V[sb] * cos(d)));
            }
        }
        Fx[i] = rt.value();
        Fx[m1 + i] = rv.value();
    }
    // J^T (form_J.cpp), as the host stores it: put(row, col, v) -> As[col + row nf]
    auto put = [&](int row, int col, double v) { As[(size_t)col + (size_t)row * nf] = v; };
    for (int a = 1 + t; a < n; a += NT) {
        DD rs, rc;   // over m != a, in m order: V_m (G sin - B cos), V_m (G cos + B sin)
        for (int q = P.y_ptr[a]; q < P.y_ptr[a + 1]; ++q) {
            const int m = P.y_col[q];
            const double d = (TH[a] - TH[m]) * kPi / 180;
            const double yr = P.y_re[q], yi = P.y_im[q];
            rs.add(V[m] * (yr * sin(d) - yi * cos(d)));
            rc.add(V[m] * (yr * cos(d) + yi * sin(d)));
        }
        for (int q = P.y_ptr[a]; q < P.y_ptr[a + 1]; ++q) {
            const int b = P.y_col[q];
            if (b < 1) continue;
            const double d = (TH[a] - TH[b]) * kPi / 180;
            const double yr = P.y_re[q], yi = P.y_im[q];
            const double sn = yr * sin(d) - yi * cos(d);
            const double cs = yr * cos(d) + yi * sin(d);
            put(a - 1, b - 1, V[a] * V[b] * sn);
            put(a - 1, m1 + b - 1, V[a] * cs);
            put(m1 + a - 1, b - 1, -V[a] * V[b] * cs);
            put(m1 + a - 1, m1 + b - 1, V[a] * sn);
        }
        const double dr = P.ydiag_re[a], di = P.ydiag_im[a];
        put(a - 1, a - 1, -dd_mul(V[a], rs));
        {
            DD x = rc;
            x.add(2 * V[a] * dr);
            put(a - 1, m1 + a - 1, x.value());
        }
        put(m1 + a - 1, a - 1, dd_mul(V[a], rc));
        {
            DD x = rs;
            x.add(-2 * V[a] * di);
            put(m1 + a - 1, m1 + a - 1, x.value());
        }
    }
}

// g = -gu^T lambda (VoltVarCtrl.cpp:1300-1317): load j of the phase sums the
// negated solution at L + ia over the V-list buses ia + 1 it sits at, in order
__global__ void gradb_g_kernel(GradPhaseDev P, int c0, const double *__restrict__ sol, int ld, double *__restrict__ g) {
    const int k = blockIdx.x, s = c0 + k;
    const int nf = 2 * (P.n - 1);
    for (int j = threadIdx.x; j < P.n_loads; j += blockDim.x) {
        double acc = 0;
        for (int q = P.ld_ptr[j]; q < P.ld_ptr[j + 1]; ++q) acc += -sol[(size_t)k * nf + P.L + P.ld_ia[q]];
        g[((size_t)s * 3 + P.x) * ld + j] = acc;
    }
}
// lambda' = inv(J^T) Fx for each matrix of the chunk: LU with partial pivoting on
// A (column-major, lda = nf) with the right-hand side eliminated along, then back
// substitution -- the host's lu_solve (fpf_vvc_grad.cpp) step for step: the first
// largest |A(i, k)| pivots, whole rows swap, the multipliers A(i, k) / A(k, k),
// A(i, j) -= l_i A(k, j) (multiply, then subtract), zero pivot-row entries and zero
// multipliers skipped.  One workgroup per matrix; the pivot row and the multiplier
// column of each step go through LDS, the update runs over their nonzeros only
// (J of a radial feeder is tree-sparse).  Back substitution by columns.
// sing[k] = 1: a zero pivot (the matrix is singular; x is not written).
constexpr int LU_NT = 256;
__global__ __launch_bounds__(LU_NT) void gradb_lu_kernel(int nf, double *__restrict__ Aall, double *__restrict__ rall,
                                                         int8_t *__restrict__ sing) {
    extern __shared__ double lsh[];
    double *const urow = lsh;                  // [nf] pivot row values (columns > k)
    double *const lcol = lsh + nf;             // [nf] multipliers (rows > k)
    int *const cidx = (int *)(lsh + 2 * nf);   // [nf] nonzero columns of the pivot row
    int *const ridx = cidx + nf;               // [nf] nonzero multipliers' rows
    __shared__ double red_v[LU_NT / 64];
    __shared__ int red_i[LU_NT / 64], cnt[2], piv_row, bad;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    double *const A = Aall + (size_t)blockIdx.x * nf * nf;
    double *const x = rall + (size_t)blockIdx.x * nf;
    auto at = [&](int i, int j) -> double & { return A[(size_t)i + (size_t)j * nf]; };
    if (t == 0) bad = 0;
    for (int k = 0; k < nf; ++k) {
        // ---- pivot: the first largest |A(i, k)|, i >= k
        double bv = -1.0;
        int bi = nf;
        for (int i = k + t; i < nf; i += LU_NT) {
            const double v = fabs(at(i, k));
            if (v > bv) { bv = v; bi = i; }
        }
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            const double ov = __shfl_xor(bv, m, 64);
            const int oi = __shfl_xor(bi, m, 64);
            if (ov > bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
        }
        if (lane == 0) { red_v[w] = bv; red_i[w] = bi; }
        __syncthreads();
        if (t == 0) {
            double v = red_v[0];
            int i = red_i[0];
            for (int q = 1; q < LU_NT / 64; ++q)
                if (red_v[q] > v || (red_v[q] == v && red_i[q] < i)) { v = red_v[q]; i = red_i[q]; }
            piv_row = i;
            if (!(v > 0.0)) bad = 1;   // (also NaN)
            cnt[0] = cnt[1] = 0;
        }
        __syncthreads();
        if (bad) break;   // (uniform)
        const int p = piv_row;
        // ---- swap rows k and p (every column, and the right-hand side)
        if (p != k) {
            for (int j = t; j < nf; j += LU_NT) {
                const double a = at(k, j);
                at(k, j) = at(p, j);
                at(p, j) = a;
            }
            if (t == 0) {
                const double a = x[k];
                x[k] = x[p];
                x[p] = a;
            }
        }
        __syncthreads();
        // ---- multipliers and the right-hand side; the pivot row's nonzeros
        const double pv = at(k, k), xk = x[k];
        for (int i = k + 1 + t; i < nf; i += LU_NT) {
            const double l = at(i, k) / pv;
            at(i, k) = l;
            if (xk != 0) x[i] -= l * xk;
            if (l != 0) {
                const int q = atomicAdd(&cnt[1], 1);
                ridx[q] = i;
                lcol[q] = l;
            }
        }
        for (int j = k + 1 + t; j < nf; j += LU_NT) {
            const double u = at(k, j);
            if (u != 0) {
                const int q = atomicAdd(&cnt[0], 1);
                cidx[q] = j;
                urow[q] = u;
            }
        }
        __syncthreads();
        // ---- the trailing update over the nonzero pairs (each element once per step)
        const int nc = cnt[0], nr = cnt[1];
        for (int e = t; e < nc * nr; e += LU_NT) {
            const int c = e / nr, r = e - c * nr;
            double &a = at(ridx[r], cidx[c]);
            a -= lcol[r] * urow[c];
        }
        __syncthreads();
    }
    if (bad) {
        if (t == 0) sing[blockIdx.x] = 1;
        return;
    }
    // ---- back substitution, column by column: x_j = x_j / U(j, j); x_i -= U(i, j) x_j, i < j
    for (int j = nf - 1; j >= 0; --j) {
        if (t == 0) x[j] = x[j] / at(j, j);
        __syncthreads();
        const double xj = x[j];
        for (int i = t; i < j; i += LU_NT) x[i] -= at(i, j) * xj;
        __syncthreads();
    }
    if (t == 0) sing[blockIdx.x] = 0;
}
}  // namespace

bool gradb_lu_fits(int nf) { return (2 * sizeof(double) + 2 * sizeof(int)) * (size_t)nf <= 150 * 1024; }

hipError_t launch_gradb_lu(int nf, int nb, double *A, double *rhs, int8_t *sing, hipStream_t st) {
    const size_t lds = (2 * sizeof(double) + 2 * sizeof(int)) * (size_t)nf;
    if (!gradb_lu_fits(nf)) return hipErrorInvalidValue;   // nf <= 6400 (feeders of ~3200 buses)
    if (lds > 64 * 1024) {
        // dynamic LDS above the default 64 KiB: a per-device setting
        static std::mutex mu;
        static std::set<int> done;
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
        std::lock_guard<std::mutex> lk(mu);
        if (!done.count(dev)) {
            const hipError_t e = hipFuncSetAttribute((const void *)gradb_lu_kernel,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
            if (e != hipSuccess) return e;
            done.insert(dev);
        }
    }
    hipLaunchKernelGGL(gradb_lu_kernel, dim3((unsigned)nb), dim3(LU_NT), lds, st, nf, A, rhs, sing);
    return hipGetLastError();
}

hipError_t launch_gradb_setup(const GradPhaseDev &P, int B, int c0, int nb, const double *vpolar, double *A,
                              double *rhs, int8_t *gstat, hipStream_t st) {
    const size_t lds = sizeof(double) * 2 * (size_t)P.n;
    if (lds > 64 * 1024) return hipErrorInvalidValue;   // (V and theta of up to 4096 buses)
    hipLaunchKernelGGL(gradb_setup_kernel, dim3((unsigned)nb), dim3(256), lds, st, P, B, c0, vpolar, A, rhs, gstat);
    return hipGetLastError();
}

hipError_t launch_gradb_g(const GradPhaseDev &P, int c0, int nb, const double *sol, int ld, double *g, hipStream_t st) {
    hipLaunchKernelGGL(gradb_g_kernel, dim3((unsigned)nb), dim3(64), 0, st, P, c0, sol, ld, g);
    return hipGetLastError();
}

namespace {
// the broadcast: cand[fr][k M + m] = pq[fr][todo[k]]
__global__ void vvc_cand_bcast_kernel(const double *__restrict__ pq, int B, const int32_t *__restrict__ todo, int K,
                                      int M, double *__restrict__ cand) {
    const size_t Bc = (size_t)K * M;
    const size_t col = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int fr = blockIdx.y;
    if (col >= Bc) return;
    cand[fr * Bc + col] = pq[(size_t)fr * B + todo[col / M]];
}
// the Q set-points: one thread per (candidate, triple)
__global__ void vvc_cand_q_kernel(const double *__restrict__ pq, int nl, int B, const int32_t *__restrict__ todo, int K,
                                  int M, const int32_t *__restrict__ triples, int T, const double *__restrict__ g,
                                  int ld, double scale, double alpha, const double *__restrict__ cstart,
                                  double *__restrict__ cand) {
    const size_t Bc = (size_t)K * M;
    const size_t col = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int t = blockIdx.y;
    if (col >= Bc) return;
    const int k = (int)(col / M), m = (int)(col % M), s = todo[k];
    const int x = triples[3 * t], i = triples[3 * t + 1], r = triples[3 * t + 2];
    double cvq = cstart[k];
    for (int j = 0; j < m; ++j) cvq = alpha * cvq;
    const double gupdate = g[((size_t)s * 3 + x) * ld + i] * scale * cvq;
    const size_t row = (size_t)(1 + 2 * x) * nl + r;   // Q of phase x = Dl column 7 + 2x
    cand[row * Bc + col] = pq[row * B + s] - gupdate;
}
}  // namespace

hipError_t launch_vvc_candidates(const double *pq, int nl, int B, const int32_t *todo, int K, int M,
                                 const int32_t *triples, int T, const double *g, int ld, double scale, double alpha,
                                 const double *cstart, double *cand, hipStream_t st) {
    const size_t Bc = (size_t)K * M;
    if (Bc == 0) return hipSuccess;
    const unsigned gx = (unsigned)((Bc + 255) / 256);
    hipLaunchKernelGGL(vvc_cand_bcast_kernel, dim3(gx, 6 * nl), dim3(256), 0, st, pq, B, todo, K, M, cand);
    if (T > 0)
        hipLaunchKernelGGL(vvc_cand_q_kernel, dim3(gx, T), dim3(256), 0, st, pq, nl, B, todo, K, M, triples, T, g, ld,
                           scale, alpha, cstart, cand);
    return hipGetLastError();
}

}  // namespace fpf
