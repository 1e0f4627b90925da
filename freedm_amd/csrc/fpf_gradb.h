// fpf_gradb.h -- the batched VVC gradient's host/device interface
// (fpf_vvc_grad.cpp builds the plan, fpf_vvc_gradb.hip runs it).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fpf {

// per-scenario gradient status (fpf_vvc_gradient_batch's gstatus)
constexpr int8_t FPF_GRAD_OK = 0;
constexpr int8_t FPF_GRAD_NONCONV = 1;    // the base solve did not converge (the reference throws)
constexpr int8_t FPF_GRAD_SINGULAR = 2;   // J singular (LU pivot 0)
constexpr int8_t FPF_GRAD_PATTERN = 3;    // V_abc_list rows differ from the plan's

// One phase's plan on the device (every pointer device memory)
struct GradPhaseDev {
    int x, L, n, nn, scan_end, n_loads;
    const int32_t *vrow;      // [n] Vpolar row of V-list entry j (-1: V = 0)
    const int8_t *vmask;      // [scan_end] 1 where a row is in the V list
    const int32_t *bs, *br;   // [L] renamed branch ends (rename_brn.cpp)
    const double *yre_sr;     // [L] Y(s_j, r_j).real()
    const int32_t *inc_ptr;   // [n] Fx: bus i + 1's branches (CSR over i < n - 1)
    const int32_t *inc_br;
    const int8_t *inc_role;   // 0: the branch starts at the bus, 1: ends there
    const int32_t *y_ptr;     // [n + 1] Y's nonzero off-diagonal entries of row a, by column
    const int32_t *y_col;
    const double *y_re, *y_im;
    const double *ydiag_re, *ydiag_im;   // [n]
    const int32_t *ld_ptr;    // [n_loads + 1] g: the V-list buses ia + 1 of load j
    const int32_t *ld_ia;
};

// scenarios c0 .. c0 + nb of a batch of B: vpolar [6][nn][B] and gstat [B] are the
// batch's, A [nb][nf][nf] (J^T, column-major) and rhs [nb][nf] the chunk's; g [B][3][ld]
hipError_t launch_gradb_setup(const GradPhaseDev &P, int B, int c0, int nb, const double *vpolar, double *A,
                              double *rhs, int8_t *gstat, hipStream_t st);
// lambda' = inv(J^T) Fx: LU with partial pivoting + solve per matrix (rhs overwritten)
// whether the LU of an nf x nf system fits the kernel's LDS (nf <= 6400)
bool gradb_lu_fits(int nf);
hipError_t launch_gradb_lu(int nf, int nb, double *A, double *rhs, int8_t *sing, hipStream_t st);
hipError_t launch_gradb_g(const GradPhaseDev &P, int c0, int nb, const double *sol, int ld, double *g, hipStream_t st);

// The step-size search's candidate batch of fpf_vvc_round_batch on the device:
// candidate column k M + m of cand [6 nl][K M] is scenario todo[k]'s loads of pq
// [6 nl][B] with, at every (phase x, load i, row r) of the triples [T][3], the Q
// set-point moved: pq - g[(s 3 + x) ld + i] * scale * c_m, c_0 = cstart[k],
// c_{m+1} = alpha c_m (VoltVarCtrl.cpp:1323, 1420-1422, 1546) -- the host loop's
// operations in its order, so the candidates are bit-identical to it
hipError_t launch_vvc_candidates(const double *pq, int nl, int B, const int32_t *todo, int K, int M,
                                 const int32_t *triples, int T, const double *g, int ld, double scale, double alpha,
                                 const double *cstart, double *cand, hipStream_t st);

}  // namespace fpf
