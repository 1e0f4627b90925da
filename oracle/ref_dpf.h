/*
 * ref_dpf.h -- TEST INFRASTRUCTURE ONLY (the parity oracle).
 *
 * A scalar C restatement of the reference's distribution power-flow path:
 *   VPQ DPF_return7(arma::mat Dl, arma::cx_mat Z)   Broker/src/vvc/DPF_return7.cpp:8-263
 * plus the VVC reductions computed on its result:
 *   loss                Broker/src/vvc/VoltVarCtrl.cpp:1152-1161
 *   Lnum_a/b/c          Broker/src/vvc/form_Yabc.cpp:8-58
 *   V_abc_list          Broker/src/vvc/V_abc_list.cpp:7-81
 *   Vmin / Vmax         Broker/src/vvc/VoltVarCtrl.cpp:1201-1207
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load
 * this code, and only as the checker / CPU baseline -- never as the product path.
 *
 * PARITY STATUS: "parity unpinned" against the reference binary.  The reference
 * needs Armadillo (absent from this image, so it cannot be compiled here) and its
 * own repository holds no golden vectors for this path (SURVEY.md section 4,
 * section 8(c)).  The restatement is cross-checked against an independent NumPy
 * restatement (oracle/np_dpf.py) and against the qualitative trace in
 * Broker/output.txt; see DESIGN.md "Oracle".
 *
 * Layouts follow Armadillo (column-major).  Complex matrices are interleaved
 * (re, im) pairs, i.e. reinterpret_cast<const double*>(arma::cx_mat::memptr()).
 */
#ifndef FREEDM_REF_DPF_H
#define FREEDM_REF_DPF_H

#ifdef __cplusplus
extern "C" {
#endif

/* status codes (mirrors include/freedm_pf.h) */
#define REF_CONVERGED      0
#define REF_NONCONVERGED   1   /* reference: Armadillo size-mismatch logic_error (DPF_return7.cpp:100-101,242) */
#define REF_BAD_INPUT     -2   /* reference: Armadillo bounds-check exception */

typedef struct ref_opts {
    double bkva;    /* 1000          DPF_return7.cpp:11 */
    double bkv;     /* 12.47         :12 */
    double vo_kv;   /* 12.47*1.015   :13 */
    double eps;     /* 0.0001        :14 */
    int    mxitr;   /* 20            :15 */
} ref_opts;

typedef struct ref_out {
    /* every pointer may be NULL; matrices are column-major like Armadillo */
    double *vpolar;  /* nn x 6 : [|Va| angA |Vb| angB |Vc| angC], substation first   */
    double *pqb;     /* nn x 6 : [Pa Qa Pb Qb Pc Qc] branch powers (kW / kVAr)         */
    double *pql;     /* nn x 6 : load powers                                           */
    double *v;       /* nn x 3 complex (interleaved) node voltages in Vpolar row order */
    double *ib;      /* (nn-1) x 3 complex : Iinj                                      */
    double *il;      /* nn x 3 complex     : Ild                                       */
    int     iters;   /* sweeps executed (i+1 at the converging sweep, mxitr otherwise) */
    int     status;  /* REF_* */
    double  errmx;   /* errmx of the last sweep                                        */
    double *errmx_trace;  /* [mxitr] errmx of every sweep executed (may be NULL)        */
} ref_out;

void ref_opts_default(ref_opts *o);

/* cnt_nodes of DPF_return7.cpp:21-37, or <0 on malformed arguments */
int ref_count_nodes(const double *dl, int nl, int ncols);

/* Static index checks equivalent to the Armadillo bounds checks that the
 * reference would trip (returns 0 or REF_BAD_INPUT). */
int ref_check(const double *dl, int nl, int ncols, int z_rows, int z_cols);

/* One DPF_return7 call.  Returns out->status. */
int ref_dpf_solve(const double *dl, int nl, int ncols,
                  const double *z, int z_rows, int z_cols,
                  const ref_opts *o, ref_out *out);

/* Lnum_a/b/c of form_Y_abc (form_Yabc.cpp:11-58). Returns 0 or REF_BAD_INPUT. */
int ref_lnum(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
             double bkva, double bkv, int lnum[3]);

/* loss (VoltVarCtrl.cpp:1152-1161) and Vmin/Vmax (V_abc_list.cpp + :1201-1207) */
void ref_vvc_reduce(const double *vpolar, const double *pqb, const double *pql, int nn,
                    const int lnum[3], double *loss, double *vmin, double *vmax);

/* Batched driver (CPU baseline and fixture generation).
 *   dl      : topology Dl (nl x ncols, column-major); its columns 6..11 are ignored
 *   pq      : per-scenario loads [6][nl][n_scen] (P1 Q1 P2 Q2 P3 Q3, scenario fastest)
 *   outputs : [col][row][n_scen] (scenario fastest), each may be NULL
 * Scenarios are statically partitioned over nthreads pthreads.
 * Returns the number of non-converged scenarios, or REF_BAD_INPUT. */
int ref_dpf_batch(const double *dl, int nl, int ncols,
                  const double *z, int z_rows, int z_cols,
                  const ref_opts *o, int n_scen, const double *pq,
                  double *vpolar, double *pqb, double *pql,
                  double *v_re, double *v_im,
                  int *iters, signed char *status,
                  double *loss, double *vmin, double *vmax,
                  int nthreads);

/* ---- the VVC round (ref_vvc.c) ----
 * Gradient of the loss w.r.t. the SST Q injections (VoltVarCtrl.cpp:1141-1325)
 * at the DPF result vpolar (nn x 6) of dl.  g, load_nodes: [3][ld];
 * n_loads[3]; stats[4] = gmin, gmax, gabs_min, cvq (the first step size).
 * Returns 0 or REF_BAD_INPUT. */
int ref_vvc_gradient(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
                     const double *vpolar, int nn, double bkva, double bkv, double beta0, int ld,
                     double *g, double *load_nodes, int *n_loads, double *stats);

/* vvc_main's numerics, sequential as the reference (VoltVarCtrl.cpp:1141-1762):
 * res[13] = ploss_orig, vmin_orig, vmax_orig, c0, stop_fwd, stop_rev, reversed,
 * sent, ploss_after, gmin, gmax, gabs_min, DPF calls. */
int ref_vvc_main(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols, const ref_opts *o,
                 double beta0, double alpha, int m_max, int ld, double *g, double *load_nodes, int *n_loads,
                 double *loss_fwd, double *loss_rev, double *dl_out, double *res);

/* ref_dpf_batch with the per-scenario errmx of the last sweep (errmx may be NULL) */
int ref_dpf_batch_ex(const double *dl, int nl, int ncols,
                     const double *z, int z_rows, int z_cols,
                     const ref_opts *o, int n_scen, const double *pq,
                     double *vpolar, double *pqb, double *pql,
                     double *v_re, double *v_im,
                     int *iters, signed char *status,
                     double *loss, double *vmin, double *vmax, double *errmx,
                     int nthreads);

#ifdef __cplusplus
}
#endif
#endif
