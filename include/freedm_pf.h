/*
 * freedm_pf.h -- C ABI of libfreedm_pf, the MI355X (gfx950) batched distribution
 * power-flow engine that replaces the FREEDM DGI Broker's VVC power-flow call.
 *
 * Reference interface replaced (vmuthuk2/FREEDM, paths relative to the repo):
 *   VPQ DPF_return7(arma::mat Dl, arma::cx_mat Z)
 *       declared Broker/src/vvc/fun_return.h:53, defined DPF_return7.cpp:8-263
 *       called   Broker/src/vvc/VoltVarCtrl.cpp:1141, 1379, 1466, 1600, 1687
 *   struct VPQ {Vpolar, PQb, PQL, Ib, IL, Qset_a/b/c}   fun_return.h:43-51
 *   plus the reductions VVC takes from each solve:
 *       loss        VoltVarCtrl.cpp:1152-1161
 *       Vmin/Vmax   VoltVarCtrl.cpp:1201-1207 with V_abc_list.cpp:7-81 and
 *                   Lnum_a/b/c of form_Yabc.cpp:46-58
 *
 * One fpf_solve_batch call evaluates B scenarios of one feeder: scenario s is
 * DPF_return7 on the feeder's Dl with columns 6..11 replaced by pq[.][.][s].
 * B = 1 with pq = Dl.colptr(6) is exactly one DPF_return7 call.
 *
 * Compiles as C89 and as C++98 -pedantic (the Broker builds with -std=c++98,
 * Broker/CMakeLists.txt:55): C linkage, <stddef.h> types only.
 *
 * Layout conventions
 *   Dl    : Nl x ncols (ncols >= 12) float64, column-major  (= arma::mat::memptr())
 *   Z     : z_rows x z_cols complex128, column-major, interleaved (re, im)
 *           (= reinterpret_cast<const double*>(arma::cx_mat::memptr()))
 *   pq    : [6][Nl][B] float64, scenario fastest; field order P1 Q1 P2 Q2 P3 Q3
 *           (= Dl columns 6..11).  For B = 1 this is Dl.colptr(6).
 *   per-scenario matrix outputs: [col][row][B], scenario fastest; for B = 1 each
 *           is the column-major Nn x 6 (or Nn x 3) Armadillo matrix of the VPQ field.
 *   Row k of every Nn-row output is node k (row 0 = substation), which is the
 *   Vpolar/PQb/PQL row order of DPF_return7.cpp:236-252.
 *
 * Error convention (no exceptions cross the ABI; the reference threw instead):
 *   return >= 0 : number of scenarios with status FPF_NONCONVERGED (results of
 *                 all scenarios are written; status[] says which)
 *   return <  0 : FPF_ERR_* ; fpf_last_error(ctx) has the message
 *
 * Threading: one fpf_ctx per host thread; calls on one ctx are not re-entrant.
 * fpf_solve_batch blocks until results are in host memory (the reference call
 * was synchronous on the Broker's io_service thread, CBroker.cpp:582-612).
 */
#ifndef FREEDM_PF_H
#define FREEDM_PF_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FPF_ABI_VERSION 3   /* 2: fpf_outputs.errmx / .guard, fpf_opts.no_guard;
                               3: FPF_EXCHANGE_FAILED, FPF_ERR_EXCHANGE, fpf_feeder_check */

/* return codes */
#define FPF_OK               0
#define FPF_ERR_ARG         -1   /* NULL / inconsistent argument                          */
#define FPF_ERR_TOPOLOGY    -2   /* Dl/Z index out of range: the reference's Armadillo     */
                                 /* bounds check throws std::logic_error here             */
#define FPF_ERR_HIP         -3   /* HIP runtime failure                                    */
#define FPF_ERR_NOMEM       -4
#define FPF_ERR_UNSUPPORTED -5   /* requested kernel cannot run this feeder               */
#define FPF_ERR_EXCHANGE    -6   /* a paired-kernel exchange wait gave up (feeders of     */
                                 /* 2049..4096 branches: two workgroups per scenario hand */
                                 /* their scan values over through L2); the scenarios     */
                                 /* concerned have status FPF_EXCHANGE_FAILED             */

/* per-scenario status */
#define FPF_CONVERGED        0
#define FPF_NONCONVERGED     1   /* no errmx < eps within mxitr sweeps; the reference     */
                                 /* throws (DPF_return7.cpp:100-101,242); we return the   */
                                 /* state after the last sweep                            */
#define FPF_EXCHANGE_FAILED  3   /* not a solve outcome: the two workgroups of a paired-  */
                                 /* kernel scenario could not exchange (a hardware or     */
                                 /* dispatch fault); V is not a result.  Counted neither  */
                                 /* as converged nor as non-converged in fpf_aggregate    */
                                 /* (n_scen - n_conv - n_nonconv of them)                 */

/* kernel selection */
#define FPF_KERNEL_AUTO      0   /* fast mode: wave if the feeder allows it; then tiled   */
                                 /* if the feeder is well formed, else generic            */
#define FPF_KERNEL_GENERIC   1   /* one lane per scenario, state streamed through HBM     */
#define FPF_KERNEL_TILED     2   /* one workgroup per scenario tile, state in LDS         */
#define FPF_KERNEL_WAVE      3   /* one wavefront per scenario, sweeps as prefix scans;   */
                                 /* fast mode, well-formed feeders of <= 256 branches     */

typedef struct fpf_ctx fpf_ctx;
typedef struct fpf_feeder fpf_feeder;

typedef struct fpf_opts {
    double bkva;       /* 1000         DPF_return7.cpp:11  */
    double bkv;        /* 12.47        :12                 */
    double vo_kv;      /* 12.47*1.015  :13                 */
    double eps;        /* 0.0001       :14                 */
    int    mxitr;      /* 20           :15                 */
    int    kernel;     /* FPF_KERNEL_*                     */
    double lb_v;       /* 0.96  load_system_data.cpp:23 (hosting counters) */
    double ub_v;       /* 1.05  load_system_data.cpp:24                    */
    int    tile;       /* scenarios per workgroup for the tiled kernel, 0 = auto */
    int    specialize; /* 1 (default): compile the tiled kernel for the feeder's topology
                          with hipRTC at fpf_feeder_create, and the wave / wave-block
                          kernel for its plan (its uniform values as constants), run by
                          launches of >= 4096 scenarios (FPF_WAVE_RTC=n: >= n, 0: never;
                          built by fpf_feeder_reserve or the first such launch, ~2.5 s
                          once per plan in a process; identical results -- a build that
                          fails or could not be resident runs the static kernel);
                          0: interpret the tiled programs, static wave kernels */
    int    exact;      /* 1: the specialised kernel repeats the reference's roundings
                          (complex divide as libgcc __divdc3, no FMA): V, PQb, PQL, loss
                          bit-identical to the oracle.  0 (default): load currents as
                          conj(S)V/|V|^2 and the branch products with FMA -- within a few
                          ulp (north-star bar: 1e-10 relative on V, same iteration counts).
                          The generic and interpreted kernels are always exact. */
    int    layout;     /* batch layout of pq and the matrix outputs (FPF_LAYOUT_*):
                          SCEN_FASTEST (0, default) pq [6][Nl][B], outputs [col][row][B];
                          SCEN_MAJOR (1) pq [B][6][Nl] -- the reference's per-call load
                          columns P1 Q1 P2 Q2 P3 Q3 of Dl (DPF_return7.cpp:46-50), one
                          scenario after another -- and outputs [B][col][row].  The
                          per-scenario scalars are [B] either way; B = 1 is the same. */
    int    no_guard;   /* 0 (default): fast-mode convergence guard.  The fast kernels sum
                          Ib(0) in another order than the reference, so a scenario whose
                          errmx lands within the rounding band of eps at some sweep could
                          stop one sweep apart from it (DPF_return7.cpp:199-210).  Such
                          scenarios are flagged in the kernel (band: 4 (Nb + 24) 2^-53
                          sum_k |IL_k|_1, the scan's worst-case rounding difference, with
                          sum_k |IL_k|_1 bounded by 1.25 sqrt(2) sum_k |S_k|_1 / min|V|
                          where the kernel forms it from the loads; fpf_api.cpp
                          guard_factor) and
                          re-solved on the exact kernel, whose decisions are the reference's
                          order of operations.  1: no guard (diagnostics). */
    int    reserved[3];
} fpf_opts;

#define FPF_LAYOUT_SCEN_FASTEST 0   /* [field][row][B]: a workgroup of consecutive scenarios reads rows */
#define FPF_LAYOUT_SCEN_MAJOR   1   /* [B][field][row]: one scenario is one contiguous block            */

typedef struct fpf_feeder_info {
    int nl;            /* rows of Dl                                  */
    int ncols;
    int nn;            /* cnt_nodes (DPF_return7.cpp:37)              */
    int nb;            /* rows with ln != 0                           */
    int n_codes;       /* line codes = max(z_rows/3, 1)               */
    int n_sep;         /* separator rows (ln == 0)                    */
    int n_taps;        /* distinct separator targets                  */
    int well_formed;   /* 1 if the tiled kernel can run it            */
    int lnum[3];       /* Lnum_a/b/c (form_Yabc.cpp:46-58)            */
    int depth;         /* longest root-to-leaf chain                  */
    int kernel;        /* kernel AUTO resolves to                     */
    int tile;          /* scenarios per workgroup (tiled)             */
    int specialized;   /* 1 if the tiled kernel is the hipRTC build   */
    int reserved[3];
} fpf_feeder_info;

/* Per-scenario outputs; every pointer may be NULL (= not produced).  Shapes
 * for FPF_LAYOUT_SCEN_FASTEST; FPF_LAYOUT_SCEN_MAJOR swaps B to the front.
 * The arrays must not overlap: the fast kernels stash a scenario's IL / Ib of
 * its last sweep in its own pql / pqb entries before writing the final values
 * (fpf_solve_batch_device returns FPF_ERR_ARG for overlapping ranges). */
typedef struct fpf_outputs {
    double      *vpolar;   /* [6][Nn][B]  |Va| angA |Vb| angB |Vc| angC (deg)  */
    double      *pqb;      /* [6][Nn][B]  branch P/Q (kW, kVAr)                */
    double      *pql;      /* [6][Nn][B]  load P/Q                             */
    double      *v_re;     /* [3][Nn][B]  complex node voltage (p.u.)          */
    double      *v_im;     /* [3][Nn][B]                                       */
    int         *iters;    /* [B] sweeps executed                              */
    signed char *status;   /* [B] FPF_CONVERGED / FPF_NONCONVERGED             */
    double      *loss;     /* [B] kW   (VoltVarCtrl.cpp:1152-1161)             */
    double      *vmin;     /* [B] p.u. (VoltVarCtrl.cpp:1201-1207)             */
    double      *vmax;     /* [B] p.u.                                         */
    double      *errmx;    /* [B] errmx = max_p |Ib(0,p) - Ibo(p)| of the scenario's last sweep,
                              the value tested against eps (DPF_return7.cpp:199-204)          */
    signed char *guard;    /* [B] 1: a convergence decision of the fast kernel fell within the
                              guard band and the scenario was re-solved on the exact kernel
                              (its results are the exact kernel's); 0 otherwise               */
} fpf_outputs;

/* Batch aggregate (the hosting-study reduction).  Also the payload of the
 * cross-GPU combine (one all-gather, folded in rank / device order by
 * fpf_aggregate_fold): fields 0 (sum) and 3..7 (sum), 1 (min), 2 (max). */
typedef struct fpf_aggregate {
    double loss_sum;   /* over converged scenarios                     */
    double vmin;       /* min over converged scenarios                 */
    double vmax;       /* max over converged scenarios                 */
    double n_conv;
    double n_nonconv;  /* status FPF_NONCONVERGED (FPF_EXCHANGE_FAILED is neither)        */
    double n_over;     /* converged with vmax > ub_v                   */
    double n_under;    /* converged with vmin < lb_v                   */
    double n_scen;
} fpf_aggregate;

int         fpf_abi_version(void);
void        fpf_opts_default(fpf_opts *opts);

int         fpf_ctx_create(int device, fpf_ctx **out);
void        fpf_ctx_destroy(fpf_ctx *ctx);
const char *fpf_last_error(const fpf_ctx *ctx);

/* Validate and upload a feeder (topology tables, Z/Zb, V0 live on the device). */
int         fpf_feeder_create(fpf_ctx *ctx, const double *dl, int nl, int ncols,
                              const double *z, int z_rows, int z_cols,
                              const fpf_opts *opts, fpf_feeder **out);
void        fpf_feeder_destroy(fpf_feeder *feeder);
int         fpf_feeder_get_info(const fpf_feeder *feeder, fpf_feeder_info *info);
/* Pre-size device scratch for batches up to max_scen (no allocation later); with
 * opts.specialize and FPF_WAVE_RTC, also build the wave kernel those batches run
 * (hipRTC, once per plan in a process) so that no solve pays for the compile. */
int         fpf_feeder_reserve(fpf_feeder *feeder, int max_scen);

/* Host-memory batch: copies in, solves, copies out; blocks.  agg may be NULL. */
int         fpf_solve_batch(fpf_feeder *feeder, int n_scen, const double *pq,
                            const fpf_outputs *out, fpf_aggregate *agg);

/* Device-memory batch: every pointer (pq, out fields, d_agg) is device memory;
 * enqueued on `stream` (a hipStream_t; NULL = the NULL/default stream, as in
 * every HIP API) and returns without synchronising.  d_agg (8 doubles, fpf_aggregate layout) may be NULL.
 * Any mix of solves on one feeder may be enqueued on different streams: the
 * library orders every launch that uses state of the feeder after the previous
 * such launch (an event per feeder) -- launches that produce an aggregate
 * (d_agg != NULL here, fpf_aggregate_device, fpf_solve_batch: the partials and
 * ticket), the generic and tiled kernels (scratch, layout copies), the paired
 * kernel (exchange areas), guarded solves whose flagged scenarios go to the
 * feeder's flag list and fixup kernel, and solves with NULL per-scenario scalar
 * outputs (they fall back to the feeder's buffers).  Solves on the wave kernels
 * (feeders of at most 2048 branches) with every per-scenario scalar output the
 * caller's, no aggregate and the guard resolved in the kernel's LDS (or
 * no_guard) use none of it and overlap freely.
 * Returns FPF_OK or an error (the non-converged count is in d_agg / status).
 * Asynchronous faults: a paired-kernel launch whose exchange gave up sets a
 * sticky word of the feeder (one per feeder, not per launch).  The next entry
 * on the feeder that reads it reports FPF_ERR_EXCHANGE once and clears it:
 * fpf_feeder_check; fpf_solve_batch_device at entry, before it enqueues anything
 * (its own batch is then NOT enqueued -- call it again); and the blocking entries
 * (fpf_solve_batch, fpf_vvc_*, fpf_areas_solve) after their own launches, where
 * the report may also come from an earlier asynchronous launch on the feeder
 * that nobody checked.  Call fpf_feeder_check after asynchronous launches to
 * attribute a fault to them. */
int         fpf_solve_batch_device(fpf_feeder *feeder, int n_scen, const double *d_pq,
                                   const fpf_outputs *d_out, double *d_agg, void *stream);
/* Wait for `stream` (a hipStream_t, NULL = the default stream), then report the
 * feeder's asynchronous faults: FPF_ERR_EXCHANGE if a paired-kernel launch on it
 * gave up an exchange since the last report (the word is cleared), else FPF_OK. */
int         fpf_feeder_check(fpf_feeder *feeder, void *stream);

/* ---- Multi-GPU study: one process, n GPUs of a node.
 * fpf_multi_create uploads the feeder to devices 0..n_gpus-1 (one context,
 * stream and feeder each) and builds an RCCL communicator over them
 * (ncclCommInitAll; xGMI inside an MI355X node).  fpf_multi_solve cuts the
 * batch into contiguous shards (fpf_multi_shard), solves every shard on its
 * device concurrently (pinned, double-buffered chunks: fpf_multi_schedule) and combines the per-device batch aggregates with one
 * grouped RCCL all-gather of the 8-double rows, folded in device order
 * (fpf_aggregate_fold: the same bits as dist.fold_aggregates) -- the only
 * exchange: per-scenario results go straight back to the caller's host arrays
 * at their global index.  pq / out / agg as fpf_solve_batch (host memory, the
 * whole batch's layout, either fpf_opts.layout).  Returns >= 0 (non-converged scenarios) or FPF_ERR_*.
 * With n_gpus = 1 the results equal fpf_solve_batch's bit for bit. */
typedef struct fpf_multi fpf_multi;
int         fpf_multi_create(int n_gpus, const double *dl, int nl, int ncols,
                             const double *z, int z_rows, int z_cols,
                             const fpf_opts *opts, fpf_multi **out);
void        fpf_multi_destroy(fpf_multi *m);
/* m = NULL: why the calling thread's last fpf_multi_create failed */
const char *fpf_multi_last_error(const fpf_multi *m);
int         fpf_multi_solve(fpf_multi *m, int n_scen, const double *pq,
                            const fpf_outputs *out, fpf_aggregate *agg);
/* the feeder handle of one device (for fpf_feeder_get_info, device batches) */
int         fpf_multi_get_feeder(fpf_multi *m, int device, fpf_feeder **out);
/* The partition (no device needed): scenarios [lo, hi) of `rank` out of
 * n_total over n_gpus, contiguous, sizes differing by at most one. */
int         fpf_multi_shard(int rank, int n_gpus, long n_total, long *lo, long *hi);
/* The order fpf_multi_solve issues its work in (no device needed): every
 * transfer goes through pinned staging in chunks of at most `chunk` scenarios,
 * double-buffered per device; round r issues chunk r of every device (pack,
 * H2D, solve, D2H; nothing waits) before it collects round r - 1 (wait,
 * unpack), so the devices run concurrently from one host thread.  ops[4 i ..]
 * = {kind (0 issue, 1 collect), device, lo, hi}; at most max_ops entries are
 * written; returns the number of operations or FPF_ERR_ARG. */
long        fpf_multi_schedule(int n_gpus, long n_scen, long chunk, long *ops, long max_ops);
/* The combine of the per-device aggregates, on the host (no device needed):
 * fpf_multi_solve all-gathers every device's aggregate (its one collective) and
 * folds the rows with this, in device order -- sums of fields 0 and 3..7
 * accumulated row after row, min of vmin, max of vmax; n = 0 gives the
 * identity.  The one-process-per-GPU form (freedm_amd/dist.py) folds the same
 * rows the same way, so both give the same bits. */
void        fpf_aggregate_fold(const fpf_aggregate *parts, int n, fpf_aggregate *out);
/* Diagnostics: collectives fpf_multi_solve has issued in this process (one per solve). */
long        fpf_multi_collectives(void);

/* ---- Multi-area solve (BASELINE config 5, the Broker_s1..s3 areas;
 * Broker_s1/src/vvc/VoltVarCtrl.cpp:327-395).  node_area[k] (k = 1..nn-1;
 * node_area[0] ignored) assigns every bus to an area; each area must be a
 * connected subtree, the area of bus 1 is the root.  Every area is solved as
 * its own feeder fed from its boundary bus (fast mode, wave kernel, the
 * opts' eps / mxitr), parents first, children's source power added to their
 * boundary bus as a load (the first outer iteration: the child subtree's total
 * load), until no boundary voltage moves by more than tol
 * (p.u.) or max_outer outer iterations.  This algorithm has no reference
 * counterpart: at its fixed point V is the monolithic solution (to the
 * solver tolerances).  out (host): v_re / v_im in the feeder's numbering,
 * iters = outer iterations, status, loss (sum of the areas' branch losses),
 * vmin / vmax; vpolar / pqb / pql must be NULL.  fpf_areas_last_error also
 * reports the last outer iteration's largest boundary move.  pq and out are
 * always FPF_LAYOUT_SCEN_FASTEST (opts.layout is ignored). */
typedef struct fpf_areas fpf_areas;
int         fpf_areas_create(fpf_ctx *ctx, const double *dl, int nl, int ncols,
                             const double *z, int z_rows, int z_cols,
                             const int *node_area, int nn, const fpf_opts *opts,
                             fpf_areas **out);
void        fpf_areas_destroy(fpf_areas *a);
const char *fpf_areas_last_error(const fpf_areas *a);
int         fpf_areas_info(const fpf_areas *a, int *n_areas, int *area_nodes, int *area_parent);
int         fpf_areas_solve(fpf_areas *a, int n_scen, const double *pq, double tol, int max_outer,
                            const fpf_outputs *out, fpf_aggregate *agg);

/* Diagnostics (no device needed): the hipRTC source fpf_feeder_create would
 * compile for this feeder's tiled kernel.  Writes at most buf_size bytes
 * (NUL-terminated) and returns the full size including the NUL, or FPF_ERR_*. */
long        fpf_feeder_rtc_source(const double *dl, int nl, int ncols,
                                  const double *z, int z_rows, int z_cols,
                                  const fpf_opts *opts, char *buf, size_t buf_size);

/* Diagnostics (no device needed): the hipRTC source of the wave kernel built for
 * this feeder's plan (its uniform values as constants; run by launches of >= n
 * scenarios when opts->specialize and FPF_WAVE_RTC=n, the static kernel otherwise).
 * big_batch: the large-batch workgroup size; full: the full-output variant.
 * Feeders of 257..2048 branches: the wave-block kernel's build.  Returns as
 * fpf_feeder_rtc_source; FPF_ERR_UNSUPPORTED if the feeder runs neither. */
long        fpf_feeder_wave_rtc_source(const double *dl, int nl, int ncols,
                                       const double *z, int z_rows, int z_cols,
                                       const fpf_opts *opts, int big_batch, int full,
                                       char *buf, size_t buf_size);
/* Diagnostics: the per-plan wave kernels built with hipRTC so far in this process. */
int         fpf_wave_rtc_builds(void);
/* Diagnostics (no device needed): compile src with the hipRTC the library uses
 * (the ROCm image's own, loaded into a private namespace so that a process which
 * loaded another HIP runtime first -- e.g. PyTorch's bundled one -- still compiles
 * with the compiler the static kernels were built with; fpf_rtc_compiler names
 * it) and the library's options (ilp: the static wave kernels' scheduler).
 * *regs (may be NULL): registers per lane (VGPRs + AGPRs) from the kernel
 * descriptor, the figure the library's residency check uses (-1: not found).
 * Writes at most buf_size bytes of the gfx950 code object and returns its full
 * size, or FPF_ERR_*. */
long        fpf_rtc_compile(const char *src, const char *name_expr, int ilp, int *regs,
                            char *buf, size_t buf_size);
const char *fpf_rtc_compiler(void);
/* Diagnostics (no device needed): the residency check the library applies to a
 * hipRTC build before loading it -- registers per lane x waves per SIMD <= 512,
 * static LDS (group segment) <= 160 KiB, and with max_priv >= 0 a private
 * segment of at most max_priv bytes per lane (the hot light-output wave builds:
 * 256, room for the call frame of the guard's exact re-solve but not for a
 * spilled sweep state; -1: no limit).  code/size: a gfx950 code object (as
 * fpf_rtc_compile writes it), kernel: its lowered kernel name, nt: threads per
 * workgroup.  regs / group / priv (may be NULL): the descriptor's registers per
 * lane, group segment and private segment bytes.  Returns 1 resident, 0 not,
 * FPF_ERR_ARG (no such kernel descriptor).
 *
 * The hipRTC the library compiles with is the ROCm image's own, loaded with
 * dlmopen into a private link-map namespace with its own libc; that libc's
 * environ is pointed at the process's environment array before every compile
 * (fpf_rtc.cpp: RtcApi::sync_env).  A compile therefore must not run while
 * another thread calls setenv / putenv, and nothing in the compiler may
 * modify the environment (it would reallocate the process's array with the
 * other libc's allocator); the library serialises its own compiles. */
int         fpf_rtc_resident(const char *code, size_t size, const char *kernel, int nt, int max_priv,
                             int *regs, int *group, int *priv);

/* Diagnostics (no device needed): the wave kernel's plan for this feeder.
 * out[0..7] = {accepted (1/0), scenarios per wavefront, slots per lane,
 * wavefronts per workgroup, LDS bytes per workgroup, gathered scan entries,
 * blocks, block-chain depth}.  Feeders of 257..2048 branches get the
 * wave-block kernel's plan: one scenario per workgroup of (wavefronts per
 * workgroup) wavefronts, reported with 1 scenario per wavefront; feeders of
 * 2049..4096 branches the paired kernel's (one scenario on two such workgroups
 * of 8 wavefronts, each holding half of the positions; LDS bytes per workgroup).
 * Returns FPF_OK or FPF_ERR_*. */
int         fpf_feeder_wave_plan(const double *dl, int nl, int ncols,
                                 const double *z, int z_rows, int z_cols,
                                 const fpf_opts *opts, int out[8]);

/* Diagnostics (no device needed): the lane kernel's plan for this feeder (one
 * lane per scenario, the feeder's positions dealt to the waves of a workgroup;
 * run by light-output scenario-fastest wave batches of >= n scenarios with
 * FPF_LANE=n).  out[0..7] = {accepted (1/0), slots per wave, waves per workgroup,
 * LDS bytes per workgroup, published backward entries, published forward
 * entries, blocks, branches}; slots (may be NULL): the first slots_len ints of
 * the per-slot table [waves][4][slots] = {Dl row, node (-1: dummy), backward
 * info, forward info}; blk (may be NULL): the first blk_len ints of the block
 * table [blocks][1 + 2 x 8] = {depth, (tap, first - 1) forward entries}.
 * Returns FPF_OK or FPF_ERR_*. */
int         fpf_feeder_lane_plan(const double *dl, int nl, int ncols,
                                 const double *z, int z_rows, int z_cols,
                                 const fpf_opts *opts, int out[8], int *slots, int slots_len,
                                 int *blk, int blk_len);
/* Diagnostics: launches of the lane kernel in this process; of those, the
 * launches that read the loads through the LDS-DMA ring (FPF_LANE_DMA=1, even
 * batches whose ring fits in LDS). */
int         fpf_lane_launches(void);
int         fpf_lane_dma_launches(void);

/* Device-memory batch aggregate over per-scenario results (deterministic
 * reduction); same layout as fpf_aggregate.  Lets a caller aggregate several
 * batches, or time the solve kernel alone. */
int         fpf_aggregate_device(fpf_feeder *feeder, int n_scen, const signed char *d_status,
                                 const double *d_loss, const double *d_vmin, const double *d_vmax,
                                 double *d_agg, void *stream);

/* Batched VVC step-size search: the reference's line search over the step
 * sizes of one gradient (VoltVarCtrl.cpp:1316-1542; the reversed search
 * :1544-1762 is the same call with a negative c0), as ONE batch.  Candidate m
 * is the control ctrl_dl with, for every load i of phase x (x = a, b, c) and
 * every row whose rbus == load_nodes[x][i] (:1334-1372),
 *     Dl(row, 7 + 2x) = ctrl_dl(row, 7 + 2x) - g[x][i] * (bkva/3) * c_m,
 *     c_0 = c0, c_{m+1} = alpha * c_m                      (:1321-1323, :1420-1422)
 * for m = 0 .. m_max.  The stop rule is the reference's: the first m with
 * loss(c_{m+1}) > loss(c_m) (:1484); on the way the direction flag drops when a
 * kept loss exceeds ploss_orig (:1530-1536).  The reference calls DPF_return7
 * 2 m + 1 times sequentially and throws on a non-converged solve. */
typedef struct fpf_line_search {
    int     stop;          /* the m whose candidate is kept (Dl_osize), -1: none within m_max */
    int     reverse;       /* 1: the reference reverses the gradient direction (flag = false) */
    int     first_nonconv; /* first m that does not converge (the reference throws), -1: none */
    int     reserved;
    double *loss;          /* [m_max + 1] caller-owned: loss at c_m (kW), required            */
    double *vmin;          /* [m_max + 1] caller-owned or NULL                                */
    double *vmax;          /* [m_max + 1] caller-owned or NULL                                */
} fpf_line_search;

/* g, load_nodes: [3][ld] row-major (phase-major), n_loads[3] <= ld entries used
 * per phase; ctrl_dl: Nl x ncols column-major with the feeder's topology.
 * Returns >= 0 (non-converged candidates) or FPF_ERR_*. */
int         fpf_vvc_line_search(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols,
                                const double *g, const double *load_nodes, const int *n_loads, int ld,
                                double c0, double alpha, int m_max, double ploss_orig,
                                fpf_line_search *res);

/* The VVC gradient (VoltVarCtrl.cpp:1141-1325): one DPF of ctrl_dl on the
 * device, then on the host, per phase: the self-impedance admittance matrix
 * (form_Yabc.cpp), V_abc_list, rename_brn, dF/dtheta, dF/dV and the Jacobian
 * (form_Ftheta.cpp, form_Fv.cpp, form_J.cpp; long double sums as the
 * reference), lambda = -inv(J^T) Fx and g_vq = -gu^T lambda.  z is the
 * feeder's Z (fpf_feeder_create's layout).  g, load_nodes: [3][ld] (phase
 * major), n_loads[3] = Lla/Llb/Llc; stats[8] (may be NULL) = gmin, gmax,
 * gabs_min, c0 = beta0/(bkva/3)/gabs_min, Ploss_orig, Vmin_orig, Vmax_orig,
 * sweeps of the base solve.  Returns FPF_OK or FPF_ERR_* (FPF_ERR_UNSUPPORTED:
 * the base solve did not converge -- the reference throws). */
int         fpf_vvc_gradient(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols,
                             const double *z, int z_rows, int z_cols, double beta0, int ld,
                             double *g, double *load_nodes, int *n_loads, double *stats);

/* The same gradient at a given DPF result (no device needed): vpolar is the
 * solve's Vpolar (nn x 6, column-major, substation first); stats[4] (may be
 * NULL) = gmin, gmax, gabs_min, c0.  Returns FPF_OK or FPF_ERR_*. */
int         fpf_vvc_gradient_at(const double *ctrl_dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
                                const double *vpolar, int nn, double bkva, double bkv, double beta0, int ld,
                                double *g, double *load_nodes, int *n_loads, double *stats);

/* The gradient of n_scen scenarios of one control table as one batch (the
 * gradient stage of VoltVarCtrl.cpp:1141-1325 per scenario, for a VVC Monte
 * Carlo over load scenarios): scenario s is ctrl_dl with its load columns 6..11
 * replaced by pq[.][.][s] (host, [6][Nl][n_scen], scenario fastest).  The base
 * solves, the V lists, Fx, J (long double sums as double-double), the LU solves
 * (a hand-written batched LU with partial pivoting, one workgroup per matrix, its
 * pivot row and column in LDS: at most 3200 load nodes per phase) and g run on
 * the device; Y,
 * the branch lists and the load lists are shared.  Every scenario's (int) load
 * tests (columns 6, 8, 10) must equal ctrl_dl's (else FPF_ERR_ARG): they fix the
 * load lists.  g [n_scen][3][ld]; load_nodes [3][ld] and n_loads [3] (shared);
 * stats [n_scen][8] = gmin, gmax, gabs_min, c0, Ploss_orig, Vmin_orig,
 * Vmax_orig, sweeps; gstatus [n_scen]: 0 ok, 1 the base solve did not converge
 * (the reference throws), 2 singular J, 3 V_abc_list rows differ from the first
 * converged scenario's (g and stats[0..3] are 0 unless 0).  Returns the number
 * of scenarios with gstatus != 0, or FPF_ERR_* (FPF_ERR_UNSUPPORTED: a phase
 * with more than 3200 load nodes -- fpf_vvc_gradient solves those on the host;
 * FPF_ERR_EXCHANGE: a paired-kernel base solve's exchange gave up).  Its device
 * scratch (the batch's loads and base-solve outputs, the plan, the dense J^T of a
 * chunk of scenarios per phase -- up to 2 GB a phase on large feeders) and a few
 * pinned host buffers stay with the feeder for the next call (and for
 * fpf_vvc_round_batch) until fpf_feeder_destroy. */
int         fpf_vvc_gradient_batch(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols,
                                   const double *z, int z_rows, int z_cols, int n_scen, const double *pq,
                                   double beta0, int ld, double *g, double *load_nodes, int *n_loads,
                                   double *stats, signed char *gstatus);

/* One whole VVC round of vvc_main (VoltVarCtrl.cpp:1141-1762): the gradient,
 * the step-size search batched (fpf_vvc_line_search's candidates: the first 32
 * step sizes as one batch, the rest as a second only when the stop rule has not
 * fired among the first), and the reversed search when the reference reverses.
 * loss_fwd / loss_rev [m_max + 1] (loss_rev may be NULL; NaN for the step sizes
 * past the stop that were not solved -- the reference never solves a candidate
 * past stop + 1), dl_out (nl x ncols): the control after the round (the kept
 * candidate, Dl = Dl_osize, :1486/1707; else ctrl_dl).  res[13] = Ploss_orig,
 * Vmin_orig, Vmax_orig, c0, stop_fwd, stop_rev, reversed, sent (the S2
 * set-points go to the slaves, :1495/1716), Ploss_after, gmin, gmax,
 * gabs_min, nonconverged (a candidate the reference solves did not converge:
 * it throws).  Returns 0, 1 (nonconverged) or FPF_ERR_*. */
int         fpf_vvc_round(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols,
                          const double *z, int z_rows, int z_cols, double beta0, double alpha,
                          int m_max, int ld, double *g, double *load_nodes, int *n_loads,
                          double *loss_fwd, double *loss_rev, double *dl_out, double *res);

/* One whole VVC round per load scenario (VoltVarCtrl.cpp:1141-1762 for a VVC
 * Monte Carlo): scenario s is ctrl_dl with its load columns 6..11 replaced by
 * pq[.][.][s] (host, [6][Nl][n_scen]).  The gradients as fpf_vvc_gradient_batch
 * (same arguments and rules: every scenario's (int) load tests must be the
 * control's); then every scenario's step sizes as device batches (the first 32
 * of every search as one, the rest of the searches whose stop rule has not
 * fired as a second), the reference's stop rule per scenario, and the same for
 * the scenarios whose search reverses (:1544-1762).  Per scenario: loss_fwd /
 * loss_rev [n_scen][m_max + 1] (may be NULL; rows of scenarios that do not
 * reverse are left as they are; NaN for step sizes not solved, past the stop),
 * pq_out [6][Nl][n_scen] the scenario's loads after the round
 * (the kept candidate's Q set-points, Dl = Dl_osize), res [n_scen][13] as
 * fpf_vvc_round's, rstatus [n_scen] the gradient's gstatus (0: the round ran).
 * Returns the number of scenarios with rstatus != 0 or a non-converged candidate
 * the reference would have solved (res[12]), or FPF_ERR_*. */
int         fpf_vvc_round_batch(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols,
                                const double *z, int z_rows, int z_cols, int n_scen, const double *pq,
                                double beta0, double alpha, int m_max, int ld, double *g,
                                double *load_nodes, int *n_loads, double *loss_fwd, double *loss_rev,
                                double *pq_out, double *res, signed char *rstatus);

/* Diagnostics: on-device check, over n seeded operand sets, that the
 * shared-reciprocal division the tiled kernel uses gives the same bits as the
 * compiler's a / b and as the libgcc __divdc3 complex division.  Returns the
 * number of mismatching results (0 expected) or FPF_ERR_*. */
long        fpf_selftest_division(int device, long n, unsigned long seed);

#ifdef __cplusplus
}
#endif
#endif /* FREEDM_PF_H */
