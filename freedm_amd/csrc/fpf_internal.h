// fpf_internal.h -- tables shared by the host side (fpf_api.cpp) and the gfx950
// kernels (fpf_kernels.hip).  Everything the kernels read about a feeder is
// precomputed once by fpf_feeder_create and lives in device memory.
#pragma once
#ifdef __HIPCC_RTC__
// hipRTC (topology-specialised tiled kernel, fpf_rtc.cpp): no system headers
using __hip_internal::int8_t;
using __hip_internal::int16_t;
using __hip_internal::int32_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
#define INFINITY __builtin_huge_val()
// the per-scenario status values of include/freedm_pf.h
#define FPF_CONVERGED 0
#define FPF_NONCONVERGED 1
#define FPF_EXCHANGE_FAILED 3
#else
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/freedm_pf.h"

#include <array>
#include <string>
#include <vector>
#endif

namespace fpf {

// One forward-sweep update V(dst) = V(src) - lng * (Ib(ib) . Zl(code)), then
// phase p zeroed when bit p of mask is set (DPF_return7.cpp:163-195).
// src < 0 means the constant V0 (the special first branch, :168).
struct FwOp {
    int32_t dst, src, ib, code, mask, pad;   // generic kernel: pad & 1 = src is the previous op's dst
};

// Backward-sweep op (DPF_return7.cpp:136-160), executed in list order:
//   kind 0 (branch)    : Ib[idx] = (Ib[idx] + Ibl) + IL[idx];  Ibl = Ib[idx]
//   kind 1 (separator) : Ib[idx] = Ib[idx] + Ibl;              Ibl = 0
//   kind | 2           : first op on Ib[idx] in the sweep: Ib[idx] reads as 0
struct BwOp {
    int32_t kind, idx;
};

// Load-current op (DPF_return7.cpp:107-130): IL[ndr-1] = conj(Sld[row]/V[ndr]).
struct IlOp {
    int32_t row, ndr;
};

// Per-node table of the tiled kernel (well-formed feeders only): node k >= 1
// owns exactly one branch row; the forward op writing V(k) and the load
// current IL(k-1) both belong to that row.
struct NodeOp {
    int32_t fw;      // index of the node's forward op (its TEMP block in FeederDev.tz)
    int32_t row;     // Dl row whose rbus == k (loads of the node)
    int32_t code;    // 0-based line code
    int32_t mask;    // phase-zeroing bits (0 for the special first branch)
    int32_t tap;     // tap-accumulator slot, -1 if no separator targets k
    int32_t slot;    // LDS state slot of node k (k itself in the interpreted layout,
                     // its schedule cell in the multi-track layout of fpf_rtc.cpp)
    int32_t pad[2];
};

// Sequential-stage programs of the tiled kernel, built for one tile size (LDS
// byte offsets are baked in).  LDS holds W = (nn + 2) slots x 3 phases x TILE
// scenarios of complex fp64 -- slot nn is a permanent zero, slot nn+1 a dummy
// sink -- then the tap accumulators T = (n_taps + 2) slots laid out the same way
// (zero and dummy last).  A sequential lane (s, p) adds its own lane offset
// (p*TILE + s)*16 to every offset.
//
// Backward program (one op per branch row, reverse row order; a separator row
// is folded into the branch op processed just before it):
//     x = (T[a] + Ibl) + W[r];  W[w] = x;  T[p] += x (if sep);  Ibl = sep ? 0 : x
// Forward program (one op per branch row, row order):
//     V = (prev ? Vprev : W[src]) - W[dst];  zero phases in mask;  W[dst] = V
// Both run in chunks of SEQ_CHUNK ops whose LDS reads are all issued first; the
// host pads chunks with identity ops so no op reads what an earlier op of its
// chunk writes.
constexpr int SEQ_CHUNK = 8;
struct SeqBw { uint32_t r, w, a, p; };     // byte offsets; p bit 31 = separator (T[p] += x; Ibl = 0)
struct SeqFw { uint32_t dst, src, flags, pad; };  // flags: bits 0-2 zero mask, bit 3 = src is previous op
constexpr uint32_t BW_SEP = 0x80000000u;
constexpr uint32_t FW_PREV = 8u;

struct FeederDev {
    // sizes
    int32_t nl, nn, ncode;
    int32_t n_il, n_bw, n_fw;
    int32_t K[3];            // Lnum_p + 1 (V_abc_list.cpp:12-17)
    int32_t n_taps, mxitr;
    // constants
    double V0[6];            // re/im per phase (DPF_return7.cpp:84-89)
    double s3;               // bkva / 3
    double eps;
    double lb_v, ub_v;
    // device tables
    const double *tz;        // [n_fw][3][3] complex interleaved: TEMP(L,a) of each
                             // forward op = cx(lng,0)*cx(1,0)*(Z(L,a)/Zb)
    const IlOp *il_ops;
    const BwOp *bw_ops;
    const FwOp *fw_ops;
    const NodeOp *node_ops;  // [nn] (index 0 unused) -- tiled only
    const SeqBw *seq_bw;     // tiled only (padded to SEQ_CHUNK)
    const SeqFw *seq_fw;     // tiled only (padded to SEQ_CHUNK)
    int32_t n_seq_bw, n_seq_fw;
    int32_t tile;            // tile the programs were built for
    int32_t prog_lds;        // 1: stage the programs in LDS; 0: read them from global memory
    int32_t n_slots;         // LDS state slots of the specialised (multi-track) layout
    int32_t slot_bytes;      // bytes per state slot of the specialised layout (padded, see fpf_api.cpp: bank_layout)
    int32_t phase_bytes;     // bytes between the phases of one slot (specialised layout)
    int32_t temp_lds;        // specialised layout: TEMP blocks staged in LDS
    const IlOp *bw_il;       // generic only, [n_bw]: the load-current op whose IL the
                             // branch op reads (the slot's last writer), row < 0: none
    // generic kernel, what a launch must initialise: the IL / Ib slots no op ever
    // writes (zeroed once), and whether V needs its V0 fill (v_init = 0: every V
    // read is of a slot a forward op wrote earlier in the sweep or in the last
    // sweep, so only V(0) is stored and sweep 0's load currents use V0)
    int32_t n_il_zero, n_ib_zero, v_init;
    const int32_t *il_zero, *ib_zero;
};

// Wave kernel (fpf_wave.hip, fast mode): SPW scenarios per wavefront, one
// segment of L = 64/SPW lanes per scenario, state in registers, both sweeps as
// segment-wide prefix scans over a depth-first order of the feeder tree in
// which every block (Dl row run between separators) is contiguous.  Node at
// position q (0..n-1) lives in slot c = q % C of segment lane q / C; per-slot
// tables are segment-lane-major, index (field*C + c)*L + lane.  Only the scan
// values other slots read (subtree ends, taps, zeroed ancestors) go through
// LDS, at a compact index.
struct WaveDev {
    int32_t n, nn, nl;       // branches (= nodes - 1), nodes, Dl rows
    int32_t spw, C;          // scenarios per wave, slots per lane
    int32_t nblk, bdepth;    // blocks, block-ancestor pairs of the deepest block
    int32_t ncomp;           // gathered positions (compact scan array; entry ncomp = 0)
    int32_t has_rel;         // some unmasked (node, phase) below a zeroed ancestor
    int32_t has_mask;        // some (node, phase) zeroed
    int32_t mxitr;
    int32_t K[3];            // Lnum_p + 1 (V_abc_list.cpp:12-17)
    int32_t dbg;             // diagnostic ablations (FPF_WAVE_DBG; results are wrong when set)
    int32_t wpb;             // wavefronts per workgroup (16, 8 or 4; fpf_api.cpp: analyse_wave)
    int32_t off_in_x;        // 1: block offsets stored over X's first nblk entries (nblk <= L, depth <= 4)
    int32_t stag_lo, stag_hi, stag_n;   // workgroups [lo, hi) start stag_n x 1 k cycles late (diagnostic)
    int32_t temp_sym;        // 1: every branch's TEMP has one common off-diagonal zm (transposed
                             //    line / transformer): slot_temp holds (z_aa - zm) x 3, zm per slot
    int32_t spec;            // 1: large launches run the per-feeder hipRTC build (fpf_opts.specialize;
                             //    fpf_rtc.cpp: wave_rtc_function), 0: the static kernel only
    double V0[6], s3, eps, lb_v, ub_v;
    const int32_t *slot_row;    // [C][L] Dl row of the slot's node (-1: empty slot)
    const int32_t *slot_node;   // [C][L] node id
    const int32_t *slot_info;   // [C][L] bits 0-2 zero mask, 3 valid, 4-12 backward index + 1 (the
                                //        slot's store), 13-21 backward index of the subtree's last
                                //        node (its gather), 22-30 forward index + 1 (its store)
    const int32_t *slot_blk;    // [C][L] block of the slot's node
    const int32_t *slot_mref;   // [3][C][L] forward index of the nearest zeroed proper ancestor, -1 none
    const double *slot_temp;    // [9][C][L] complex: TEMP = lng*Z/Zb of the node's branch, row-major
                                // (l, a); temp_sym: [4][C][L] (z_aa - zm for a = 0..2, zm)
    const int32_t *blk_pairs;   // [bdepth][2][nblk] (plus, minus) forward indices; pad = ncomp (zero)
    // per-workgroup staging of a tile's loads (fpf_wave.hip, wave_stage_tables): for
    // chunk c = u NT + t (16 bytes of pq) the STG double index of each of its two
    // halves; scenario-major {dst0, dst1}, scenario-fastest {pq line, dst0}
    // (dst1 = dst0 + 2); stage_u chunks per thread, 0: no tables (generic walk)
    const int32_t *stage_smaj, *stage_l0;
    int32_t stage_u;
    // the V write-out, table-driven: element i = u NT + t of the tile's V block
    // ([SPB][3][Nn] scenario major, [3 Nn][SPB] scenario fastest) at STG double2
    // index out_*[i] (row 0: the scenario's V0S); out_u per thread, 0: none
    const int32_t *out_smaj, *out_l0;
    int32_t out_u;
    // per-wave IO (scenario major, wave_io_units): a wave stages its own
    // scenarios' loads (stage_uw chunks per lane of the stage_smaj table) and
    // writes its own V (out_uw elements per lane of out_smaj) -- no workgroup
    // barrier waits for the slowest wave's loads or sweeps; 0: the workgroup's IO
    int32_t stage_uw, out_uw;
    // the sequential-order plan (fpf_api.cpp: analyse_wave_lag; FULL variant only):
    // per slot the extra backward pair of a post-add target and the index of the
    // previous sweep's V the slot stores (slot_lagx: hi | lo << 9 | (index + 1) << 18),
    // per block its chain's base (blk_base: -1 V0, else that index); nlag entries
    int32_t has_lag, nlag;
    const int32_t *slot_lagx, *blk_base;
    double rv0[3];              // 1/|V0_p|^2 (the flat start's first load currents)
    // wave-block kernel (fpf_wblk.hip): one scenario per workgroup of wps
    // wavefronts (L = 64 wps lanes, C slots per lane) for feeders of 257..2048
    // branches; wps = 0: the per-wavefront kernel above.  TEMP = lng * Zl(code)
    // factorised: per slot lng and code, per code Zl (temp_sym: z_aa - zm x 3, zm;
    // else the 9 entries row-major (l, a))
    int32_t wps, ncode;
    // convergence guard (fpf_opts.no_guard = 0): a decision whose errmx lies within
    // guard_k * sum_k |IL_k|_1 of eps is flagged for the exact re-solve
    // (fpf_api.cpp: guard_factor); 0 = off
    double guard_k;
    const double *slot_lng;     // [C][L]
    const int32_t *slot_code;   // [C][L] 0-based line code
    const double *code_z;       // [ncode][4 or 9] complex
    // paired wave-block kernel (fpf_wcoop.hip): feeders of 2049..4096 branches, one
    // scenario on coop = 2 workgroups (8 wavefronts, C = 4 each), workgroup g holding
    // the positions [g P, ...) of the depth-first order; the per-slot tables are
    // [2][C][L].  slot_info there: bits 0-2 zero mask, 3 valid, 4-17 backward index
    // + 1, 18-31 the subtree end's backward index (unsigned); slot_info2: forward
    // index + 1.  Backward / forward indices number the gathered positions in
    // position order, so workgroup 1 owns the entries from nb_split / nf_split on.
    // The two workgroups exchange their scan values through xch (coop_nslot areas
    // of coop_area doubles, one per scenario in flight) and xsync (arrival counts
    // [nslot], area generations [nslot], error word).  coop = 0: not this kernel.
    int32_t coop, nb_c, nf_c, nb_split, nf_split, coop_nslot, coop_area;
    const int32_t *slot_info2;
    double *xch;
    unsigned *xsync;
    double *xvm;                // zeroed phases: per area [3][nn] |V| of the last sweep (the V_abc_list ranking)
    unsigned *xerr_host;        // sticky: set (system scope) when an exchange wait gave up; pinned host memory
    int32_t coop_spin;          // polls before a wait gives up (2^21; FPF_TEST_COOP_SPIN overrides, tests only)
};

// Lane kernel (fpf_lane.hip, fast mode, feeders of at most LANE_NW * LANE_NS
// branches): one lane per scenario, 64 scenarios per workgroup of LANE_NW
// wavefronts; the depth-first positions are dealt to the waves in contiguous
// runs, position q of wave w in slot i (q = first_w + i), the slot's V (then its
// scan values) in that wave's registers for the whole solve.  Every wave runs
// the same code; what differs per slot is wave-uniform data read with scalar
// loads.  The waves meet in LDS (per-lane columns: one scenario per lane in
// every wave) at four barriers per sweep.
constexpr int LANE_NW = 8, LANE_NS = 16, LANE_BD = 8, LANE_TW = 8;
struct LaneDev {
    int32_t n, nn, nl;       // branches, nodes, Dl rows
    int32_t nE, nG;          // published backward (subtree-end) / forward (tap, first - 1) entries
    int32_t nblk, mxitr;
    double V0[6], rv0[3], s3, eps, lb_v, ub_v, guard_k;
    // [LANE_NW][4][ns] per wave, per field, per slot (a wave's run padded with
    // dummy slots: row 0, node -1, gather the zero entry, block of the wave's last
    // position): Dl row; node id; backward info: bit 0 a real slot, bits 1-15
    // published index + 1 (a subtree end), bits 16-31 the index the slot gathers
    // (its subtree's end; the zero entry for a dummy); forward info: bits 0-15
    // published index + 1, bits 16-29 block, bit 30 the slot starts a block or is
    // the wave's first (its V offset is resolved there)
    const int32_t *slot;
    // [LANE_NW][ns][LANE_TW]: TEMP as z_aa - zm (a = 0..2), zm (complex), 0 on a
    // dummy slot
    const double *temp;
    int32_t ns;              // slots per wave (4, 8, 12 or 16: the kernel instantiation)
    const int32_t *blk;      // [nblk][1 + 2 LANE_BD]: depth, then (tap, first - 1) forward indices
    int32_t stagger;         // cycles the first-round workgroups of every other CU wait (launch_lane)
};

// Device views of the caller's output buffers ([col][row][B], scenario fastest).
struct OutDev {
    double *vpolar, *pqb, *pql, *v_re, *v_im;
    int32_t *iters;
    int8_t *status;
    double *loss, *vmin, *vmax;
    // fused batch aggregate (specialised kernel): agg != NULL -> every workgroup
    // publishes its tile's 8 partials, the last one to arrive combines them
    double *agg;
    double *partials;        // [grid][8]
    unsigned *ticket;        // arrival counter, 0 between launches
    // wave kernel only (the multi-area solve, fpf_areas.cpp): per-scenario
    // source voltage [6][B] (re/im per phase) in place of V0, and the power
    // entering at the source [6][B] = PQb row 0 (P1 Q1 P2 Q2 P3 Q3, kW / kVAr)
    const double *vsrc;
    double *s_in;
    // batch layout (fpf_opts.layout) of pq and the matrix outputs: 0 [field][row][B],
    // 1 [B][field][row] (the wave kernels read / write it natively; the host
    // transposes around the generic and tiled kernels, fpf_layout.hip)
    int32_t smaj;
    // per-scenario errmx of the last sweep and the guard flag (fpf_outputs; may be NULL)
    double *errmx;
    int8_t *guard;
    // fast kernels with the guard on: scenarios whose convergence decision fell in the
    // guard band, appended as they finish (flag_ids [B]); NULL = guard off.  flag_out
    // (host API): the aggregating workgroup copies the final count there
    unsigned *flag_count;
    int32_t *flag_ids;
    unsigned *flag_out;
    // the guard's local mode (wave kernel, a solve without an aggregate): each
    // workgroup re-solves the scenarios it flagged itself on the exact body
    // (fpf_generic_body.h: g3_fixup_local) with fix_dev's op lists, its state in
    // the workgroup's LDS; fix_dev = NULL: the flags go to the batch's list and a
    // dpf_fixup_kernel launch re-solves them
    const struct FeederDev *fix_dev;
    // the multi-area solve's device-side stop (fpf_areas.cpp): *skip != 0 -> the
    // launch does nothing (the outer loop has converged; later iterations were
    // enqueued before the host looked).  NULL: always solve.  Wave kernels only.
    const int32_t *skip;
    // the multi-area solve's warm start (wave kernels, [field][row][B] batches only):
    // the sweeps start from these voltages ([3][Nn][B] re / im, the previous outer
    // iteration's V of the area) instead of the flat V0 of DPF_return7.cpp:92-96.
    // NULL: the reference's flat start
    const double *vinit_re, *vinit_im;
    // the multi-area solve's links folded into the solve (plain wave kernel only,
    // fpf_areas.cpp): device memory, NULL: none.  move: the outer iteration's
    // boundary-move slot (an atomic max of the double's bits)
    const struct AreaHook *hook;
    unsigned long long *move;
    // the convergence test's eps for this launch (device memory; wave kernel, no
    // guard); NULL: fpf_opts.eps
    const double *eps_dev;
    // the multi-area solve's stop test fused into the last area's solve: the
    // workgroup that takes the last ticket runs areas_stop_test(*check, ctl)
    // (ctl = the skip flag's array).  NULL: none
    const struct AreaLink *check;
    unsigned *check_ticket;
};

// The exact re-solve of flagged scenarios (fpf_generic.hip: dpf_fixup_kernel):
// scenario flag_ids[j] of the batch (B scenarios, layout smaj) for j < *flag_count,
// outputs at their batch index, then the batch aggregate again if agg != NULL;
// the count is reset to 0 for the next launch.
constexpr int FIXUP_BLOCKS = 1;   // one workgroup: 4 x 21 scenarios per pass

// (device-visible: also compiled by hipRTC, fpf_rtc.cpp)
// the multi-area solve's fused exchange kernels (fpf_areas_kernels.hip): up to
// AREA_MAX_KIDS children of one area per launch -- the local row of a child's
// bus and its source power (add_rows), or the child's boundary bus and its
// source-voltage array (gather_vsrc_all)
constexpr int AREA_MAX_KIDS = 8;
struct AreaKids {
    int n;
    int lrow[AREA_MAX_KIDS];
    double *ptr[AREA_MAX_KIDS];
};
// the links of one area folded into its wave-kernel solve (OutDev::hook): after
// the loads are staged, the rows its children hang off get the children's source
// powers added (pre: base + s_in, scaled like the loads); after the sweeps, each
// child's boundary bus voltage (local node post_lb >= 1) becomes its source
// voltage and the largest move joins *OutDev::move
struct AreaHook {
    int pre_n, post_n;
    int pre_lrow[AREA_MAX_KIDS], post_lb[AREA_MAX_KIDS];
    const double *pre_sin[AREA_MAX_KIDS];
    double *post_vsrc[AREA_MAX_KIDS];
};
// the per-scenario results of up to AREA_MAX_FOLD areas, folded in one launch
constexpr int AREA_MAX_FOLD = 8;
struct AreaFold {
    int n, first;
    const double *loss[AREA_MAX_FOLD], *vmin[AREA_MAX_FOLD], *vmax[AREA_MAX_FOLD];
    const int8_t *status[AREA_MAX_FOLD];
};
// one launch between two area solves of an outer iteration (fpf_areas.cpp): the
// solved area's children's source voltages (post; V [3][nn][B]), the next area's
// child rows (pre; work / base [6][nl][B]), the iteration's stop test (check)
struct AreaLink {
    const double *v_re, *v_im;
    int nn, nl;
    AreaKids post, pre;
    double *work;
    const double *base;
    unsigned long long *move_acc, *move_chk, *move_clr;   // the iteration's move (two slots, by parity)
    double *last;
    double tol;
    int check, single;
    // inexact outer iterations (check): the next iteration's inner eps
    // *eps_dev = clamp(inexact * move, eps, eps_first); stop only after an
    // iteration solved to eps itself.  eps_dev NULL: every solve to eps
    double *eps_dev;
    double eps, eps_first, inexact;
};
// the end of an outer iteration (link_kernel, or the last workgroup of the last
// area's solve: OutDev::check), once every boundary move of the iteration is in:
// the outer count, the move, the next iteration's inner eps, the stop flag ctl[0]
__device__ inline void areas_stop_test(const AreaLink &L, int32_t *ctl) {
    const double m = __longlong_as_double((long long)*L.move_chk);
    const int outer = ctl[1] + 1;
    ctl[1] = outer;
    *L.last = m;
    *L.move_clr = 0ull;
    bool exact = true;   // this iteration's solves ran to eps
    if (L.eps_dev) exact = *L.eps_dev <= L.eps;
    const bool done = L.single || (outer > 1 && m <= L.tol && exact);
    // (the first iteration's move compares with the previous solve's source
    // voltages: it does not set the next eps)
    if (L.eps_dev) *L.eps_dev = outer == 1 ? L.eps_first : fmax(L.eps, fmin(L.eps_first, L.inexact * m));
    if (done) ctl[0] = 1;
}

#ifndef __HIPCC_RTC__
}  // namespace fpf
struct fpf_feeder;
namespace fpf {
int ctx_device(const fpf_ctx *ctx);   // the HIP device of a context
// fpf_solve_batch_device with the wave kernel's two extra per-scenario arrays
// (OutDev::vsrc, OutDev::s_in; both device memory, may be NULL)
int solve_batch_device_ex(fpf_feeder *f, int n_scen, const double *d_pq, const fpf_outputs *d_out, double *d_agg,
                          void *stream, const double *d_vsrc, double *d_s_in, int layout,
                          unsigned *d_flag_out = nullptr, const int32_t *d_skip = nullptr,
                          const double *d_vinit_re = nullptr, const double *d_vinit_im = nullptr,
                          const AreaHook *d_hook = nullptr, unsigned long long *d_move = nullptr,
                          const double *d_eps = nullptr, const AreaLink *d_check = nullptr,
                          unsigned *d_check_ticket = nullptr);
// the exact re-solve of the scenarios a deferred (d_flag_out) guarded solve flagged
int fixup_batch_device(fpf_feeder *f, int n_scen, const double *d_pq, const fpf_outputs *d_out, double *d_agg,
                       void *stream, int layout);
// record msg as the feeder's context's last error (fpf_last_error) and return code
int feeder_fail(fpf_feeder *f, int code, const std::string &msg);
// Scratch of the VVC batch paths (fpf_vvc_grad.cpp), cached on the feeder by slot
// across calls: device memory (or pinned host memory, host = true) of at least
// `bytes`, grown on demand (the only hipMalloc / hipFree of a repeated call),
// freed with the feeder.  nullptr on failure (the feeder's context has the error).
void *feeder_buf(fpf_feeder *f, int slot, size_t bytes, bool host = false);
// FPF_ERR_EXCHANGE (with the message) if the feeder's paired-kernel fault word is
// set, clearing it; FPF_OK otherwise (fpf_api.cpp)
int take_exchange_fault(fpf_feeder *f);
// fpf_solve_batch in an explicit batch layout (internal callers build their own
// batches in FPF_LAYOUT_SCEN_FASTEST whatever the feeder's fpf_opts.layout)
int solve_batch_host(fpf_feeder *f, int n_scen, const double *pq, const fpf_outputs *out, fpf_aggregate *agg,
                     int layout);
// fpf_vvc.cpp: the step-size search; lazy > 1 solves the first `lazy` candidates
// and the rest only if the stop rule has not fired (fpf_vvc_round)
int vvc_line_search(fpf_feeder *feeder, const double *ctrl_dl, int nl, int ncols, const double *g,
                    const double *load_nodes, const int *n_loads, int ld, double c0, double alpha, int m_max,
                    double ploss_orig, fpf_line_search *res, int lazy);
// launchers (fpf_generic.hip, fpf_tiled.hip, fpf_rtc.cpp)
hipError_t launch_generic(const FeederDev &f, int n_scen, const double *pq, double *scratch,
                          size_t ld, const OutDev &o, hipStream_t st);
hipError_t launch_tiled(const FeederDev &f, int n_scen, const double *pq, const OutDev &o, hipStream_t st);
hipError_t launch_fixup(const FeederDev &f, int n_scen, const double *pq, double *scratch, size_t ld, const OutDev &o,
                        hipStream_t st);
size_t fixup_scratch_ld();
hipError_t launch_aggregate(int n_scen, const int8_t *status, const double *loss,
                            const double *vmin, const double *vmax, double lb_v, double ub_v,
                            double *d_agg, double *partials, unsigned *ticket, hipStream_t st);
hipError_t launch_wave(const WaveDev &w, int n_scen, const double *pq, const OutDev &o, hipStream_t st);
hipError_t launch_lane(const LaneDev &l, int n_scen, const double *pq, const OutDev &o, hipStream_t st);
// the lane kernel's dynamic LDS: with the loads' DMA rings (dma) or without (the
// plan's check and the guard's local re-solve use the smaller, dma = false)
size_t lane_lds_bytes(const LaneDev &l, bool dma = false);
int lane_min_scen();   // launches from this size run the lane kernel (FPF_LANE: 0 never, 1 always, n)
// the staging tables of a wave-kernel geometry (WaveDev::stage_smaj / stage_l0,
// [u][NT] int2 each); returns the chunks per thread, 0 if above the kernel's limit
int wave_stage_tables(const WaveDev &w, std::vector<int32_t> &smaj, std::vector<int32_t> &l0);
// the write-out tables (WaveDev::out_smaj / out_l0, [u][NT] int); 0 if above the limit
int wave_out_tables(const WaveDev &w, std::vector<int32_t> &smaj, std::vector<int32_t> &l0);
// per-wave IO units (WaveDev::stage_uw / out_uw) of a geometry whose tables exist
// (stage_u / out_u set); 0 where a wave's share exceeds the kernel's limit
void wave_io_units(WaveDev &w);
size_t wave_lds_bytes(const WaveDev &w);
hipError_t launch_transpose(const double *in, double *out, size_t rows, size_t cols, hipStream_t st);
hipError_t launch_wblk(const WaveDev &w, int n_scen, const double *pq, const OutDev &o, hipStream_t st);
size_t wblk_lds_bytes(const WaveDev &w);
hipError_t launch_wcoop(const WaveDev &w, int n_scen, const double *pq, const OutDev &o, hipStream_t st);
size_t wcoop_lds_bytes(const WaveDev &w);
// whether an area solve of n scenarios runs the plain wave kernel (hooks apply)
bool wave_hooks_supported(fpf_feeder *f, int n_scen);
constexpr int COOP_NSLOT = 1024;   // exchange areas of the paired kernel (scenarios in flight <= 256)
inline size_t wave_any_lds_bytes(const WaveDev &w) {
    return w.coop ? wcoop_lds_bytes(w) : (w.wps ? wblk_lds_bytes(w) : wave_lds_bytes(w));
}
bool wblk_geometry(int n, int *wps, int *c);
bool wave_geometry(int n, int *spw, int *c);
int wave_scenarios_per_block(const WaveDev &w);
bool wave_wpb_supported(int spw, int c, int wpb);
size_t tiled_lds_bytes(const FeederDev &f, int tile);
size_t tiled_lds_bytes_rtc(const FeederDev &f, int tile);
int tiled_max_tile(const FeederDev &f);
int tiled_threads(const FeederDev &f, int tile);

// Multi-track schedule of the sequential stages (fpf_api.cpp: schedule_tracks).
// The feeder's blocks (Dl row runs between separator rows) are list-scheduled
// onto T tracks; each block occupies consecutive steps of one track.  Forward
// runs steps 0..S-1, backward the same cells in reverse, so a cell's LDS slot
// serves both.  Node k scheduled at (step s, track t) lives in slot
// base[s] + t (pack_slots): every track finds its cell of step s at the same
// offset from its own base, and the combs of different steps interleave.
// Slots 0..T-1 hold V0; T more pad the end.
struct TrackSched {
    int T = 1, S = 0, n_slots = 0;
    std::vector<int> cell;                 // [S*T] node or -1
    std::vector<int> step, track;          // [nn] of each node (node 0: -1)
    std::vector<int> base;                 // [S] slot of track 0's cell at step s
    std::vector<unsigned> active;          // [S] bit t: track t has a node at step s
    std::vector<int> slot_of;              // [nn] state slot of each node (node 0: 0)
    std::vector<int> fw_src;               // [nn] forward source node (0 = V0)
    std::vector<int> fw_mask;              // [nn] phase-zeroing bits
    std::vector<std::vector<int>> children;// [nn] first nodes of the child blocks, in accumulation order
    std::vector<char> bw_reset;            // [nn] Ibl = 0 before this node's backward op
    int slot(int k) const { return k == 0 ? 0 : slot_of[k]; }
};

// topology-specialised tiled kernel (fpf_rtc.cpp)
struct RtcSpec {
    int tile, nn, n_taps, nt;
    int maxt = 1;                         // tasks per lane
    int min_waves = 4;                    // __launch_bounds__ minimum waves per SIMD
    int ahead = 2;                        // LDS operand lookahead of the sequential stages (steps; more costs registers)
    int ns = 21;                          // scenarios per sequential wave (3*T*ns <= 64)
    int ps = 0, slot = 0;                 // phase / slot strides of the state layout (16-byte units)
    bool keep_ib = true;                  // keep the last sweep's Ib for the PQb output
    bool exact = false;                   // fpf_opts.exact: the reference's roundings
    bool full_k = false;                  // every Lnum_p + 1 == nn: V_abc_list keeps all rows
    bool temp_lds = true;                 // stage the TEMP blocks in LDS (else read from global)
    long stagger = 0;                     // diagnostic (FPF_RTC_STAGGER=cycles,shift)
    int stagger_shift = 8;
    TrackSched ts;
};
struct RtcKernel {
    hipModule_t mod;
    hipFunction_t fn;
    int nt;
};
std::string rtc_source(const RtcSpec &spec);
int rtc_build(int device, const RtcSpec &spec, RtcKernel *out, std::string *err);
void rtc_release(const RtcKernel &k);   // drop one reference; the last unloads the code object
hipError_t rtc_launch(const RtcKernel &k, const FeederDev &f, int n_scen, const double *pq, const OutDev &o,
                      hipStream_t st);
// the wave kernel (w.wps: the wave-block kernel) compiled for one plan (its
// uniform values as constants, fpf_wave_body.h / fpf_wblk_body.h: FPF_WSPEC) and
// variant; built on first use, kept for the
// process.  NULL if the build failed (the static kernel runs)
hipFunction_t wave_rtc_function(int device, const WaveDev &w, bool full);
hipFunction_t wave_rtc_function_src(int device, const WaveDev &w, bool full);   // (uncached by plan)
// the smallest launch that runs it (FPF_WAVE_RTC: 0 never, 1 always, n; default 2048)
int wave_rtc_min();
std::string wave_rtc_source(const WaveDev &w, bool full, std::string *name);
#endif

}  // namespace fpf
