// fpf_api.cpp -- host side of libfreedm_pf (C ABI declared in include/freedm_pf.h).
//
// Feeder creation turns the reference's Dl/Z arguments into device tables once:
//   * the index checks Armadillo would perform inside DPF_return7 (any
//     violation = the reference throws => FPF_ERR_TOPOLOGY),
//   * the sweep as op lists (load-current, backward, forward) for the generic
//     kernel, with the feeder-static ZGEMM TEMP = lng * Z/Zb per forward op,
//   * for well-formed feeders, the per-node tables and sequential-stage programs
//     of the tiled kernel,
//   * Lnum_a/b/c of form_Y_abc for the Vmin/Vmax reduction.
// Solves only launch kernels; nothing is computed on the host per scenario.
#include "../../include/freedm_pf.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <cstdlib>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "fpf_internal.h"
#include "fpf_math.hpp"

#pragma clang fp contract(off)

using namespace fpf;

struct fpf_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
};

struct fpf_feeder {
    fpf_ctx *ctx = nullptr;
    fpf_opts opts{};
    fpf_feeder_info info{};
    FeederDev dev{};
    void *d_tables = nullptr;
    // generic-kernel scratch
    double *d_scratch = nullptr;
    size_t scratch_ld = 0;
    // per-scenario internal outputs (used when the caller passes NULL)
    int cap = 0;
    int32_t *d_iters = nullptr;
    int8_t *d_status = nullptr;
    double *d_loss = nullptr, *d_vmin = nullptr, *d_vmax = nullptr;
    // host-API staging
    size_t stage_bytes = 0;
    void *d_stage = nullptr;
    double *d_agg = nullptr;
    // fused aggregate of the specialised kernel: per-tile partials + arrival ticket
    double *d_partials = nullptr;
    size_t partials_cap = 0;      // tiles
    unsigned *d_ticket = nullptr;
    // topology-specialised tiled kernel (hipRTC), if built
    bool rtc = false;
    RtcKernel rtc_kernel{};      // without the PQb output (no Ib kept in registers)
    RtcKernel rtc_kernel_ib{};   // with PQb: built on the first solve that asks for it
    bool rtc_ib = false;
    RtcSpec rtc_spec;
    // wave kernel (fast mode); wdev_big: the same tables launched with the
    // waves per workgroup of large batches
    void *d_wave = nullptr;
    void *d_stage_tab = nullptr;   // the wave kernel's staging tables (both geometries)
    WaveDev wdev{}, wdev_big{};
    // the lane kernel (fpf_lane.hip): one lane per scenario; large light-output
    // scenario-fastest batches of the feeders it accepts (analyse_lane)
    void *d_lane = nullptr;
    LaneDev ldev{};
    bool lane_ok = false;
    void *d_xch = nullptr, *d_xsync = nullptr, *d_xvm = nullptr;   // the paired wave-block kernel's exchange
    unsigned *h_xerr = nullptr;   // its sticky fault word (pinned, coherent; the kernel sets it at system scope)
    // the partials + ticket scratch is shared by every aggregating launch on
    // this feeder (fused wave/specialised aggregate, fpf_aggregate_device): a
    // launch on another stream than the previous one first waits for it
    hipEvent_t agg_event = nullptr;
    hipStream_t agg_stream = nullptr;
    bool agg_pending = false;
    // scenario-major batches on the generic / tiled kernels: layout-0 copies of
    // pq and the matrix outputs, transposed around the launch (fpf_layout.hip)
    double *d_lay = nullptr;
    size_t lay_bytes = 0;
    // host-API results: pinned staging, one device-to-host copy for small outputs
    void *h_stage = nullptr;
    size_t h_stage_bytes = 0;
    // auto choice between the interpreted tiled and the generic kernel, made
    // per batch (both table sets are built): tiled below AUTO_GENERIC_MIN_SCEN
    bool auto_batch = false;
    // convergence guard of the fast kernels (fpf_opts.no_guard = 0): the scenarios
    // flagged in the guard band [flag_cap] and their count (0 between solves: the
    // fixup kernel resets it), and the fixup kernel's scratch (fixup_scratch_ld columns)
    bool guard = false;
    unsigned *d_flag_count = nullptr;
    int32_t *d_flag_ids = nullptr;
    int flag_cap = 0;
    double *d_fix_scratch = nullptr;
    // the guard's local mode inside the wave kernel (solves without an aggregate):
    // the exact op lists as a device-side FeederDev
    FeederDev *d_fixdev = nullptr;
    // the VVC batch paths' cached scratch (fpf::feeder_buf): [slot] = (pointer, bytes)
    std::vector<std::pair<void *, size_t>> bufs_dev, bufs_host;
};

// The guard band of the fast kernels' convergence test (fpf_opts.no_guard).
// Ib(0) is a sum of the Nb load currents; the reference adds them in row order
// (a recursive sum, rounding error <= (Nb - 1) u sum |IL|, u = 2^-53), the fast
// kernels as a lane-local prefix plus a DPP scan (height <= 16: <= 16 u sum |IL|),
// and their IL differ by a few u (one refined reciprocal vs __divdc3, <= 8 u
// |IL|).  errmx compares this sweep's Ib(0) with the last one's, so its two
// evaluations differ by at most about 2 (Nb + 24) u sum_k |IL_k|_1 (the iterates'
// own differences, ~Nb u |V0 - V|, are smaller still); the band is twice that.
static double guard_factor(int nb) { return 4.0 * (nb + 24) * 0x1p-53; }

static int fail(fpf_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
}
int fpf::feeder_fail(fpf_feeder *f, int code, const std::string &msg) { return fail(f ? f->ctx : nullptr, code, msg); }

void *fpf::feeder_buf(fpf_feeder *f, int slot, size_t bytes, bool host) {
    if (!f || slot < 0) return nullptr;
    auto &v = host ? f->bufs_host : f->bufs_dev;
    if ((size_t)slot >= v.size()) v.resize((size_t)slot + 1, {nullptr, 0});
    auto &b = v[(size_t)slot];
    bytes = std::max<size_t>(bytes, 256);
    if (b.first && b.second >= bytes) return b.first;
    if (b.first) (void)(host ? hipHostFree(b.first) : hipFree(b.first));
    b = {nullptr, 0};
    // (a little headroom: the next batch of a study is often slightly larger)
    const size_t want = bytes + bytes / 8;
    const hipError_t e = host ? hipHostMalloc(&b.first, want) : hipMalloc(&b.first, want);
    if (e != hipSuccess) {
        b = {nullptr, 0};
        fail(f->ctx, FPF_ERR_HIP, std::string("scratch allocation: ") + hipGetErrorString(e));
        return nullptr;
    }
    b.second = want;
    return b.first;
}

#define HIPCHK(ctx, expr)                                                                      \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess)                                                                  \
            return fail(ctx, FPF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_));   \
    } while (0)

extern "C" int fpf_abi_version(void) { return FPF_ABI_VERSION; }

extern "C" void fpf_opts_default(fpf_opts *o) {
    if (!o) return;
    std::memset(o, 0, sizeof(*o));
    o->bkva = 1000;             // DPF_return7.cpp:11
    o->bkv = 12.47;             // :12
    o->vo_kv = 12.47 * 1.015;   // :13
    o->eps = 0.0001;            // :14
    o->mxitr = 20;              // :15
    o->kernel = FPF_KERNEL_AUTO;
    o->lb_v = 0.96;             // load_system_data.cpp:23
    o->ub_v = 1.05;             // load_system_data.cpp:24
    o->tile = 0;
    o->specialize = 1;
    o->exact = 0;
}

extern "C" int fpf_ctx_create(int device, fpf_ctx **out) {
    if (!out) return FPF_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return FPF_ERR_HIP;
    if (device < 0 || device >= n) return FPF_ERR_ARG;
    fpf_ctx *c = new fpf_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return FPF_ERR_HIP;
    }
    *out = c;
    return FPF_OK;
}

extern "C" void fpf_ctx_destroy(fpf_ctx *c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" const char *fpf_last_error(const fpf_ctx *c) { return c ? c->err.c_str() : "null context"; }

int fpf::ctx_device(const fpf_ctx *c) { return c ? c->device : 0; }

// ---------------------------------------------------------------------------- feeder analysis

namespace {

struct HostFeeder {
    int nl = 0, ncols = 0, nn = 0, nb = 0, ncode = 1, n_sep = 0;
    std::vector<double> dl;       // column-major copy
    std::vector<cx> zl;           // [ncode][3][3] Z/Zb
    std::vector<int32_t> zmask;   // per code
    std::vector<IlOp> il;
    std::vector<BwOp> bw;
    std::vector<FwOp> fw;
    std::vector<double> tz;       // [n_fw][9] interleaved
    int lnum[3] = {0, 0, 0};
    // tiled
    bool wf = false;
    std::string wf_why;
    std::vector<NodeOp> node;
    struct BwIdx { int k, a, p; };            // node, tap read (-1 none), separator target (-1 none)
    struct FwIdx { int dst, src, mask; };
    std::vector<BwIdx> bwi;
    std::vector<FwIdx> fwi;
    std::vector<SeqBw> seq_bw;
    std::vector<SeqFw> seq_fw;
    int n_taps = 0, depth = 0;
    TrackSched ts;                 // multi-track schedule of the specialised kernel
    std::vector<NodeOp> node_rtc;  // node table with the schedule's slots
    double at(int i, int j) const { return dl[(size_t)i + (size_t)j * nl]; }
};

bool to_int(double x, int *v) {
    if (!(std::fabs(x) < 2147483647.0)) return false;
    *v = (int)x;
    return true;
}
bool to_uword(double x, int bound, int *v) {
    if (!(x > -1.0) || !(x < (double)bound)) return false;
    *v = (int)x;
    return true;
}

// Index checks equivalent to the Armadillo bounds checks of DPF_return7; fills op lists.
std::string build_ops(HostFeeder &h, const double *z, int z_rows, int z_cols, const fpf_opts &o) {
    const int nl = h.nl;
    int cnt = 0;
    for (int i = 0; i < nl; ++i) {
        int v;
        if (!to_int(h.at(i, 0), &v)) return "Dl(:,0) not finite";
        if (v != 0) cnt++;
        if (h.at(i, 0) == 0) h.n_sep++;
        else h.nb++;
    }
    h.nn = cnt + 1;   // DPF_return7.cpp:37
    const int nn = h.nn;
    if (z_rows >= 3 && z_cols < 3) return "Z needs 3 columns";
    const int rz = z_rows / 3;
    h.ncode = rz > 0 ? rz : 1;
    // Zl = Z / Zb per code (DPF_return7.cpp:64-80); zeros(3,3) if Z has < 3 rows
    const double Zb = 1000 * std::pow(o.bkv, 2) / o.bkva;
    h.zl.assign((size_t)h.ncode * 9, mk(0, 0));
    for (int i = 0; i < rz; ++i)
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                size_t zi = (size_t)(3 * i + r) + (size_t)c * z_rows;
                h.zl[(size_t)i * 9 + r * 3 + c] = cdiv(mk(z[2 * zi], z[2 * zi + 1]), mk(Zb, 0.0));
            }
    h.zmask.assign(h.ncode, 0);
    for (int i = 0; i < h.ncode; ++i)
        for (int p = 0; p < 3; ++p) {
            cx d = h.zl[(size_t)i * 9 + p * 3 + p];
            if (d.re == 0 && d.im == 0) h.zmask[i] |= 1 << p;   // abs(Ztemp(p,p)) == 0 :180-192
        }
    if (nn - 1 < 1) return "no branches";
    // load currents :107-130
    for (int j = 0; j < nl; ++j)
        if (h.at(j, 0) > 0) {
            int ndr;
            if (!to_int(h.at(j, 2), &ndr) || ndr < 0 || ndr >= nl || ndr - 1 < 0 || ndr - 1 >= nn)
                return "row " + std::to_string(j) + ": rbus out of range (V / IL index)";
            h.il.push_back({j, ndr});
        }
    // backward sweep :136-160
    for (int m = nl - 1; m >= 0; --m) {
        if (h.at(m, 0) == 0) {
            int node;
            if (m + 1 >= nl) return "trailing separator row (sbus(m+1) out of range)";
            if (!to_int(h.at(m + 1, 1), &node) || node - 1 < 0 || node - 1 >= nn - 1)
                return "separator row " + std::to_string(m) + ": tap sbus(m+1) out of range";
            h.bw.push_back({1, node - 1});
        } else {
            int ndr;
            if (!to_int(h.at(m, 2), &ndr) || ndr - 1 < 0 || ndr - 1 >= nn - 1)
                return "row " + std::to_string(m) + ": rbus out of range (Ib index)";
            h.bw.push_back({0, ndr - 1});
        }
    }
    // forward sweep :163-195
    auto add_fw = [&](int m, int dst, int src, int ib, int lcd, int mask) {
        FwOp op{dst, src, ib, lcd - 1, mask, 0};
        h.fw.push_back(op);
        const double lng = h.at(m, 4);
        for (int L = 0; L < 3; ++L)
            for (int a = 0; a < 3; ++a) {
                cx t = zgemm_temp(lng, h.zl[(size_t)(lcd - 1) * 9 + L * 3 + a]);
                h.tz.push_back(t.re);
                h.tz.push_back(t.im);
            }
    };
    {
        int lcd1;
        if (!to_int(h.at(0, 3), &lcd1) || lcd1 < 1 || lcd1 > h.ncode) return "row 0: line code out of range";
        if (nl < 2) return "Dl needs at least 2 rows";
        if (!std::isfinite(h.at(0, 4))) return "row 0: length not finite";
        add_fw(0, 1, -1, 0, lcd1, 0);   // V(1) = V0 - lng(0)*Ib.row(0)*Ztemp, no zeroing
    }
    for (int m = 1; m < nl; ++m) {
        if (h.at(m, 0) != 0) {
            int lcd, src, ib, dst;
            if (!to_int(h.at(m, 3), &lcd) || lcd < 1 || lcd > h.ncode)
                return "row " + std::to_string(m) + ": line code out of range";
            if (!to_uword(h.at(m, 1), nl, &src)) return "row " + std::to_string(m) + ": sbus out of range";
            if (!to_uword(h.at(m, 2) - 1, nn - 1, &ib)) return "row " + std::to_string(m) + ": rbus-1 out of range";
            if (!to_uword(h.at(m, 2), nl, &dst)) return "row " + std::to_string(m) + ": rbus out of range";
            if (!std::isfinite(h.at(m, 4))) return "row " + std::to_string(m) + ": length not finite";
            add_fw(m, dst, src, ib, lcd, h.zmask[lcd - 1]);
        }
    }
    if (nl < nn) return "Dl has fewer rows than nodes (V_nodes index)";
    return "";
}

// Lnum_a/b/c of form_Y_abc (form_Yabc.cpp:11-58)
std::string build_lnum(HostFeeder &h, const double *z, int z_rows, const fpf_opts &o) {
    const double Zb = std::pow(o.bkv, 2) / o.bkva * 1000;
    int lbr = 0;
    for (int i = 0; i < h.nl; ++i)
        if (h.at(i, 0) > 0) lbr++;
    std::vector<cx> brn((size_t)std::max(lbr, 1) * 3, mk(0, 0));
    int j = 0;
    for (int i = 0; i < h.nl && j < lbr; ++i) {
        const int code = (int)h.at(i, 3);
        const int idx = 3 * (code - 1);
        if ((int)h.at(i, 0) != 0) {
            if (idx < 0 || idx + 2 >= z_rows) return "form_Y_abc: line code out of range";
            for (int p = 0; p < 3; ++p) {
                size_t zi = (size_t)(idx + p) + (size_t)p * z_rows;
                cx zz = mk(z[2 * zi], z[2 * zi + 1]);
                if (code == 7) {
                    brn[(size_t)j * 3 + p] = zz;
                } else {
                    const double lng = h.at(i, 4);
                    cx t = mk(zz.re * lng, zz.im * lng);
                    brn[(size_t)j * 3 + p] = mk(t.re / Zb, t.im / Zb);
                }
            }
            ++j;
        }
    }
    for (int p = 0; p < 3; ++p) {
        int c = 0;
        for (int i = 0; i < lbr; ++i)
            if (std::hypot(brn[(size_t)i * 3 + p].re, brn[(size_t)i * 3 + p].im) > 0) c++;
        h.lnum[p] = c;
    }
    return "";
}

// Well-formedness for the tiled kernel (DESIGN.md "Tiled kernel"): the op lists
// can then run in per-node tasks with every Ib/IL/V slot living at node index.
void analyse_tiled(HostFeeder &h) {
    const int nl = h.nl, nn = h.nn;
    auto no = [&](const std::string &why) { h.wf = false; h.wf_why = why; };
    h.node.assign(nn, NodeOp{-1, -1, -1, 0, -1, 0, {0, 0}});
    for (int k = 0; k < nn; ++k) h.node[k].slot = k;   // interpreted layout: slot k = node k
    if (nn > 8192) return no("more than 8192 nodes");
    std::vector<int> row_of(nn, -1);
    std::vector<int> seen(nn, 0);
    seen[0] = 1;
    int fwi = 0;
    for (int m = 0; m < nl; ++m) {
        const double ln = h.at(m, 0);
        if (ln == 0) continue;
        if (!(ln >= 1) || ln != std::floor(ln)) return no("branch number not a positive integer");
        const double rb = h.at(m, 2), sb = h.at(m, 1);
        if (rb != std::floor(rb) || sb != std::floor(sb)) return no("fractional bus number");
        const int k = (int)rb, src = (int)sb;
        if (k < 1 || k >= nn) return no("rbus outside 1..nn-1");
        if (row_of[k] >= 0) return no("duplicate rbus");
        if (m == 0 && (k != 1 || src != 0)) return no("row 0 is not branch 0 -> 1");
        if (src < 0 || src >= nn || !seen[src]) return no("sbus not fed by an earlier row");
        row_of[k] = m;
        seen[k] = 1;
        NodeOp &nd = h.node[k];
        nd.fw = fwi;
        nd.row = m;
        nd.code = h.fw[fwi].code;
        nd.mask = h.fw[fwi].mask;
        nd.tap = -1;
        ++fwi;
    }
    for (int k = 1; k < nn; ++k)
        if (row_of[k] < 0) return no("node without a branch row");
    // taps: distinct separator targets
    std::vector<int> tap_of(nn, -1);
    h.n_taps = 0;
    for (int m = 0; m < nl; ++m)
        if (h.at(m, 0) == 0) {
            const int t = (int)h.at(m + 1, 1);
            if (tap_of[t] < 0) tap_of[t] = h.n_taps++;
            h.node[t].tap = tap_of[t];
        }
    if (h.n_taps > 32766) return no("too many taps");
    // sequential programs in index form: a separator row folds into the branch
    // op processed just before it (row m+1, DPF_return7.cpp:138-146)
    h.bwi.clear();
    h.fwi.clear();
    for (int m = nl - 1; m >= 0; --m) {
        if (h.at(m, 0) == 0) {
            h.bwi.back().p = tap_of[(int)h.at(m + 1, 1)];
        } else {
            const int k = (int)h.at(m, 2);
            h.bwi.push_back({k, tap_of[k], -1});
        }
    }
    for (const FwOp &op : h.fw) h.fwi.push_back({op.dst, op.src < 0 ? 0 : op.src, op.mask});
    // depth of the node tree (longest chain) for the info record
    std::vector<int> dep(nn, 0);
    int d = 0;
    for (const FwOp &op : h.fw) {
        dep[op.dst] = (op.src < 0 ? 0 : dep[op.src]) + 1;
        d = std::max(d, dep[op.dst]);
    }
    h.depth = d;
    h.wf = true;
}

// Tables of the wave kernel (fpf_wave.hip).  Accepts well-formed feeders of at
// most 256 branches whose backward chains are the feeder tree: a branch row
// that follows another branch row starts at that row's receiving bus, so the
// Ib the backward sweep hands up a block (DPF_return7.cpp:147-157) flows to the
// node's forward source (:176-178) -- the sweep then computes subtree sums.
constexpr size_t WAVE_LDS_BUDGET = 159 * 1024;   // 160 KiB per CU minus the kernel's static LDS
// batches from here on use WaveHost::wpb_big_batch (and, fpf_rtc.cpp, the per-plan
// build): config 2's 4 096-scenario batch on 4-wave workgroups with the per-plan
// build 37.3 us against 38.9-39.2 on one 8-wave workgroup per CU, static (profiles/r05wio)
constexpr int WAVE_SMALL_WPB_MIN_SCEN = 4096;
// ... but only for the geometries whose small workgroups keep the registers of
// the large ones (fpf_wave_body.h: WaveGeom::eff_minw): with C = 4 both run 2 waves
// per SIMD at 256 VGPRs; the C <= 2 geometries' 4-wave workgroups would be launched
// for 3 waves per SIMD at 168 VGPRs and spill (config 5's 36-bus area, <2,2,4>:
// 37-41 us a launch against 22-27 us on 8-wave workgroups, profiles/r06s2_c5)
static bool wave_small_wpb_regs_ok(int spw, int C) { return spw * C > 2 && C > 2; }

struct WaveHost {
    bool ok = false;
    std::string why;
    int n = 0, spw = 0, C = 0, nblk = 0, bdepth = 0, ncomp = 0, has_rel = 0, has_mask = 0, wpb = 0, off_in_x = 0;
    int temp_sym = 0;
    int wpb_big_batch = 0;
    int wps = 0;                     // wave-block kernel: wavefronts per scenario (0: per-wavefront kernel)
    int coop = 0, nb_c = 0, nf_c = 0, nb_split = 0, nf_split = 0;   // paired wave-block kernel (fpf_wcoop.hip)
    std::vector<int32_t> row, node, info, blk, mref, pairs, info2;
    std::vector<double> temp;
    std::vector<double> lng, code_z;   // wave-block kernel: per slot lng, per code Zl (fpf_internal.h)
    std::vector<int32_t> code;
    // the sequential-order plan (analyse_wave_lag): tables the tree plan declines
    int has_lag = 0, nlag = 0;
    std::vector<int32_t> lagx;    // [C][L] extra backward pair hi | lo << 9 | (V_prev store index + 1) << 18
    std::vector<int32_t> bbase;   // [nblk] base of a block's chain: -1 V0, else the V_prev entry
};

// The tables of the paired wave-block kernel (fpf_wcoop.hip, 2049..4096
// branches): the positions [0, P) of the depth-first order on workgroup 0, [P, n)
// on workgroup 1 (P = ceil(n / 2)), C slots per lane of 512; the gathered
// positions numbered in position order so that each workgroup owns one range of
// the backward and of the forward index space.
static void analyse_coop(const HostFeeder &h, WaveHost &w, int n, int C, int wps, int nblk, int maxd, int has_mask,
                         const std::vector<int> &par, const std::vector<int> &at, const std::vector<int> &pos,
                         const std::vector<int> &blk, const std::vector<int> &size, const std::vector<int> &bfirst) {
    auto no = [&](const std::string &why) { w.ok = false; w.why = why; };
    const int L = 64 * wps, P = (n + 1) / 2;
    if (P > C * L || n - P > C * L) return no("paired wave-block kernel: more than 2 x 2048 positions");
    if (nblk > L || maxd > 6) return no("paired wave-block kernel: block chains beyond the register-resolved form");
    // the kernel packs block (9 bits), forward index + 1 (14 bits) and line code (9
    // bits) into one register per slot (fpf_wcoop.hip sx)
    if (h.ncode > 512) return no("paired wave-block kernel: more than 512 line codes");
    std::vector<char> isb(n, 0), isf(n, 0);
    for (int q = 0; q < n; ++q) isb[q + size[at[q]] - 1] = 1;
    for (int b = 1; b < nblk; ++b) {
        isf[pos[par[bfirst[b]]]] = 1;
        isf[pos[bfirst[b]] - 1] = 1;
    }
    std::vector<int> cb(n, -1), cf(n, -1);
    int nb = 0, nf = 0, nbs = 0, nfs = 0;
    for (int q = 0; q < n; ++q) {
        if (q == P) {
            nbs = nb;
            nfs = nf;
        }
        if (isb[q]) cb[q] = nb++;
        if (isf[q]) cf[q] = nf++;
    }
    const int ncomp = std::max(nb, nf);
    if (ncomp > 16000) return no("paired wave-block kernel: too many gathered positions");
    int bdepth = 0;
    std::vector<std::vector<std::pair<int, int>>> chainp(nblk);
    for (int b = 1; b < nblk; ++b) {
        for (int j = b; j != 0; j = blk[par[bfirst[j]]]) chainp[b].push_back({cf[pos[par[bfirst[j]]]], cf[pos[bfirst[j]] - 1]});
        bdepth = std::max(bdepth, (int)chainp[b].size());
    }
    w.pairs.assign((size_t)std::max(bdepth, 1) * 2 * nblk, ncomp);
    for (int b = 1; b < nblk; ++b)
        for (size_t j = 0; j < chainp[b].size(); ++j) {
            w.pairs[(2 * j) * nblk + b] = chainp[b][j].first;
            w.pairs[(2 * j + 1) * nblk + b] = chainp[b][j].second;
        }
    const size_t S = (size_t)2 * C * L;
    w.row.assign(S, -1);
    w.node.assign(S, -1);
    w.info.assign(S, (int32_t)((uint32_t)ncomp << 18));   // empty slot: gathers the zero entry, stores nothing
    w.info2.assign(S, 0);
    w.blk.assign(S, 0);
    w.lng.assign(S, 0.0);
    w.code.assign(S, 0);
    bool zsym = !getenv("FPF_WAVE_NO_SYM");
    for (int q = 0; q < n; ++q) {
        const int k = at[q], g = q >= P, ql = q - g * P, i = (g * C + ql % C) * L + ql / C;
        const NodeOp &nd = h.node[k];
        w.row[i] = nd.row;
        w.node[i] = k;
        w.info[i] = (int32_t)((uint32_t)(nd.mask & 7) | 8u | ((uint32_t)(cb[q] + 1) << 4) | ((uint32_t)cb[q + size[k] - 1] << 18));
        w.info2[i] = cf[q] + 1;
        w.blk[i] = blk[k];
        w.lng[i] = h.at(nd.row, 4);
        w.code[i] = nd.code;
        const cx *z = &h.zl[(size_t)nd.code * 9];
        for (int j = 1; j < 9 && zsym; ++j)
            if (j % 4 != 0) zsym = z[j].re == z[1].re && z[j].im == z[1].im;
    }
    const int ntz = zsym ? 4 : 9;
    w.code_z.assign((size_t)h.ncode * ntz * 2, 0.0);
    for (int cd = 0; cd < h.ncode; ++cd) {
        const cx *z = &h.zl[(size_t)cd * 9];
        for (int j = 0; j < ntz; ++j) {
            const cx v = !zsym ? z[j] : (j < 3 ? csub(z[4 * j], z[1]) : z[1]);
            w.code_z[((size_t)cd * ntz + j) * 2] = v.re;
            w.code_z[((size_t)cd * ntz + j) * 2 + 1] = v.im;
        }
    }
    w.temp_sym = zsym ? 1 : 0;
    w.n = n;
    w.spw = 1;
    w.C = C;
    w.nblk = nblk;
    w.bdepth = bdepth;
    w.ncomp = ncomp;
    w.has_rel = 0;
    w.has_mask = has_mask;
    w.off_in_x = 0;
    w.wps = wps;
    w.coop = 2;
    w.nb_c = nb;
    w.nf_c = nf;
    w.nb_split = nbs;
    w.nf_split = nfs;
    WaveDev probe{};
    probe.wps = wps;
    probe.coop = 2;
    probe.nl = h.nl;
    probe.nblk = nblk;
    probe.ncomp = ncomp;
    probe.temp_sym = w.temp_sym;
    probe.ncode = h.ncode;
    if (wcoop_lds_bytes(probe) > WAVE_LDS_BUDGET) return no("paired wave-block kernel: LDS budget exceeded");
    w.wpb = w.wpb_big_batch = wps;
    w.ok = true;
}

// Tables of the wave kernel for the Dl tables the tree plan above declines -- a
// lateral block listed before its tap's row, a block whose rows do not chain
// (row m + 1 not starting at row m's receiving bus), a branch fed from a node
// whose row comes later -- which the reference solves with its sequential
// semantics (DPF_return7.cpp:134-195).  Two forests over the nodes, both
// following row order:
//   * backward (:134-160): Ibl flows from row m + 1 to row m inside a block, so
//     row m's node is the P-parent of row m + 1's node; a block head hangs off its
//     tap t = sbus(head) when the separator before it is processed before t's row
//     (t's row comes earlier: Ib(t) takes the block's total and hands it up); else
//     the block's total is added to Ib(t) after t's row was processed ("post-add":
//     Ib(t) alone takes it) and the head is a P-root.  With every P-subtree a
//     contiguous range of a depth-first order, Ib(k) = Einc[last(k)] - Eexc[pos(k)]
//     plus, at a post-add target, one more such difference over its detached trees
//     (laid out one after another);
//   * forward (:163-195): V(r_m) = V(sbus_m) - drop_m with V(sbus_m) of this sweep
//     when sbus_m's row comes earlier ("new"), of the previous sweep otherwise
//     (V_prev, "old"; V0 for the substation and row 0).  The forward paths are cut
//     into F-segments, runs of consecutive positions each fed by the one before;
//     a segment's base is V at its F-parent (a block-offset chain of Ginc pairs, as
//     the tree plan's blocks) or, at an F-root, V0 or V_prev of its source -- which
//     the slot holding that source stores into LDS at the top of every sweep.
// Zeroed phases (on the wave kernel: up to 256 branches) as the tree plan's: V = 0
// and IL = 0 on them; a live phase below a zeroed F-ancestor (restarting from 0
// there) is declined; the loss takes the reference's PQb / PQL form (the kernel's
// FULL variant).
void analyse_wave_lag(const HostFeeder &h, WaveHost &w, const std::string &tree_why) {
    auto no = [&](const std::string &why) { w.ok = false; w.why = tree_why + "; sequential-order plan: " + why; };
    if (getenv("FPF_NO_WAVE_LAG")) return no("disabled (FPF_NO_WAVE_LAG)");
    const int nl = h.nl, nn = h.nn, n = nn - 1;
    int spw = 0, C = 0, wps = 0;
    if (!wave_geometry(n, &spw, &C)) {
        // one scenario per workgroup of wps wavefronts (fpf_wblk.hip, up to 2048 branches)
        if (!wblk_geometry(n, &wps, &C)) return no("more than 2048 branches");
        spw = 1;
    }
    const int L = wps ? 64 * wps : 64 / spw;
    std::vector<int> row_of(nn, -1), fw_of(nn, -1);
    {
        int fwi = 0;
        for (int m = 0; m < nl; ++m) {
            if (h.at(m, 0) == 0) continue;
            const double rb = h.at(m, 2), sb = h.at(m, 1);
            if (rb != std::floor(rb) || sb != std::floor(sb) || !(h.at(m, 0) >= 1) || h.at(m, 0) != std::floor(h.at(m, 0)))
                return no("fractional bus or branch number");
            const int k = (int)rb, src = (int)sb;
            if (k < 1 || k >= nn) return no("rbus outside 1..nn-1");
            if (row_of[k] >= 0) return no("duplicate rbus");
            if (m == 0 && k != 1) return no("row 0 is not a branch to node 1");
            if (m > 0 && (src < 0 || src >= nn)) return no("sbus outside 0..nn-1");
            row_of[k] = m;
            fw_of[k] = fwi++;
        }
        for (int k = 1; k < nn; ++k)
            if (row_of[k] < 0) return no("node without a branch row");
    }
    // zeroed phases (a line code without that phase, :180-192): V(k, p) = 0 on them
    // and IL = 0 there; the wave-block kernel's sequential-order plan declines them
    int has_mask = 0;
    for (int k = 1; k < nn; ++k)
        if (h.fw[fw_of[k]].mask & 7) has_mask = 1;
    if (has_mask && wps) return no("zeroed phases past 256 branches (the generic kernel runs them)");
    // P-forest (backward) and F-forest (forward)
    std::vector<int> ppar(nn, -1), post(nn, -1), fpar(nn, -1), fsrc(nn, 0);   // fsrc: an F-root's source (0: V0)
    std::vector<int> chain(nn, -1);
    std::vector<std::vector<int>> lat(nn), detached(nn);
    for (int m = 0; m < nl; ++m) {
        if (h.at(m, 0) == 0) continue;
        const int k = (int)h.at(m, 2);
        if (m == 0) {
            fsrc[k] = 0;   // V(1) = V0 - drop (:163-168)
        } else {
            const int sb = (int)h.at(m, 1);
            if (sb == 0) fsrc[k] = 0;                       // V(0) is never written: V0
            else if (row_of[sb] < m) fpar[k] = sb;          // this sweep's V(sbus)
            else fsrc[k] = sb;                              // the previous sweep's
            if (h.at(m - 1, 0) != 0) {
                const int pk = (int)h.at(m - 1, 2);
                ppar[k] = pk;
                chain[pk] = k;
            } else {
                const int t = sb;   // the separator at m - 1 adds into Ib(sbus(m)) (:138-146)
                if (row_of[t] < m - 1) {
                    ppar[k] = t;
                    lat[t].push_back(k);
                } else {
                    post[k] = t;
                    detached[t].push_back(k);
                }
            }
        }
    }
    // depth-first order of the P-forest: node 1's tree, then the detached trees
    // grouped by their post-add target (one range per target)
    std::vector<int> pos(nn, -1), at, size(nn, 1);
    std::vector<int> lo_t(nn, -1), hi_t(nn, -1);
    auto dfs = [&](int root) {
        std::vector<int> st = {root};
        while (!st.empty()) {
            const int k = st.back();
            st.pop_back();
            pos[k] = (int)at.size();
            at.push_back(k);
            for (int l : lat[k]) st.push_back(l);
            if (chain[k] >= 0) st.push_back(chain[k]);
        }
    };
    dfs(1);
    for (int t = 1; t < nn; ++t) {
        if (detached[t].empty()) continue;
        lo_t[t] = (int)at.size();
        for (int hd : detached[t]) dfs(hd);
        hi_t[t] = (int)at.size() - 1;
    }
    if ((int)at.size() != n) return no("the backward structure does not reach every node");
    for (int q = n - 1; q > 0; --q)
        if (ppar[at[q]] >= 1) size[ppar[at[q]]] += size[at[q]];
    // F-segments: runs of positions each fed (this sweep) by the one before
    std::vector<int> blk(n, 0), bfirst;
    for (int q = 0; q < n; ++q) {
        if (q == 0 || fpar[at[q]] != at[q - 1]) bfirst.push_back(q);
        blk[q] = (int)bfirst.size() - 1;
    }
    const int nblk = (int)bfirst.size();
    if (nblk > 511) return no("too many forward segments");
    // V_prev sources
    std::vector<int> lagid(nn, -1);
    int nlag = 0;
    for (int b = 0; b < nblk; ++b) {
        const int hd = at[bfirst[b]];
        if (fpar[hd] < 0 && fsrc[hd] > 0 && lagid[fsrc[hd]] < 0) lagid[fsrc[hd]] = nlag++;
    }
    if (nlag > (wps ? 1024 : 64)) return no("too many sources of the previous sweep");
    // gathered positions: backward = P-subtree ends; forward = F-parents of
    // segment heads and the positions before segment heads
    std::vector<int> cb(n, -1), cf(n, -1);
    int nb_c = 0, nf_c = 0;
    for (int q = 0; q < n; ++q) {
        const int e = q + size[at[q]] - 1;
        if (cb[e] < 0) cb[e] = nb_c++;
    }
    auto needf = [&](int q) { if (cf[q] < 0) cf[q] = nf_c++; };
    for (int b = 1; b < nblk; ++b) {
        const int hd = at[bfirst[b]];
        if (fpar[hd] >= 0) needf(pos[fpar[hd]]);
        needf(bfirst[b] - 1);
    }
    // a live phase below a zeroed node m on this sweep's forward path restarts from
    // 0 there: V(k, p) = Vr(k) - Vr(m), Vr = the segment base - the path sum before
    // the zeroing (the tree plan's rule on the F-forest: m the nearest zeroed
    // F-ancestor; a source of the previous sweep brings its zeroed V along)
    std::vector<std::array<int, 3>> mref(nn, {-1, -1, -1});
    int has_rel = 0;
    for (int k = 1; k < nn && has_mask; ++k)
        for (int p = 0; p < 3; ++p) {
            if ((h.fw[fw_of[k]].mask >> p) & 1) continue;
            int guard = 0;
            for (int a = fpar[k]; a >= 1 && guard <= nn; a = fpar[a], ++guard)
                if ((h.fw[fw_of[a]].mask >> p) & 1) {
                    mref[k][p] = a;
                    has_rel = 1;
                    break;
                }
        }
    // (measured: V = Vr(k) - Vr(m), a difference of two ~1 p.u. values, missed the
    // 1e-10 relative bar on the small V below the zeroed node -- 5.0e-10 on a
    // shuffled 60-bus table, tests/test_gpu_lag.py -- so these tables keep the
    // generic kernel, as the paired wave-block kernel's do)
    if (has_rel) return no("a live phase below a zeroed one (the generic kernel runs it)");
    for (int k = 1; k < nn; ++k)
        for (int p = 0; p < 3; ++p)
            if (mref[k][p] >= 1) needf(pos[mref[k][p]]);
    const bool off_in_x = false;
    const int ncomp = std::max(std::max(nb_c, nf_c), 1);
    if (ncomp > 510) return no("too many gathered positions");
    // block chains: (F-parent, head - 1) per level up to a root segment,
    // (zero, head - 1) for a root segment past position 0, and its base
    std::vector<std::vector<std::pair<int, int>>> chainp(nblk);
    std::vector<int32_t> bbase(nblk, -1);
    int bdepth = 0;
    for (int b = 1; b < nblk; ++b) {
        int cur = b, guard = 0;
        while (true) {
            const int hq = bfirst[cur], hd = at[hq];
            if (fpar[hd] >= 0) {
                chainp[b].push_back({cf[pos[fpar[hd]]], cf[hq - 1]});
                cur = blk[pos[fpar[hd]]];
            } else {
                if (hq > 0) chainp[b].push_back({ncomp, cf[hq - 1]});
                bbase[b] = fsrc[hd] > 0 ? lagid[fsrc[hd]] : -1;
                break;
            }
            if (++guard > nn) return no("forward chain does not end");
        }
        bdepth = std::max(bdepth, (int)chainp[b].size());
    }
    w.pairs.assign((size_t)std::max(bdepth, 1) * 2 * nblk, ncomp);
    for (int b = 1; b < nblk; ++b)
        for (size_t j = 0; j < chainp[b].size(); ++j) {
            w.pairs[(2 * j) * nblk + b] = chainp[b][j].first;
            w.pairs[(2 * j + 1) * nblk + b] = chainp[b][j].second;
        }
    const size_t S = (size_t)C * L;
    w.row.assign(S, -1);
    w.node.assign(S, -1);
    w.info.assign(S, (ncomp << 13));
    w.blk.assign(S, 0);
    w.mref.assign(3 * S, -1);
    w.temp.assign(9 * S * 2, 0.0);
    w.lagx.assign(S, ncomp | (ncomp << 9));
    for (int q = 0; q < n; ++q) {
        const int k = at[q], c = q % C, lane = q / C, i = c * L + lane;
        w.row[i] = row_of[k];
        w.node[i] = k;
        w.info[i] = (int32_t)((uint32_t)((h.fw[fw_of[k]].mask & 7) | 8 | ((cb[q] + 1) << 4) | (cb[q + size[k] - 1] << 13) |
                                         ((cf[q] + 1) << 22)));
        w.blk[i] = blk[q];
        for (int p = 0; p < 3; ++p)
            if (mref[k][p] >= 1) w.mref[(p * C + c) * L + lane] = cf[pos[mref[k][p]]];
        int hi = ncomp, lo = ncomp;
        if (lo_t[k] >= 0) {
            hi = cb[hi_t[k]];
            lo = cb[lo_t[k] - 1];
        }
        w.lagx[i] = hi | (lo << 9) | ((lagid[k] + 1) << 18);
        for (int j = 0; j < 9; ++j) {
            w.temp[((j * C + c) * L + lane) * 2 + 0] = h.tz[(size_t)fw_of[k] * 18 + 2 * j];
            w.temp[((j * C + c) * L + lane) * 2 + 1] = h.tz[(size_t)fw_of[k] * 18 + 2 * j + 1];
        }
    }
    bool sym = !getenv("FPF_WAVE_NO_SYM");
    for (int q = 0; q < n && sym; ++q) {
        const double *t = &h.tz[(size_t)fw_of[at[q]] * 18];
        for (int j = 1; j < 9 && sym; ++j)
            if (j % 4 != 0) sym = t[2 * j] == t[2] && t[2 * j + 1] == t[3];
    }
    if (sym) {
        std::vector<double> ts(4 * S * 2, 0.0);
        for (int q = 0; q < n; ++q) {
            const int c = q % C, lane = q / C;
            const double *t = &h.tz[(size_t)fw_of[at[q]] * 18];
            for (int a = 0; a < 3; ++a) {
                ts[((a * C + c) * L + lane) * 2 + 0] = t[2 * (4 * a)] - t[2];
                ts[((a * C + c) * L + lane) * 2 + 1] = t[2 * (4 * a) + 1] - t[3];
            }
            ts[((3 * C + c) * L + lane) * 2 + 0] = t[2];
            ts[((3 * C + c) * L + lane) * 2 + 1] = t[3];
        }
        w.temp.swap(ts);
    }
    w.temp_sym = sym ? 1 : 0;
    if (wps) {
        // TEMP = lng * Zl(code), factorised as the tree plan's wave-block tables
        w.temp.clear();
        w.lng.assign(S, 0.0);
        w.code.assign(S, 0);
        bool zsym = !getenv("FPF_WAVE_NO_SYM");
        for (int q = 0; q < n; ++q) {
            const int k = at[q], i = (q % C) * L + q / C;
            w.lng[i] = h.at(row_of[k], 4);
            w.code[i] = h.fw[fw_of[k]].code;
            const cx *z = &h.zl[(size_t)w.code[i] * 9];
            for (int j = 1; j < 9 && zsym; ++j)
                if (j % 4 != 0) zsym = z[j].re == z[1].re && z[j].im == z[1].im;
        }
        const int ntz = zsym ? 4 : 9;
        w.code_z.assign((size_t)h.ncode * ntz * 2, 0.0);
        for (int cd = 0; cd < h.ncode; ++cd) {
            const cx *z = &h.zl[(size_t)cd * 9];
            for (int j = 0; j < ntz; ++j) {
                const cx v = !zsym ? z[j] : (j < 3 ? csub(z[4 * j], z[1]) : z[1]);
                w.code_z[((size_t)cd * ntz + j) * 2] = v.re;
                w.code_z[((size_t)cd * ntz + j) * 2 + 1] = v.im;
            }
        }
        w.temp_sym = zsym ? 1 : 0;
    }
    w.bbase = bbase;
    w.n = n;
    w.spw = spw;
    w.C = C;
    w.nblk = nblk;
    w.bdepth = bdepth;
    w.ncomp = ncomp;
    w.has_rel = has_rel;
    w.has_mask = has_mask;
    w.off_in_x = off_in_x ? 1 : 0;
    w.wps = wps;
    w.has_lag = 1;
    w.nlag = nlag;
    if (wps) {
        WaveDev probe{};
        probe.wps = wps;
        probe.nl = nl;
        probe.nblk = nblk;
        probe.bdepth = bdepth;
        probe.ncomp = ncomp;
        probe.temp_sym = w.temp_sym;
        probe.ncode = h.ncode;
        probe.nlag = nlag;
        if (wblk_lds_bytes(probe) > WAVE_LDS_BUDGET) return no("wave-block kernel: the scenario's loads exceed LDS");
        w.wpb = w.wpb_big_batch = wps;
        w.ok = true;
        return;
    }
    WaveDev probe{};
    probe.spw = spw;
    probe.C = C;
    probe.nl = nl;
    probe.nblk = nblk;
    probe.bdepth = bdepth;
    probe.ncomp = ncomp;
    probe.off_in_x = 0;
    probe.temp_sym = w.temp_sym;
    probe.nlag = nlag;
    const int big = spw * C <= 2 ? 16 : 8, small = big / 2;
    auto lds_at = [&](int wpb) { probe.wpb = wpb; return wave_lds_bytes(probe); };
    int wpb = 0;
    if (lds_at(big) <= WAVE_LDS_BUDGET) wpb = big;
    else if (lds_at(small) <= WAVE_LDS_BUDGET) wpb = small;
    else return no("per-scenario LDS above the budget");
    w.wpb = wpb;
    w.wpb_big_batch = (wave_small_wpb_regs_ok(spw, C) && 2 * (lds_at(small) + 1024) <= 160 * 1024) ? small : wpb;
    w.ok = true;
}

void analyse_wave(const HostFeeder &h, WaveHost &w) {
    auto no = [&](const std::string &why) { w.ok = false; w.why = why; };
    if (!h.wf) return analyse_wave_lag(h, w, "not well formed: " + h.wf_why);
    const int nl = h.nl, nn = h.nn, n = nn - 1;
    int spw = 0, C = 0, wps = 0, coop = 0;
    if (!wave_geometry(n, &spw, &C)) {
        // one scenario per workgroup of wps wavefronts (fpf_wblk.hip); above 2048
        // branches one scenario per pair of such workgroups (fpf_wcoop.hip)
        if (!wblk_geometry(n, &wps, &C)) {
            if (n > 2 * 2048 || getenv("FPF_NO_COOP")) return no("more than 4096 branches");
            coop = 2;
            wps = 8;
            C = 4;
        }
        spw = 1;
    }
    const int L = wps ? 64 * wps : 64 / spw;
    std::vector<int> par(nn, -1), chain(nn, -1);
    std::vector<std::vector<int>> lat(nn);
    for (int m = 0; m < nl; ++m) {
        if (h.at(m, 0) == 0) continue;
        const int k = (int)h.at(m, 2), src = m == 0 ? 0 : (int)h.at(m, 1);
        par[k] = src;
        if (m == 0) continue;
        if (h.at(m - 1, 0) != 0) {
            if ((int)h.at(m - 1, 2) != src)
                return analyse_wave_lag(h, w, "row " + std::to_string(m) + ": the backward chain leaves the feeder tree");
            chain[src] = k;
        } else {
            lat[src].push_back(k);
        }
    }
    // depth-first order, in-block child first: blocks and subtrees are contiguous
    std::vector<int> pos(nn, -1), at, blk(nn, 0), size(nn, 1), bfirst;
    std::vector<int> st = {1};
    bfirst.push_back(1);
    while (!st.empty()) {
        const int k = st.back();
        st.pop_back();
        pos[k] = (int)at.size();
        at.push_back(k);
        for (int l : lat[k]) {
            blk[l] = (int)bfirst.size();
            bfirst.push_back(l);
            st.push_back(l);
        }
        if (chain[k] >= 0) {
            blk[chain[k]] = blk[k];
            st.push_back(chain[k]);
        }
    }
    if ((int)at.size() != n) return no("feeder tree does not reach every node from node 1");
    for (int q = n - 1; q > 0; --q) size[par[at[q]]] += size[at[q]];
    const int nblk = (int)bfirst.size();
    if (nblk > 511) return no("too many blocks");
    // nearest zeroed proper ancestor per (node, phase)
    std::vector<std::array<int, 3>> mref(nn, {-1, -1, -1});
    int has_rel = 0, has_mask = 0;
    for (int k = 1; k < nn; ++k) {
        if (h.node[k].mask & 7) has_mask = 1;
        for (int p = 0; p < 3; ++p) {
            if ((h.node[k].mask >> p) & 1) continue;
            for (int a = par[k]; a >= 1; a = par[a])
                if ((h.node[a].mask >> p) & 1) {
                    mref[k][p] = a;
                    has_rel = 1;
                    break;
                }
        }
    }
    // a live phase below a zeroed ancestor m restarts from 0, V(k) = A(m) - A(k): on
    // the wave-block kernel's prefix sums over up to 2048 positions that difference
    // of two ~1 p.u. values misses the 1e-10 bar on the small result (3.8e-10 on the
    // 2048-bus test feeder), so such feeders keep the generic kernel there
    if (coop && has_rel) return no("paired wave-block kernel: a live phase below a zeroed one (the generic kernel runs it)");
    // with a live phase below a zeroed ancestor m the wave-block kernel's forward
    // scan is segmented at block heads (block-local path sums, fpf_wblk.hip): V(k)
    // = A(m) - A(k) is then a difference of two small path sums (the unsegmented
    // prefix sums over up to 2048 positions lost ~6 digits there: 3.8e-10
    // relative); block offsets sum the taps' values only
    const bool seg = wps && !coop && has_rel;
    // positions whose scan values other slots gather, in two index spaces that
    // share one LDS array X (the backward values are dead before the forward
    // ones are stored): backward = subtree ends; forward = taps, the positions
    // before lateral blocks, zeroed ancestors
    std::vector<int> cb(n, -1), cf(n, -1);
    int nb_c = 0, nf_c = 0;
    for (int q = 0; q < n; ++q) {
        const int e = q + size[at[q]] - 1;
        if (cb[e] < 0) cb[e] = nb_c++;
    }
    auto needf = [&](int q) { if (cf[q] < 0) cf[q] = nf_c++; };
    for (int b = 1; b < nblk; ++b) {
        needf(pos[par[bfirst[b]]]);
        if (!seg) needf(pos[bfirst[b]] - 1);
    }
    for (int k = 1; k < nn; ++k)
        for (int p = 0; p < 3; ++p)
            if (mref[k][p] >= 1) needf(pos[mref[k][p]]);
    int maxd = 0;
    for (int b = 1; b < nblk; ++b) {
        int d = 0;
        for (int j = b; j != 0; j = blk[par[bfirst[j]]]) ++d;
        maxd = std::max(maxd, d);
    }
    // bank-aware numbering of one space: the entries one 16-lane group of a
    // gather reads (ds_read_b128 serves four such groups, MI355X_MICROARCH.md
    // LDS) get distinct 16-byte units mod 16 where a coloring allows
    static const int grp[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                   {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                   {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                   {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    auto color_space = [&](std::vector<int> &comp, int &ncomp, bool backward) {
        std::vector<std::vector<char>> adj(ncomp, std::vector<char>(ncomp, 0));
        auto clique = [&](const std::vector<int> &v) {
            for (size_t a = 0; a < v.size(); ++a)
                for (size_t b = a + 1; b < v.size(); ++b)
                    if (v[a] != v[b]) adj[v[a]][v[b]] = adj[v[b]][v[a]] = 1;
        };
        if (backward) {
            for (const auto &g : grp)
                for (int c = 0; c < C; ++c) {
                    std::vector<int> v;
                    for (int ln : g) {
                        const int q = (ln % L) * C + c;
                        if (q < n) v.push_back(comp[q + size[at[q]] - 1]);
                    }
                    clique(v);
                }
        } else {
            for (const auto &g : grp)
                for (int jd = 0; jd < maxd; ++jd)
                    for (int side = 0; side < 2; ++side) {
                        std::vector<int> v;
                        for (int ln : g) {
                            int b = ln % L, j = b, d = 0;
                            if (b == 0 || b >= nblk) continue;
                            for (; j != 0 && d < jd; j = blk[par[bfirst[j]]]) ++d;
                            if (j == 0) continue;
                            v.push_back(side ? comp[pos[bfirst[j]] - 1] : comp[pos[par[bfirst[j]]]]);
                        }
                        clique(v);
                    }
        }
        std::vector<int> order(ncomp), color(ncomp, -1), deg(ncomp, 0);
        for (int a = 0; a < ncomp; ++a) {
            order[a] = a;
            for (int b = 0; b < ncomp; ++b) deg[a] += adj[a][b];
        }
        std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return deg[a] > deg[b]; });
        std::vector<int> used(16, 0), renum(ncomp);
        for (int a : order) {
            int best = -1;
            for (int col = 0; col < 16 && best < 0; ++col) {
                bool ok = true;
                for (int b = 0; b < ncomp && ok; ++b)
                    if (adj[a][b] && color[b] == col) ok = false;
                if (ok) best = col;
            }
            if (best < 0) best = (int)(std::min_element(used.begin(), used.end()) - used.begin());
            color[a] = best;
            renum[a] = best + 16 * used[best]++;
        }
        int top = 0;
        for (int a = 0; a < ncomp; ++a) top = std::max(top, renum[a] + 1);
        if (top > ncomp + 8) return;   // the holes would cost more LDS than the conflicts: keep the dense numbering
        for (int q = 0; q < n; ++q)
            if (comp[q] >= 0) comp[q] = renum[comp[q]];
        ncomp = top;   // holes allowed
    };
    if (coop) return analyse_coop(h, w, n, C, wps, nblk, maxd, has_mask, par, at, pos, blk, size, bfirst);
    if (!wps) {   // (the bank colouring assumes one scenario within a wavefront)
        color_space(cb, nb_c, true);
        color_space(cf, nf_c, false);
    }
    // entry ncomp of X is the permanent zero; in the common case the block
    // offsets are stored over X's first nblk entries (off_in_x, fpf_wave.hip)
    const bool off_in_x = !wps && nblk <= L && maxd <= 4;   // = the kernel's register-resolved path (WAVE_BD)
    const int ncomp = std::max(std::max(nb_c, nf_c), off_in_x ? nblk : 0);
    if (ncomp > 510) return no("too many gathered positions");
    // off(b) = sum over b's block-ancestor chain of Ginc[tap] - Ginc[first - 1]
    std::vector<std::vector<std::pair<int, int>>> chainp(nblk);
    int bdepth = 0;
    for (int b = 1; b < nblk; ++b) {
        for (int j = b; j != 0; j = blk[par[bfirst[j]]])
            chainp[b].push_back({cf[pos[par[bfirst[j]]]], seg ? -1 : cf[pos[bfirst[j]] - 1]});
        bdepth = std::max(bdepth, (int)chainp[b].size());
    }
    w.pairs.assign((size_t)std::max(bdepth, 1) * 2 * nblk, ncomp);
    for (int b = 1; b < nblk; ++b)
        for (size_t j = 0; j < chainp[b].size(); ++j) {
            w.pairs[(2 * j) * nblk + b] = chainp[b][j].first;
            w.pairs[(2 * j + 1) * nblk + b] = chainp[b][j].second < 0 ? ncomp : chainp[b][j].second;
        }
    const size_t S = (size_t)C * L;
    w.row.assign(S, -1);
    w.node.assign(S, -1);
    w.info.assign(S, (ncomp << 13));   // empty slot: gathers the zero entry, stores nothing
    w.blk.assign(S, 0);                // empty slot: block 0
    w.mref.assign(3 * S, -1);
    w.temp.assign(9 * S * 2, 0.0);
    for (int q = 0; q < n; ++q) {
        const int k = at[q], c = q % C, lane = q / C, i = c * L + lane;
        const NodeOp &nd = h.node[k];
        w.row[i] = nd.row;
        w.node[i] = k;
        w.info[i] = (int32_t)((uint32_t)((nd.mask & 7) | 8 | ((cb[q] + 1) << 4) | (cb[q + size[k] - 1] << 13) |
                                         ((cf[q] + 1) << 22)) |
                              (seg && bfirst[blk[k]] == k ? 0x80000000u : 0u));   // bit 31: block head (segmented scan)
        w.blk[i] = blk[k];
        for (int p = 0; p < 3; ++p)
            if (mref[k][p] >= 1) w.mref[(p * C + c) * L + lane] = cf[pos[mref[k][p]]];
        for (int j = 0; j < 9; ++j) {
            w.temp[((j * C + c) * L + lane) * 2 + 0] = h.tz[(size_t)nd.fw * 18 + 2 * j];
            w.temp[((j * C + c) * L + lane) * 2 + 1] = h.tz[(size_t)nd.fw * 18 + 2 * j + 1];
        }
    }
    // TEMP with one common off-diagonal value per branch, [[z1 zm zm][zm z2 zm]
    // [zm zm z3]] (the transposed lines and transformers of load_system_data's
    // Z): the drop of phase a is (z_a - zm) Ib_a + zm (Ib_1 + Ib_2 + Ib_3) -- 4
    // complex per slot instead of 9 (fast mode only; a few ulp of rounding)
    bool sym = !getenv("FPF_WAVE_NO_SYM");
    for (int q = 0; q < n && sym; ++q) {
        const double *t = &h.tz[(size_t)h.node[at[q]].fw * 18];
        for (int j = 1; j < 9 && sym; ++j)
            if (j % 4 != 0) sym = t[2 * j] == t[2] && t[2 * j + 1] == t[3];   // off-diagonal j = 1, 2, 3, 5, 6, 7
    }
    if (sym) {
        std::vector<double> ts(4 * S * 2, 0.0);
        for (int q = 0; q < n; ++q) {
            const int c = q % C, lane = q / C;
            const double *t = &h.tz[(size_t)h.node[at[q]].fw * 18];
            for (int a = 0; a < 3; ++a) {
                ts[((a * C + c) * L + lane) * 2 + 0] = t[2 * (4 * a)] - t[2];
                ts[((a * C + c) * L + lane) * 2 + 1] = t[2 * (4 * a) + 1] - t[3];
            }
            ts[((3 * C + c) * L + lane) * 2 + 0] = t[2];
            ts[((3 * C + c) * L + lane) * 2 + 1] = t[3];
        }
        w.temp.swap(ts);
    }
    w.temp_sym = sym ? 1 : 0;
    if (wps) {
        // TEMP = lng * Zl(code), factorised (fpf_wblk.hip): per slot lng and code,
        // per code Zl -- sym: every code's Zl has one common off-diagonal value
        w.temp.clear();
        w.lng.assign(S, 0.0);
        w.code.assign(S, 0);
        bool zsym = !getenv("FPF_WAVE_NO_SYM");
        for (int q = 0; q < n; ++q) {
            const int k = at[q], i = (q % C) * L + q / C;
            const NodeOp &nd = h.node[k];
            w.lng[i] = h.at(nd.row, 4);
            w.code[i] = nd.code;
            const cx *z = &h.zl[(size_t)nd.code * 9];
            for (int j = 1; j < 9 && zsym; ++j)
                if (j % 4 != 0) zsym = z[j].re == z[1].re && z[j].im == z[1].im;
        }
        const int ntz = zsym ? 4 : 9;
        w.code_z.assign((size_t)h.ncode * ntz * 2, 0.0);
        for (int cd = 0; cd < h.ncode; ++cd) {
            const cx *z = &h.zl[(size_t)cd * 9];
            for (int j = 0; j < ntz; ++j) {
                const cx v = !zsym ? z[j] : (j < 3 ? csub(z[4 * j], z[1]) : z[1]);
                w.code_z[((size_t)cd * ntz + j) * 2] = v.re;
                w.code_z[((size_t)cd * ntz + j) * 2 + 1] = v.im;
            }
        }
        w.temp_sym = zsym ? 1 : 0;
    }
    w.n = n;
    w.spw = spw;
    w.C = C;
    w.nblk = nblk;
    w.bdepth = bdepth;
    w.ncomp = ncomp;
    w.has_rel = has_rel;
    w.has_mask = has_mask;
    w.off_in_x = off_in_x ? 1 : 0;
    w.wps = wps;
    if (wps) {
        WaveDev probe{};
        probe.wps = wps;
        probe.nl = nl;
        probe.nblk = nblk;
        probe.bdepth = bdepth;
        probe.ncomp = ncomp;
        probe.temp_sym = w.temp_sym;
        probe.ncode = h.ncode;
        probe.has_rel = has_rel;
        if (wblk_lds_bytes(probe) > WAVE_LDS_BUDGET) return no("wave-block kernel: the scenario's loads exceed LDS");
        w.wpb = w.wpb_big_batch = wps;
        w.ok = true;
        return;
    }
    // waves per workgroup: the smaller workgroup when two of them fit in a CU's
    // LDS (each then stages its loads and writes its V while the other sweeps;
    // the registers allow 2 waves per SIMD = 8 per CU for these geometries),
    // else the larger one if it fits, else the smaller one alone
    WaveDev probe{};
    probe.spw = spw;
    probe.C = C;
    probe.nl = nl;
    probe.nblk = nblk;
    probe.bdepth = bdepth;
    probe.ncomp = ncomp;
    probe.off_in_x = w.off_in_x;
    probe.temp_sym = w.temp_sym;
    const int big = spw * C <= 2 ? 16 : 8, small = big / 2;
    auto lds_at = [&](int wpb) { probe.wpb = wpb; return wave_lds_bytes(probe); };
    // Measured (profiles/r02a, 123-bus): two 8-scenario workgroups per CU are
    // 11 % faster on a 131 072-scenario batch (config 4), one 16-scenario
    // workgroup 6 % faster on a 4 096 batch then (config 2, static kernels); with
    // the per-plan hipRTC build of the 4-wave geometry config 2 runs 4 % faster on
    // two 8-scenario workgroups (profiles/r05wio) -- so wpb_big_batch is used from
    // WAVE_SMALL_WPB_MIN_SCEN = 4096, the per-plan build's threshold.
    int wpb = 0, wpb_big_batch = 0;
    if (lds_at(big) <= WAVE_LDS_BUDGET) wpb = big;
    else if (lds_at(small) <= WAVE_LDS_BUDGET) wpb = small;
    else return no("per-scenario LDS above the budget");
    wpb_big_batch = (wave_small_wpb_regs_ok(spw, C) && 2 * (lds_at(small) + 1024) <= 160 * 1024) ? small : wpb;
    if (const char *e = getenv("FPF_WAVE_WPB")) {   // experiments
        const int x = atoi(e);
        if (wave_wpb_supported(spw, C, x) && lds_at(x) <= WAVE_LDS_BUDGET) wpb = wpb_big_batch = x;
    }
    w.wpb = wpb;
    w.wpb_big_batch = wpb_big_batch;
    w.ok = true;
}

// Tables of the lane kernel (fpf_lane.hip): the wave kernel's depth-first
// order (in-block child first: subtrees and blocks are contiguous) dealt to
// LANE_NW waves in contiguous runs of at most ns <= LANE_NS positions, each run
// padded with dummy slots to ns.  Accepts what the wave kernel's tree plan
// accepts, minus zeroed phases and non-symmetric TEMP, up to LANE_NW * LANE_NS
// branches.
struct LaneHost {
    bool ok = false;
    std::string why;
    int n = 0, ns = 0, nE = 0, nG = 0, nblk = 0;
    std::vector<int32_t> slot;   // [LANE_NW][4][ns]
    std::vector<double> temp;   // [LANE_NW][ns][LANE_TW]
    std::vector<int32_t> blk;    // [nblk][1 + 2 LANE_BD]
};

void analyse_lane(const HostFeeder &h, const fpf_opts &o, LaneHost &L) {
    auto no = [&](const std::string &why) { L.ok = false; L.why = why; };
    if (!h.wf) return no("not well formed: " + h.wf_why);
    const int nl = h.nl, nn = h.nn, n = nn - 1;
    if (n > LANE_NW * LANE_NS) return no("more than " + std::to_string(LANE_NW * LANE_NS) + " branches");
    std::vector<int> par(nn, -1), chain(nn, -1);
    std::vector<std::vector<int>> lat(nn);
    for (int m = 0; m < nl; ++m) {
        if (h.at(m, 0) == 0) continue;
        const int k = (int)h.at(m, 2), src = m == 0 ? 0 : (int)h.at(m, 1);
        par[k] = src;
        if (m == 0) continue;
        if (h.at(m - 1, 0) != 0) {
            if ((int)h.at(m - 1, 2) != src) return no("the backward chains leave the feeder tree");
            chain[src] = k;
        } else {
            lat[src].push_back(k);
        }
    }
    for (int k = 1; k < nn; ++k)
        if (h.node[k].mask & 7) return no("zeroed phases");
    // depth-first order, in-block child first (analyse_wave)
    std::vector<int> pos(nn, -1), at, blk(nn, 0), size(nn, 1), bfirst;
    std::vector<int> st = {1};
    bfirst.push_back(1);
    while (!st.empty()) {
        const int k = st.back();
        st.pop_back();
        pos[k] = (int)at.size();
        at.push_back(k);
        for (int l : lat[k]) {
            blk[l] = (int)bfirst.size();
            bfirst.push_back(l);
            st.push_back(l);
        }
        if (chain[k] >= 0) {
            blk[chain[k]] = blk[k];
            st.push_back(chain[k]);
        }
    }
    if ((int)at.size() != n) return no("feeder tree does not reach every node from node 1");
    for (int q = n - 1; q > 0; --q) size[par[at[q]]] += size[at[q]];
    const int nblk = (int)bfirst.size();
    if (nblk > 0x3fff) return no("too many blocks");
    // TEMP with one common off-diagonal value per branch (fast mode's symmetric form)
    for (int q = 0; q < n; ++q) {
        const double *t = &h.tz[(size_t)h.node[at[q]].fw * 18];
        for (int j = 1; j < 9; ++j)
            if (j % 4 != 0 && !(t[2 * j] == t[2] && t[2 * j + 1] == t[3])) return no("TEMP not symmetric");
    }
    // published entries: subtree ends (backward), taps and first - 1 of the lateral
    // blocks (forward), in position order; the entry after both is the zero
    std::vector<int> cb(n, -1), cf(n, -1);
    int nE = 0, nG = 0;
    for (int q = 0; q < n; ++q) {
        const int e = q + size[at[q]] - 1;
        if (cb[e] < 0) cb[e] = 0;
    }
    for (int q = 0; q < n; ++q)
        if (cb[q] == 0) cb[q] = nE++;
    for (int b = 1; b < nblk; ++b) {
        cf[pos[par[bfirst[b]]]] = 0;
        cf[pos[bfirst[b]] - 1] = 0;
    }
    for (int q = 0; q < n; ++q)
        if (cf[q] == 0) cf[q] = nG++;
    const int zero = std::max(nE, nG);
    L.blk.assign((size_t)nblk * (1 + 2 * LANE_BD), 0);
    for (int b = 1; b < nblk; ++b) {
        int d = 0;
        for (int j = b; j != 0; j = blk[par[bfirst[j]]], ++d) {
            if (d >= LANE_BD) return no("block nesting deeper than " + std::to_string(LANE_BD));
            L.blk[(size_t)b * (1 + 2 * LANE_BD) + 1 + 2 * d] = cf[pos[par[bfirst[j]]]];
            L.blk[(size_t)b * (1 + 2 * LANE_BD) + 2 + 2 * d] = cf[pos[bfirst[j]] - 1];
        }
        L.blk[(size_t)b * (1 + 2 * LANE_BD)] = d;
    }
    // the waves' runs: the first n % NW waves one position more
    int cmax = (n + LANE_NW - 1) / LANE_NW, ns = 4;
    while (ns < cmax) ns += 4;
    if (const char *e = getenv("FPF_LANE_NS")) {   // experiments: a larger instantiation
        const int v = atoi(e);
        if (v >= ns && v <= LANE_NS && v % 4 == 0) ns = v;
    }
    L.slot.assign((size_t)LANE_NW * ns * 4, 0);
    L.temp.assign((size_t)LANE_NW * ns * LANE_TW, 0.0);
    int q0 = 0;
    for (int w = 0; w < LANE_NW; ++w) {
        const int cnt = n / LANE_NW + (w < n % LANE_NW ? 1 : 0);
        int lastb = 0;
        for (int i = 0; i < ns; ++i) {
            // the wave's table [4][ns] (struct of arrays: one scalar load per field)
            int32_t sl_[4];
            int32_t *const sl = sl_;
            double *tp = &L.temp[((size_t)w * ns + i) * LANE_TW];
            if (i < cnt) {
                const int q = q0 + i, k = at[q];
                const NodeOp &nd = h.node[k];
                const int e = q + size[k] - 1;
                const bool start = i == 0 || bfirst[blk[k]] == k;
                sl[0] = nd.row;
                sl[1] = k;
                // bit 0: a real slot; published: the subtree ends (leaves); gathered:
                // this subtree's end
                sl[2] = 1 | ((cb[q] >= 0 ? cb[q] + 1 : 0) << 1) | (cb[e] << 16);
                sl[3] = (cf[q] + 1) | (blk[k] << 16) | (start ? 1 << 30 : 0);
                const double *t = &h.tz[(size_t)nd.fw * 18];
                for (int a = 0; a < 3; ++a) {
                    tp[2 * a] = t[2 * (4 * a)] - t[2];
                    tp[2 * a + 1] = t[2 * (4 * a) + 1] - t[3];
                }
                tp[6] = t[2];
                tp[7] = t[3];
                lastb = blk[k];
            } else {
                // a dummy slot: row 0's loads scaled by 0, TEMP 0, gathers the zero entry
                sl[0] = 0;
                sl[1] = -1;
                sl[2] = zero << 16;
                sl[3] = (lastb << 16) | (i == 0 ? 1 << 30 : 0);
            }
            for (int k = 0; k < 4; ++k) L.slot[((size_t)w * 4 + k) * ns + i] = sl[k];
        }
        q0 += cnt;
    }
    L.n = n;
    L.ns = ns;
    L.nE = nE;
    L.nG = nG;
    L.nblk = nblk;
    LaneDev probe{};
    probe.nE = nE;
    probe.nG = nG;
    if (lane_lds_bytes(probe) > WAVE_LDS_BUDGET - 2048) return no("published entries exceed LDS");
    L.ok = true;
}

// Chunked sequential programs for one tile size (see fpf_internal.h).
void build_seq_programs(HostFeeder &h, int tile) {
    const int nn = h.nn, U = SEQ_CHUNK;
    const uint32_t slot = 3u * (uint32_t)tile * 16u;
    const uint32_t w_bytes = (uint32_t)(nn + 2) * slot;
    auto W = [&](int k) { return (uint32_t)k * slot; };
    auto T = [&](int t) { return w_bytes + (uint32_t)t * slot; };
    const int ZW = nn, DW = nn + 1, ZT = h.n_taps, DT = h.n_taps + 1;
    h.seq_bw.clear();
    h.seq_fw.clear();
    // backward: no op may read or add into a T slot an earlier op of its chunk adds into
    std::vector<int> written;
    auto pad_bw = [&]() {
        while (h.seq_bw.size() % U) h.seq_bw.push_back({W(ZW), W(DW), T(ZT), T(DT)});
        written.clear();
    };
    for (const auto &op : h.bwi) {
        const bool clash = (op.a >= 0 && std::count(written.begin(), written.end(), op.a)) ||
                           (op.p >= 0 && std::count(written.begin(), written.end(), op.p));
        if (clash) pad_bw();
        const uint32_t p = op.p >= 0 ? (T(op.p) | BW_SEP) : T(DT);
        h.seq_bw.push_back({W(op.k), W(op.k), T(op.a >= 0 ? op.a : ZT), p});
        if (op.p >= 0) written.push_back(op.p);
        if (h.seq_bw.size() % U == 0) written.clear();
    }
    pad_bw();
    // forward: V(src) comes from the previous op (register) or from LDS written
    // before this chunk; otherwise the chunk is closed first
    std::vector<int> wrote;
    int prev_dst = -1;
    auto pad_fw = [&]() {
        while (h.seq_fw.size() % U) h.seq_fw.push_back({W(DW), W(ZW), 0u, 0u});
        wrote.clear();
        prev_dst = -1;
    };
    for (const auto &op : h.fwi) {
        const bool prev = op.src != 0 && op.src == prev_dst;
        if (!prev && op.src != 0 && std::count(wrote.begin(), wrote.end(), op.src)) pad_fw();
        const bool prev2 = op.src != 0 && op.src == prev_dst;
        h.seq_fw.push_back({W(op.dst), W(op.src), (uint32_t)op.mask | (prev2 ? FW_PREV : 0u), 0u});
        wrote.push_back(op.dst);
        prev_dst = op.dst;
        if (h.seq_fw.size() % U == 0) wrote.clear();
    }
    pad_fw();
}

bool wants_rtc(const HostFeeder &h, const fpf_opts &o) {
    const char *lim = getenv("FPF_RTC_MAX_OPS");
    const size_t max_ops = lim ? (size_t)atol(lim) : 1024;
    return h.wf && o.specialize && (o.kernel == FPF_KERNEL_AUTO || o.kernel == FPF_KERNEL_TILED) &&
           h.bwi.size() <= max_ops;
}

// Multi-track list schedule of the sequential stages (fpf_internal.h: TrackSched).
// Units are the feeder's blocks (Dl row runs between separator rows), each on
// consecutive steps of one track.  Node v must come at least one step (D for
// a fully prefetched LDS read) after node u for every cross-block dependency
// u -> v: the forward source of a row that is not its block predecessor
// (DPF_return7.cpp:176-178) and, backward, a tap before the first node of each
// child block (the separator's Ib(sbus(m+1)) += Ibl, :138-146).  Blocks are
// placed highest bottom-level first on the track where they can start earliest.
TrackSched schedule_tracks(const HostFeeder &h, int T, int D, unsigned seed = 0) {
    const int nl = h.nl, nn = h.nn;
    TrackSched ts;
    ts.T = T;
    ts.fw_src.assign(nn, 0);
    ts.fw_mask.assign(nn, 0);
    ts.children.assign(nn, {});
    ts.bw_reset.assign(nn, 0);
    std::vector<std::vector<int>> blk(1);
    std::vector<int> blk_of(nn, -1), pos(nn, -1);
    for (int m = 0; m < nl; ++m) {
        if (h.at(m, 0) == 0) {
            if (!blk.back().empty()) blk.emplace_back();
            continue;
        }
        const int k = (int)h.at(m, 2);
        blk_of[k] = (int)blk.size() - 1;
        pos[k] = (int)blk.back().size();
        blk.back().push_back(k);
        ts.fw_src[k] = m == 0 ? 0 : (int)h.at(m, 1);   // row 0 reads V0 (:168)
        ts.fw_mask[k] = h.node[k].mask;
    }
    if (blk.back().empty()) blk.pop_back();
    const int nb = (int)blk.size();
    // children in the backward accumulation order: descending separator row
    for (int m = nl - 1; m >= 0; --m)
        if (h.at(m, 0) == 0) ts.children[(int)h.at(m + 1, 1)].push_back((int)h.at(m + 1, 2));
    for (const auto &b : blk) ts.bw_reset[b.back()] = 1;
    // cross-block dependencies u -> v
    std::vector<std::vector<int>> dep_in(nn), dep_out(nn);
    for (int b = 0; b < nb; ++b)
        for (size_t i = 0; i < blk[b].size(); ++i) {
            const int k = blk[b][i], src = ts.fw_src[k];
            if (src != 0 && !(i > 0 && blk[b][i - 1] == src)) { dep_in[k].push_back(src); dep_out[src].push_back(k); }
        }
    for (int k = 1; k < nn; ++k)
        for (int c : ts.children[k]) { dep_in[c].push_back(k); dep_out[k].push_back(c); }
    // bottom levels (deps always point to later rows, so reverse row order works)
    std::vector<int> bl(nn, 1);
    for (int b = nb - 1; b >= 0; --b)
        for (int i = (int)blk[b].size() - 1; i >= 0; --i) {
            const int k = blk[b][i];
            int v = 1 + ((size_t)i + 1 < blk[b].size() ? bl[blk[b][i + 1]] : 0);
            for (int w : dep_out[k]) v = std::max(v, D + bl[w]);
            bl[k] = v;
        }
    std::vector<std::vector<int>> pred(nb);
    for (int b = 0; b < nb; ++b)
        for (int k : blk[b])
            for (int u : dep_in[k])
                if (blk_of[u] != b) pred[b].push_back(blk_of[u]);
    std::vector<int> free(T, 0);
    std::vector<char> done(nb, 0);
    ts.step.assign(nn, -1);
    ts.track.assign(nn, -1);
    // seed 0: bottom level, ties to the earlier block; other seeds perturb the
    // priorities (xorshift) so the caller can keep the shortest of many tries
    std::vector<double> prio(nb);
    unsigned x = seed * 2654435761u + 12345u;
    for (int b = 0; b < nb; ++b) {
        x ^= x << 13; x ^= x >> 17; x ^= x << 5;
        prio[b] = bl[blk[b][0]] + (seed ? 0.999 * ((x & 0xffff) / 65536.0) * (1 + (seed % 4)) : -1e-6 * b);
    }
    for (int n = 0; n < nb; ++n) {
        int best = -1;
        for (int b = 0; b < nb; ++b) {
            if (done[b]) continue;
            bool ready = true;
            for (int p : pred[b]) ready = ready && done[p];
            if (ready && (best < 0 || prio[b] > prio[best])) best = b;
        }
        int est = 0;
        for (size_t i = 0; i < blk[best].size(); ++i)
            for (int u : dep_in[blk[best][i]])
                if (blk_of[u] != best) est = std::max(est, ts.step[u] + std::max(D, 1) - (int)i);
        int bt = 0, bs = INT32_MAX;
        for (int t = 0; t < T; ++t) {
            const int st = std::max(free[t], est);
            if (st < bs) { bs = st; bt = t; }
        }
        if (best == 0) { bt = 0; bs = 0; }   // node 1 (row 0) first, on track 0
        for (size_t i = 0; i < blk[best].size(); ++i) {
            ts.step[blk[best][i]] = bs + (int)i;
            ts.track[blk[best][i]] = bt;
        }
        free[bt] = bs + (int)blk[best].size();
        done[best] = 1;
    }
    ts.S = *std::max_element(free.begin(), free.end());
    ts.cell.assign((size_t)ts.S * T, -1);
    for (int k = 1; k < nn; ++k) ts.cell[(size_t)ts.step[k] * T + ts.track[k]] = k;
    ts.n_slots = T + ts.S * T + T;
    return ts;
}

// Comb packing of the schedule's cells into LDS slots: step s gets the lowest
// base b >= T such that b + t is free for every track t active at s.  A track
// idle at s then points at a slot that may belong to another step -- it reads
// there but never stores (fpf_rtc.cpp).  Slots 0..T-1 hold V0 (any track reads
// it at offset 0), so node slots start at T and cross-track reads at
// slot - t never go negative.
void pack_slots(TrackSched &ts, int nn) {
    const int T = ts.T, S = ts.S;
    ts.base.assign(S, T);
    ts.active.assign(S, 0u);
    ts.slot_of.assign(nn, 0);
    std::vector<char> used((size_t)T + (size_t)S * T + 2 * T, 0);
    int hi = T - 1, lo = T;
    for (int s = 0; s < S; ++s) {
        unsigned act = 0;
        for (int t = 0; t < T; ++t)
            if (ts.cell[(size_t)s * T + t] >= 0) act |= 1u << t;
        ts.active[s] = act;
        while (used[lo]) ++lo;
        int b = lo;
        for (;; ++b) {
            bool ok = true;
            for (int t = 0; t < T && ok; ++t)
                if (((act >> t) & 1) && used[(size_t)b + t]) ok = false;
            if (ok) break;
        }
        ts.base[s] = b;
        for (int t = 0; t < T; ++t)
            if ((act >> t) & 1) {
                used[(size_t)b + t] = 1;
                ts.slot_of[ts.cell[(size_t)s * T + t]] = b + t;
                hi = std::max(hi, b + t);
            }
    }
    ts.n_slots = std::max(hi + 1, *std::max_element(ts.base.begin(), ts.base.end()) + T) + T;
}

// LDS bank model of the state layout (MI355X_MICROARCH.md, LDS table): element
// (slot j, phase p, scenario s) sits at 16-byte unit j*SL + p*PS + s.  A
// ds_read_b128 serves four 16-lane groups and is conflict-free when a group's
// lanes hit distinct units mod 16; ds_write_b128 serves eight 8-lane groups,
// distinct mod 8.  Returns the worst multiplicity over the groups.
int bank_degree(const int units[64], bool write) {
    static const int rg[4][16] = {{0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
                                  {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
                                  {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
                                  {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};
    int worst = 1;
    const int ng = write ? 8 : 4, gs = write ? 8 : 16, mod = write ? 8 : 16;
    for (int g = 0; g < ng; ++g) {
        int cnt[16] = {0};
        for (int i = 0; i < gs; ++i) {
            const int ln = write ? g * 8 + i : rg[g][i];
            if (units[ln] < 0) continue;
            worst = std::max(worst, ++cnt[units[ln] % mod]);
        }
    }
    return worst;
}

struct BankLayout { int ps = 0, sl = 0, s_deg = 99, p_deg = 99; };

// Phase stride PS >= tile and slot stride SL >= 3*PS (16-byte units) that make
// the sequential lanes (phase p, track t, scenario s -> lane (p*T + t)*NS + s,
// at comb offsets base + t) conflict-free with the least padding, then the
// fewest conflicts of the parallel lanes (16 scenarios of each of 4 nodes per
// wave; compute-bound, so second).
BankLayout bank_layout(int T, int NS, int tile, int max_sl = 1 << 30) {
    BankLayout best;
    int units[64];
    for (int ps = tile; ps <= tile + 8; ++ps)
        for (int sl = 3 * ps; sl <= std::min(3 * ps + 16, max_sl); ++sl) {
            int sd = 1;
            for (int wv = 0; wv < 2; ++wv)
                for (int base = 0; base < 4; ++base)
                    for (int w = 0; w < 2; ++w) {
                        std::fill(units, units + 64, -1);
                        for (int p = 0; p < 3; ++p)
                            for (int t = 0; t < T; ++t)
                                for (int q = 0; q < NS; ++q)
                                    units[(p * T + t) * NS + q] = (base + t) * sl + p * ps + wv * NS + q;
                        sd = std::max(sd, bank_degree(units, w == 1));
                    }
            int pd = 1;
            static const int nodes[3][4] = {{0, 1, 2, 3}, {5, 9, 2, 7}, {3, 10, 17, 24}};
            for (const auto &nd : nodes)
                for (int p = 0; p < 3; ++p) {
                    for (int ln = 0; ln < 64; ++ln) {
                        const int k = ln / tile, q = ln % tile;
                        units[ln] = k < 4 ? nd[k] * sl + p * ps + q : -1;
                    }
                    pd = std::max(pd, bank_degree(units, false));
                }
            if (sd < best.s_deg || (sd == best.s_deg && (sl < best.sl || (sl == best.sl && pd < best.p_deg)))) {
                best.ps = ps;
                best.sl = sl;
                best.s_deg = sd;
                best.p_deg = pd;
            }
        }
    return best;
}

// The specialised kernel's plan: tile, tracks, scenarios per sequential wave,
// layout.  Largest tile whose tasks fit 1024 lanes x 2 and whose state fits
// LDS; among (T, NS) for that tile the lowest estimated sequential-stage time
// (steps x bank-conflict degree, sequential waves spread over the 4 SIMDs).
struct RtcPlan {
    TrackSched ts;
    int tile = 0, ns = 0, nt = 0, maxt = 0, wpc = 1;
    BankLayout lay;
};

constexpr int MAX_TILE = 16;   // = MAX_SEQ_TILE of fpf_tiled_body.h (flag arrays)
// Auto choice between the interpreted tiled kernel and the generic kernel (no
// hipRTC plan): per batch.  The generic kernel needs >= ~32 k scenarios (one
// wavefront per SIMD) to hide its memory latency; the tiled kernel scales
// linearly from few scenarios (profiles/r01i/autotile: 123- to
// 1024-bus feeders, generic faster at 65 536, tiled faster at 4 096).
constexpr int AUTO_GENERIC_MIN_SCEN = 32768;

bool plan_rtc(const HostFeeder &h, const fpf_opts &o, RtcPlan *out) {
    int force_t = 0;
    if (const char *e = getenv("FPF_RTC_TRACKS")) force_t = atoi(e);
    std::vector<TrackSched> by_t(5);
    for (int T = 1; T <= 4; ++T) {
        if (force_t && T != force_t) continue;
        for (int D = 1; D <= 4; ++D) {
            for (unsigned seed = 0; seed < (T == 1 ? 1u : 64u); ++seed) {
                TrackSched s = schedule_tracks(h, T, T == 1 ? 1 : D, seed);
                if (by_t[T].S == 0 || s.S < by_t[T].S || (s.S == by_t[T].S && seed == 0)) by_t[T] = std::move(s);
            }
            if (T == 1) break;
        }
        pack_slots(by_t[T], h.nn);
    }
    const int nb = h.nn - 1;
    // workgroups per CU: 2 lets one tile's latency-bound sequential stage overlap
    // the other tile's parallel stages (each then gets half the LDS and 512 threads)
    int wpc = 1;
    if (const char *e = getenv("FPF_RTC_WPC")) wpc = std::max(1, std::min(2, atoi(e)));
    // (two resident tiles: leave the allocation granularity some room)
    const size_t lds_budget = (size_t)160 * 1024 / wpc - (wpc > 1 ? 2048 : 0);
    int tmax = std::min(MAX_TILE, (1024 / wpc * 2) / std::max(nb, 1));
    if (o.tile > 0) tmax = std::min(tmax, o.tile);
    for (int tile = tmax; tile >= 1; --tile) {
        double best_cost = 1e30;
        for (int T = 1; T <= 4; ++T) {
            if (by_t[T].S == 0) continue;
            const int nsmax = std::min(21, 64 / (3 * T));
            int tried = 0;
            for (int w = 1; w <= 4; ++w) {
                const int ns = (tile + w - 1) / w;   // NS scenarios per sequential wave, w waves
                if (ns > nsmax || ns == tried) continue;
                if (const char *e = getenv("FPF_RTC_NS"))
                    if (atoi(e) > 0 && atoi(e) != ns) continue;
                tried = ns;
                // the largest slot stride that fits the LDS budget, then the layout
                FeederDev probe{};
                probe.n_slots = by_t[T].n_slots;
                probe.n_fw = (int)h.fw.size();
                probe.temp_lds = 1;
                int max_sl = 0;
                for (int sl = 3 * tile; sl <= 3 * tile + 40; ++sl) {
                    probe.slot_bytes = sl * 16;
                    if (tiled_lds_bytes_rtc(probe, tile) <= lds_budget) max_sl = sl;
                }
                if (max_sl == 0) continue;
                const BankLayout lay = bank_layout(T, ns, tile, max_sl);
                if (lay.sl == 0) continue;
                const int nws = (tile + ns - 1) / ns;
                // cycles per step of one sequential wave vs the waves sharing the CU's
                // LDS (MI355X, 123-bus, stamps of the whole stage: 2 waves ~81, 4 ~110;
                // tools/ubench/gen_step.py: a bare step ~50 alone, ~80 with 4 waves)
                static const double step_cyc[5] = {0, 60, 81, 100, 110};
                const double cost = by_t[T].S * step_cyc[std::min(nws, 4)] * (double)std::max(lay.s_deg, 1) *
                                        (nws > 4 ? (nws + 3) / 4 : 1) + 0.01 * T;
                if (cost < best_cost) {
                    best_cost = cost;
                    out->ts = by_t[T];
                    out->tile = tile;
                    out->ns = ns;
                    out->lay = lay;
                }
            }
        }
        if (best_cost < 1e30) {
            int n = 1024 / wpc, m = 2;
            if (const char *g = getenv("FPF_RTC_GEOM")) {
                int gn = 0, gm = 0;
                if (sscanf(g, "%d,%d", &gn, &gm) == 2 && (gn == 256 || gn == 512 || gn == 1024) && gm >= 1 && gm <= 4) {
                    n = gn;
                    m = gm;
                }
            }
            while (m < 4 && tile * nb > n * m) ++m;
            while (n > 256 && tile * nb <= (n / 2) * m) n /= 2;
            if (tile * nb > n * m || (tile + out->ns - 1) / out->ns > n / 64) continue;
            out->nt = n;
            out->maxt = m;
            out->wpc = wpc;
            return true;
        }
    }
    return false;
}

RtcSpec make_rtc_spec(const HostFeeder &h, const RtcPlan &pl, const fpf_opts &o) {
    RtcSpec sp;
    sp.tile = pl.tile;
    sp.nn = h.nn;
    sp.n_taps = h.n_taps;
    sp.nt = pl.nt;
    sp.maxt = pl.maxt;
    sp.min_waves = std::max(1, pl.wpc * pl.nt / 256);   // waves per SIMD of wpc resident tiles
    if (const char *g = getenv("FPF_RTC_GEOM")) {
        int n = 0, m = 0, w = 0;
        if (sscanf(g, "%d,%d,%d", &n, &m, &w) == 3 && w >= 1 && w <= 8) sp.min_waves = w;
    }
    if (const char *a = getenv("FPF_RTC_AHEAD")) sp.ahead = std::max(1, atoi(a));
    sp.ts = pl.ts;
    sp.ns = pl.ns;
    sp.ps = pl.lay.ps;
    sp.slot = pl.lay.sl;
    sp.exact = o.exact != 0;
    if (const char *e = getenv("FPF_RTC_TEMP_GLOBAL")) sp.temp_lds = atoi(e) == 0;
    if (const char *g = getenv("FPF_RTC_STAGGER")) {
        long c = 0;
        int sh = 8;
        if (sscanf(g, "%ld,%d", &c, &sh) >= 1) {
            sp.stagger = std::max(0L, c);
            sp.stagger_shift = std::max(0, std::min(20, sh));
        }
    }
    sp.full_k = true;
    for (int p = 0; p < 3; ++p) sp.full_k = sp.full_k && h.lnum[p] + 1 >= h.nn;
    return sp;
}

// the node table of the specialised layout
std::vector<NodeOp> node_table_rtc(const HostFeeder &h, const TrackSched &ts) {
    std::vector<NodeOp> v = h.node;
    for (int k = 0; k < h.nn; ++k) v[k].slot = ts.slot(k);
    return v;
}

template <class T>
size_t push_blob(std::vector<char> &blob, const std::vector<T> &v) {
    size_t off = (blob.size() + 255) & ~(size_t)255;
    blob.resize(off + std::max<size_t>(v.size() * sizeof(T), 8));
    if (!v.empty()) std::memcpy(blob.data() + off, v.data(), v.size() * sizeof(T));
    return off;
}

}  // namespace

extern "C" int fpf_feeder_create(fpf_ctx *ctx, const double *dl, int nl, int ncols, const double *z,
                                 int z_rows, int z_cols, const fpf_opts *opts, fpf_feeder **out) {
    if (!ctx || !out || !dl || nl < 1 || ncols < 12 || z_rows < 0 || (z_rows > 0 && !z))
        return fail(ctx, FPF_ERR_ARG, "fpf_feeder_create: bad arguments (Dl needs >= 12 columns)");
    *out = nullptr;
    fpf_opts o;
    if (opts) o = *opts;
    else fpf_opts_default(&o);
    if (o.mxitr < 1 || !(o.bkva > 0) || !(o.bkv > 0)) return fail(ctx, FPF_ERR_ARG, "bad fpf_opts");
    if (o.layout != FPF_LAYOUT_SCEN_FASTEST && o.layout != FPF_LAYOUT_SCEN_MAJOR)
        return fail(ctx, FPF_ERR_ARG, "fpf_opts.layout: FPF_LAYOUT_SCEN_FASTEST or FPF_LAYOUT_SCEN_MAJOR");

    HostFeeder h;
    h.nl = nl;
    h.ncols = ncols;
    h.dl.assign(dl, dl + (size_t)nl * ncols);
    std::string why = build_ops(h, z, z_rows, z_cols, o);
    if (why.empty()) why = build_lnum(h, z, z_rows, o);
    if (!why.empty()) return fail(ctx, FPF_ERR_TOPOLOGY, "feeder rejected (the reference would throw): " + why);
    analyse_tiled(h);
    WaveHost wh;
    analyse_wave(h, wh);
    // kernel choice: the wave kernel for fast mode, the tiled kernel for exact
    // mode (or a feeder the wave kernel refuses), the generic kernel otherwise
    int kern = o.kernel;
    if (kern == FPF_KERNEL_AUTO && !o.exact && wh.ok) kern = FPF_KERNEL_WAVE;
    if (kern == FPF_KERNEL_WAVE && (!wh.ok || o.exact))
        return fail(ctx, FPF_ERR_UNSUPPORTED,
                    o.exact ? "wave kernel: fast mode only (exact = 0)" : "wave kernel: " + wh.why);
    RtcPlan plan;
    const bool have_plan = kern != FPF_KERNEL_WAVE && wants_rtc(h, o) && plan_rtc(h, o, &plan);
    if (have_plan) {
        h.ts = plan.ts;
        h.node_rtc = node_table_rtc(h, plan.ts);
    }

    fpf_feeder *f = new fpf_feeder();
    f->ctx = ctx;
    f->opts = o;
    fpf_feeder_info &in = f->info;
    in.nl = nl;
    in.ncols = ncols;
    in.nn = h.nn;
    in.nb = h.nb;
    in.n_codes = h.ncode;
    in.n_sep = h.n_sep;
    in.n_taps = h.n_taps;
    in.well_formed = h.wf ? 1 : 0;
    for (int p = 0; p < 3; ++p) in.lnum[p] = h.lnum[p];
    in.depth = h.depth;

    // tile of the interpreted tiled kernel (its sequential programs are built for it)
    int tile = 0;
    if (h.wf) {
        FeederDev probe{};
        probe.nn = h.nn;
        probe.n_taps = h.n_taps;
        tile = tiled_max_tile(probe);
        if (o.tile > 0) tile = std::min(tile, o.tile);
    }
    if (tile >= 1) build_seq_programs(h, tile);
    // upload all tables as one blob
    std::vector<char> blob;
    const size_t o_tz = push_blob(blob, h.tz);
    const size_t o_il = push_blob(blob, h.il);
    // generic kernel: flag (kind | 2) the first op touching each Ib slot in a
    // sweep, so it starts from the constant 0 instead of re-zeroing and
    // re-reading the slot (slots no op touches are zeroed once per launch)
    std::vector<BwOp> bw_dev = h.bw;
    {
        std::vector<char> touched(h.nn > 0 ? h.nn : 1, 0);
        for (auto &op : bw_dev)
            if (op.idx >= 0 && op.idx < (int)touched.size() && !touched[op.idx]) {
                touched[op.idx] = 1;
                op.kind |= 2;
            }
    }
    const size_t o_bw = push_blob(blob, bw_dev);
    // generic kernel: the backward sweep evaluates IL(idx) itself from the op
    // that last writes that slot in the load-current pass (list order)
    std::vector<IlOp> bw_il(h.bw.size(), IlOp{-1, 0});
    {
        std::vector<IlOp> last(h.nn > 0 ? h.nn : 1, IlOp{-1, 0});
        for (const auto &op : h.il)
            if (op.ndr - 1 >= 0 && op.ndr - 1 < (int)last.size()) last[op.ndr - 1] = op;
        for (size_t q = 0; q < h.bw.size(); ++q)
            if (h.bw[q].kind == 0 && h.bw[q].idx >= 0 && h.bw[q].idx < (int)last.size()) bw_il[q] = last[h.bw[q].idx];
    }
    const size_t o_bwil = push_blob(blob, bw_il);
    // generic kernel: flag (pad | 1) a forward op whose source V is the one the
    // previous op writes, so it is carried in registers
    std::vector<FwOp> fw_dev = h.fw;
    for (size_t q = 0; q < fw_dev.size(); ++q) {
        fw_dev[q].pad = 0;
        if (q > 0 && fw_dev[q].src >= 0 && fw_dev[q].src == fw_dev[q - 1].dst) fw_dev[q].pad = 1;
    }
    const size_t o_fw = push_blob(blob, fw_dev);
    // generic kernel: the launch-time initialisation it can skip (FeederDev)
    std::vector<int32_t> il_zero, ib_zero;
    int v_init = 0;
    {
        const int nn = h.nn;
        std::vector<char> il_w(nn, 0), ib_w(nn > 1 ? nn - 1 : 1, 0), v_w(nl, 0);
        for (const auto &op : h.il)
            if (op.ndr - 1 >= 0 && op.ndr - 1 < nn) il_w[op.ndr - 1] = 1;
        for (const auto &op : h.bw)
            if (op.idx >= 0 && op.idx < (int)ib_w.size()) ib_w[op.idx] = 1;
        for (int k = 0; k < nn; ++k)
            if (!il_w[k]) il_zero.push_back(k);
        for (int k = 0; k < nn - 1; ++k)
            if (!ib_w[k]) ib_zero.push_back(k);
        // V: a forward source must have been written earlier in the list (else sweep
        // 0 reads V0 there); every V a load current or the post-processing reads
        // (nodes 1..nn-1) must have a forward writer
        for (const auto &op : h.fw) {
            if (op.src >= 0 && !v_w[op.src]) v_init = 1;
            if (op.dst >= 0 && op.dst < nl) v_w[op.dst] = 1;
        }
        for (const auto &op : h.il)
            if (op.ndr < 0 || op.ndr >= nl || !v_w[op.ndr]) v_init = 1;
        for (int k = 1; k < nn; ++k)
            if (k >= nl || !v_w[k]) v_init = 1;
        if (nl > 0 && v_w[0]) v_init = 1;   // V(0) is stored once as V0 when v_init = 0
    }
    if (il_zero.empty()) il_zero.push_back(-1);
    if (ib_zero.empty()) ib_zero.push_back(-1);
    const size_t o_ilz = push_blob(blob, il_zero), o_ibz = push_blob(blob, ib_zero);
    const size_t o_node = push_blob(blob, h.node);
    const size_t o_node_rtc = push_blob(blob, h.node_rtc);
    const size_t o_sbw = push_blob(blob, h.seq_bw);
    const size_t o_sfw = push_blob(blob, h.seq_fw);
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipMalloc(&f->d_tables, blob.size());
    if (e == hipSuccess) e = hipMemcpy(f->d_tables, blob.data(), blob.size(), hipMemcpyHostToDevice);
    e = e == hipSuccess ? hipMalloc(&f->d_agg, 8 * sizeof(double)) : e;
    e = e == hipSuccess ? hipMalloc(&f->d_ticket, sizeof(unsigned)) : e;
    e = e == hipSuccess ? hipMemset(f->d_ticket, 0, sizeof(unsigned)) : e;
    if (e != hipSuccess) {
        fpf_feeder_destroy(f);
        return fail(ctx, FPF_ERR_HIP, std::string("feeder upload: ") + hipGetErrorString(e));
    }
    char *base = (char *)f->d_tables;
    FeederDev &d = f->dev;
    d.nl = nl;
    d.nn = h.nn;
    d.ncode = h.ncode;
    d.n_il = (int)h.il.size();
    d.n_bw = (int)h.bw.size();
    d.n_fw = (int)h.fw.size();
    for (int p = 0; p < 3; ++p) d.K[p] = h.lnum[p] + 1;
    d.n_taps = h.n_taps;
    d.mxitr = o.mxitr;
    const double vo = o.vo_kv / o.bkv;   // :84
    d.V0[0] = vo;
    d.V0[1] = 0;
    d.V0[2] = (-0.5) * vo;
    d.V0[3] = (-0.5 * std::sqrt(3.0)) * vo;
    d.V0[4] = (-0.5) * vo;
    d.V0[5] = (0.5 * std::sqrt(3.0)) * vo;
    d.s3 = o.bkva / 3;
    d.eps = o.eps;
    d.lb_v = o.lb_v;
    d.ub_v = o.ub_v;
    d.tz = (const double *)(base + o_tz);
    d.il_ops = (const IlOp *)(base + o_il);
    d.bw_ops = (const BwOp *)(base + o_bw);
    d.bw_il = (const IlOp *)(base + o_bwil);
    d.il_zero = (const int32_t *)(base + o_ilz);
    d.ib_zero = (const int32_t *)(base + o_ibz);
    d.n_il_zero = il_zero[0] < 0 ? 0 : (int)il_zero.size();
    d.n_ib_zero = ib_zero[0] < 0 ? 0 : (int)ib_zero.size();
    d.v_init = getenv("FPF_GENERIC_VINIT") ? 1 : v_init;
    d.fw_ops = (const FwOp *)(base + o_fw);
    d.node_ops = (const NodeOp *)(base + o_node);
    d.seq_bw = (const SeqBw *)(base + o_sbw);
    d.seq_fw = (const SeqFw *)(base + o_sfw);
    d.n_seq_bw = (int)h.seq_bw.size();
    d.n_seq_fw = (int)h.seq_fw.size();
    d.tile = tile;
    d.prog_lds = 1;
    if (tile >= 1 && tiled_lds_bytes(d, tile) > 160 * 1024) d.prog_lds = 0;   // programs stay in HBM/L2

    if (kern == FPF_KERNEL_WAVE) {
        WaveDev &w = f->wdev;
        std::vector<char> wb;
        const size_t o_row = push_blob(wb, wh.row), o_node = push_blob(wb, wh.node), o_info = push_blob(wb, wh.info);
        const size_t o_blk = push_blob(wb, wh.blk);
        const size_t o_mref = push_blob(wb, wh.mref);
        const size_t o_tmp = push_blob(wb, wh.temp), o_pairs = push_blob(wb, wh.pairs);
        const size_t o_lng = push_blob(wb, wh.lng), o_code = push_blob(wb, wh.code), o_cz = push_blob(wb, wh.code_z);
        const size_t o_info2 = push_blob(wb, wh.info2);
        const size_t o_lagx = push_blob(wb, wh.lagx), o_bbase = push_blob(wb, wh.bbase);
        e = hipMalloc(&f->d_wave, wb.size());
        if (e == hipSuccess) e = hipMemcpy(f->d_wave, wb.data(), wb.size(), hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            fpf_feeder_destroy(f);
            return fail(ctx, FPF_ERR_HIP, std::string("wave tables upload: ") + hipGetErrorString(e));
        }
        char *wbase = (char *)f->d_wave;
        w.n = wh.n;
        w.nn = h.nn;
        w.nl = nl;
        w.spw = wh.spw;
        w.C = wh.C;
        w.nblk = wh.nblk;
        w.bdepth = wh.bdepth;
        w.ncomp = wh.ncomp;
        w.has_rel = wh.has_rel;
        w.has_mask = wh.has_mask;
        w.wpb = wh.wpb;
        w.off_in_x = wh.off_in_x;
        w.temp_sym = wh.temp_sym;
        w.dbg = getenv("FPF_WAVE_DBG") ? atoi(getenv("FPF_WAVE_DBG")) : 0;
        w.spec = o.specialize ? 1 : 0;
        w.mxitr = o.mxitr;
        for (int p = 0; p < 3; ++p) w.K[p] = d.K[p];
        for (int i = 0; i < 6; ++i) w.V0[i] = d.V0[i];
        w.s3 = d.s3;
        w.eps = d.eps;
        for (int p = 0; p < 3; ++p) w.rv0[p] = 1.0 / (d.V0[2 * p] * d.V0[2 * p] + d.V0[2 * p + 1] * d.V0[2 * p + 1]);
        w.lb_v = d.lb_v;
        w.ub_v = d.ub_v;
        w.slot_row = (const int32_t *)(wbase + o_row);
        w.slot_node = (const int32_t *)(wbase + o_node);
        w.slot_info = (const int32_t *)(wbase + o_info);
        w.slot_blk = (const int32_t *)(wbase + o_blk);
        w.slot_mref = (const int32_t *)(wbase + o_mref);
        w.slot_temp = (const double *)(wbase + o_tmp);
        w.blk_pairs = (const int32_t *)(wbase + o_pairs);
        w.wps = wh.wps;
        w.ncode = h.ncode;
        w.slot_lng = (const double *)(wbase + o_lng);
        w.slot_code = (const int32_t *)(wbase + o_code);
        w.code_z = (const double *)(wbase + o_cz);
        w.has_lag = wh.has_lag;
        w.nlag = wh.nlag;
        w.slot_lagx = (const int32_t *)(wbase + o_lagx);
        w.blk_base = (const int32_t *)(wbase + o_bbase);
        if (wh.coop) {
            // the paired kernel's exchange areas (one per scenario in flight) and
            // their arrival counts / generations (zeroed before every launch)
            w.coop = wh.coop;
            w.nb_c = wh.nb_c;
            w.nf_c = wh.nf_c;
            w.nb_split = wh.nb_split;
            w.nf_split = wh.nf_split;
            w.slot_info2 = (const int32_t *)(wbase + o_info2);
            w.coop_nslot = COOP_NSLOT;
            w.coop_area = (48 + 6 * (wh.nb_c + wh.nf_c) + 15) & ~15;
            e = hipMalloc(&f->d_xch, sizeof(double) * (size_t)w.coop_nslot * w.coop_area);
            if (e == hipSuccess) e = hipMalloc(&f->d_xsync, sizeof(unsigned) * (2 * (size_t)w.coop_nslot + 16));
            if (e == hipSuccess) e = hipMemset(f->d_xsync, 0, sizeof(unsigned) * (2 * (size_t)w.coop_nslot + 16));
            if (e != hipSuccess) {
                fpf_feeder_destroy(f);
                return fail(ctx, FPF_ERR_HIP, std::string("paired kernel exchange areas: ") + hipGetErrorString(e));
            }
            w.xch = (double *)f->d_xch;
            w.xsync = (unsigned *)f->d_xsync;
            // the sticky fault word: host memory the kernel writes when an exchange
            // gives up, so the asynchronous entry reports it without a synchronisation
            e = hipHostMalloc((void **)&f->h_xerr, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent);
            if (e != hipSuccess) {
                fpf_feeder_destroy(f);
                return fail(ctx, FPF_ERR_HIP, std::string("paired kernel fault word: ") + hipGetErrorString(e));
            }
            *(volatile unsigned *)f->h_xerr = 0;
            e = hipHostGetDevicePointer((void **)&w.xerr_host, f->h_xerr, 0);
            if (e != hipSuccess) {
                fpf_feeder_destroy(f);
                return fail(ctx, FPF_ERR_HIP, std::string("paired kernel fault word: ") + hipGetErrorString(e));
            }
            // polls before a hand-off wait gives up; FPF_TEST_COOP_SPIN (tests only)
            // makes every wait give up at once to exercise the fault path
            w.coop_spin = 1 << 21;
            if (const char *sp = getenv("FPF_TEST_COOP_SPIN")) w.coop_spin = std::max(0, atoi(sp));
            if (wh.has_mask) {   // the zeroed phases' |V| rows (the V_abc_list ranking)
                e = hipMalloc(&f->d_xvm, sizeof(double) * (size_t)w.coop_nslot * 3 * h.nn);
                if (e != hipSuccess) {
                    fpf_feeder_destroy(f);
                    return fail(ctx, FPF_ERR_HIP, std::string("paired kernel |V| rows: ") + hipGetErrorString(e));
                }
                w.xvm = (double *)f->d_xvm;
            }
        }
        if (wave_any_lds_bytes(w) > WAVE_LDS_BUDGET) {
            fpf_feeder_destroy(f);
            return fail(ctx, FPF_ERR_UNSUPPORTED, "wave kernel: LDS budget exceeded");
        }
        if (!o.no_guard) {
            f->guard = true;
            w.guard_k = guard_factor(wh.n);
            const size_t ld = fixup_scratch_ld(), per = (size_t)6 * (2 * d.nl + 2 * d.nn - 1);
            e = hipMalloc(&f->d_flag_count, sizeof(unsigned));
            if (e == hipSuccess) e = hipMemset(f->d_flag_count, 0, sizeof(unsigned));
            if (e == hipSuccess) e = hipMalloc(&f->d_fix_scratch, sizeof(double) * per * ld);
            if (e == hipSuccess) e = hipMalloc(&f->d_fixdev, sizeof(FeederDev));
            if (e == hipSuccess) e = hipMemcpy(f->d_fixdev, &d, sizeof(FeederDev), hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                fpf_feeder_destroy(f);
                return fail(ctx, FPF_ERR_HIP, std::string("guard buffers: ") + hipGetErrorString(e));
            }
        }
        f->wdev_big = w;
        f->wdev_big.wpb = wh.wpb_big_batch;
        // the lane kernel's plan (fpf_lane.hip): large light-output batches
        if (!wh.wps && !wh.coop && !getenv("FPF_NO_LANE")) {
            LaneHost lh;
            analyse_lane(h, o, lh);
            if (lh.ok) {
                std::vector<char> lb;
                const size_t o_ls = push_blob(lb, lh.slot), o_lt = push_blob(lb, lh.temp), o_lb = push_blob(lb, lh.blk);
                e = hipMalloc(&f->d_lane, lb.size());
                if (e == hipSuccess) e = hipMemcpy(f->d_lane, lb.data(), lb.size(), hipMemcpyHostToDevice);
                if (e != hipSuccess) {
                    fpf_feeder_destroy(f);
                    return fail(ctx, FPF_ERR_HIP, std::string("lane tables upload: ") + hipGetErrorString(e));
                }
                LaneDev &l = f->ldev;
                l.n = lh.n;
                l.nn = h.nn;
                l.nl = nl;
                l.nE = lh.nE;
                l.nG = lh.nG;
                l.nblk = lh.nblk;
                l.mxitr = o.mxitr;
                l.ns = lh.ns;
                for (int i = 0; i < 6; ++i) l.V0[i] = d.V0[i];
                for (int p = 0; p < 3; ++p) l.rv0[p] = w.rv0[p];
                l.s3 = d.s3;
                l.eps = d.eps;
                l.lb_v = d.lb_v;
                l.ub_v = d.ub_v;
                l.guard_k = w.guard_k;
                l.slot = (const int32_t *)((char *)f->d_lane + o_ls);
                l.temp = (const double *)((char *)f->d_lane + o_lt);
                l.blk = (const int32_t *)((char *)f->d_lane + o_lb);
                f->lane_ok = true;
            }
        }
        if (!w.wps) {
            // the table-driven staging of both launch geometries (fpf_wave.hip)
            std::vector<int32_t> sm[2], l0[2], om[2], o0[2];
            int U[2], UO[2];
            WaveDev *wv[2] = {&f->wdev, &f->wdev_big};
            std::vector<char> tb;
            size_t off[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
            for (int g = 0; g < 2; ++g) {
                U[g] = wave_stage_tables(*wv[g], sm[g], l0[g]);
                UO[g] = wave_out_tables(*wv[g], om[g], o0[g]);
                if (U[g]) {
                    off[g][0] = push_blob(tb, sm[g]);
                    off[g][1] = push_blob(tb, l0[g]);
                }
                if (UO[g]) {
                    off[g][2] = push_blob(tb, om[g]);
                    off[g][3] = push_blob(tb, o0[g]);
                }
            }
            if (!tb.empty()) {
                e = hipMalloc(&f->d_stage_tab, tb.size());
                if (e == hipSuccess) e = hipMemcpy(f->d_stage_tab, tb.data(), tb.size(), hipMemcpyHostToDevice);
                if (e != hipSuccess) {
                    fpf_feeder_destroy(f);
                    return fail(ctx, FPF_ERR_HIP, std::string("staging tables: ") + hipGetErrorString(e));
                }
            }
            for (int g = 0; g < 2; ++g) {
                wv[g]->stage_u = U[g];
                wv[g]->stage_smaj = U[g] ? (const int32_t *)((char *)f->d_stage_tab + off[g][0]) : nullptr;
                wv[g]->stage_l0 = U[g] ? (const int32_t *)((char *)f->d_stage_tab + off[g][1]) : nullptr;
                wv[g]->out_u = UO[g];
                wv[g]->out_smaj = UO[g] ? (const int32_t *)((char *)f->d_stage_tab + off[g][2]) : nullptr;
                wv[g]->out_l0 = UO[g] ? (const int32_t *)((char *)f->d_stage_tab + off[g][3]) : nullptr;
                wave_io_units(*wv[g]);
            }
        }
    }
    // auto: the interpreted tiled kernel only pays with several scenarios per
    // workgroup; below that (large feeders, e.g. 2048-bus at tile 1: 794 ms vs
    // 112 ms per 65536-scenario batch, profiles/r01f) the generic kernel wins
    bool auto_batch = false;
    if (kern == FPF_KERNEL_AUTO) {
        auto_batch = h.wf && !have_plan && tile >= 1;
        // reported kernel: the one a large (hosting-study) batch runs
        kern = (h.wf && have_plan) ? FPF_KERNEL_TILED : FPF_KERNEL_GENERIC;
    }
    if (kern == FPF_KERNEL_TILED && (!h.wf || (tile < 1 && !have_plan))) {
        fpf_feeder_destroy(f);
        return fail(ctx, FPF_ERR_UNSUPPORTED,
                    "tiled kernel needs a well-formed feeder that fits in LDS: " + (h.wf ? std::string("too large") : h.wf_why));
    }
    in.kernel = kern;
    f->auto_batch = auto_batch;
    if (kern == FPF_KERNEL_TILED && have_plan) {
        const RtcSpec sp = make_rtc_spec(h, plan, o);
        std::string err;
        RtcSpec sp0 = sp;
        sp0.keep_ib = false;
        if (rtc_build(ctx->device, sp0, &f->rtc_kernel, &err) == 0) {
            f->rtc = true;
            f->rtc_spec = sp;
            d.node_ops = (const NodeOp *)(base + o_node_rtc);   // the schedule's slots
            d.tile = plan.tile;
            d.n_slots = plan.ts.n_slots;
            d.slot_bytes = plan.lay.sl * 16;
            d.phase_bytes = plan.lay.ps * 16;
            d.temp_lds = sp.temp_lds ? 1 : 0;
        } else {
            ctx->err = err;   // not fatal: the interpreted tiled kernel runs instead
        }
    }
    if (kern == FPF_KERNEL_TILED && !f->rtc && tile < 1) {
        fpf_feeder_destroy(f);
        return fail(ctx, FPF_ERR_UNSUPPORTED, "specialised kernel failed and the interpreted one does not fit: " + ctx->err);
    }
    in.tile = (kern == FPF_KERNEL_TILED || auto_batch) ? d.tile
                                                        : (kern == FPF_KERNEL_WAVE ? wave_scenarios_per_block(f->wdev) : 0);
    in.specialized = f->rtc ? 1 : 0;
    *out = f;
    return FPF_OK;
}

extern "C" void fpf_feeder_destroy(fpf_feeder *f) {
    if (!f) return;
    (void)hipSetDevice(f->ctx->device);
    (void)hipFree(f->d_tables);
    (void)hipFree(f->d_lane);
    (void)hipFree(f->d_scratch);
    (void)hipFree(f->d_iters);
    (void)hipFree(f->d_status);
    (void)hipFree(f->d_loss);
    (void)hipFree(f->d_vmin);
    (void)hipFree(f->d_vmax);
    (void)hipFree(f->d_stage);
    (void)hipFree(f->d_agg);
    (void)hipFree(f->d_partials);
    (void)hipFree(f->d_ticket);
    (void)hipFree(f->d_wave);
    (void)hipFree(f->d_stage_tab);
    (void)hipFree(f->d_xch);
    (void)hipFree(f->d_xsync);
    (void)hipFree(f->d_xvm);
    if (f->h_xerr) (void)hipHostFree(f->h_xerr);
    (void)hipFree(f->d_lay);
    (void)hipHostFree(f->h_stage);
    (void)hipFree(f->d_flag_count);
    (void)hipFree(f->d_flag_ids);
    (void)hipFree(f->d_fix_scratch);
    (void)hipFree(f->d_fixdev);
    if (f->agg_event) (void)hipEventDestroy(f->agg_event);
    for (auto &b : f->bufs_dev) (void)hipFree(b.first);
    for (auto &b : f->bufs_host) (void)hipHostFree(b.first);
    if (f->rtc) rtc_release(f->rtc_kernel);
    if (f->rtc_ib) rtc_release(f->rtc_kernel_ib);
    delete f;
}

// Order a launch that uses state of the feeder (aggregate partials / ticket, the
// guard's flag list, scratch, exchange areas, its own output buffers) on `st`
// after the previous such launch; call agg_after() once it is enqueued.
static hipError_t agg_before(fpf_feeder *f, hipStream_t st) {
    if (!f->agg_event) {
        hipError_t e = hipEventCreateWithFlags(&f->agg_event, hipEventDisableTiming);
        if (e != hipSuccess) return e;
    }
    if (f->agg_pending && f->agg_stream != st) return hipStreamWaitEvent(st, f->agg_event, 0);
    return hipSuccess;
}
// the wave kernel's launch geometry for a batch of n_scen scenarios: the
// large-batch workgroups from WAVE_STATIC_BIG_MIN_SCEN on, and from
// WAVE_SMALL_WPB_MIN_SCEN on where the per-plan build runs the launch (light
// outputs, no zeroed phases or sequential-order plan, fpf_wave.hip: launch_wave)
// -- the static kernel is ~6 % slower on the small workgroups there (profiles/r05wio)
constexpr int WAVE_STATIC_BIG_MIN_SCEN = 16384;
static const WaveDev &wave_dev_for(const fpf_feeder *f, int n_scen, bool full = false) {
    const WaveDev &w = f->wdev;
    const bool rtc = w.spec && !full && !w.has_mask && !w.has_lag && n_scen >= wave_rtc_min();
    return n_scen >= WAVE_STATIC_BIG_MIN_SCEN || (rtc && n_scen >= WAVE_SMALL_WPB_MIN_SCEN) ? f->wdev_big : f->wdev;
}

// a wave-kernel launch that runs the lane kernel instead (fpf_lane.hip): its
// plan exists, the batch is large enough (FPF_LANE), scenario fastest, light
// outputs, the feeder's own source and flat start
static bool lane_for(const fpf_feeder *f, int n_scen, const OutDev &o) {
    // (the kernel's 32-bit buffer offsets: the whole batch below 4 GiB; V's two
    // planes both or neither)
    return f->lane_ok && n_scen >= lane_min_scen() && (size_t)6 * f->ldev.nl * n_scen * 8 < ((size_t)1 << 32) &&
           !o.v_re == !o.v_im && !o.smaj && !o.vpolar && !o.pqb && !o.pql && !o.vsrc &&
           !o.s_in && !o.skip && !o.vinit_re && !o.hook && !o.eps_dev && !o.check;
}

// the kernel a batch of n_scen scenarios runs on
static int kernel_for(const fpf_feeder *f, int n_scen) {
    if (f->auto_batch) return n_scen >= AUTO_GENERIC_MIN_SCEN ? FPF_KERNEL_GENERIC : FPF_KERNEL_TILED;
    return f->info.kernel;
}

static hipError_t agg_after(fpf_feeder *f, hipStream_t st) {
    f->agg_stream = st;
    f->agg_pending = true;
    return hipEventRecord(f->agg_event, st);
}

// the options the feeder was created with (fpf_vvc.cpp)
double fpf_feeder_bkva(const fpf_feeder *f) { return f->opts.bkva; }
double fpf_feeder_bkv(const fpf_feeder *f) { return f->opts.bkv; }

extern "C" int fpf_feeder_get_info(const fpf_feeder *f, fpf_feeder_info *info) {
    if (!f || !info) return FPF_ERR_ARG;
    *info = f->info;
    return FPF_OK;
}

extern "C" int fpf_feeder_reserve(fpf_feeder *f, int max_scen) {
    if (!f || max_scen < 0) return FPF_ERR_ARG;
    fpf_ctx *ctx = f->ctx;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (f->guard && max_scen > f->flag_cap) {   // the flag list holds every scenario of a batch
        (void)hipFree(f->d_flag_ids);
        f->d_flag_ids = nullptr;
        f->flag_cap = 0;
        HIPCHK(ctx, hipMalloc(&f->d_flag_ids, sizeof(int32_t) * std::max(max_scen, 1)));
        f->flag_cap = max_scen;
    }
    // the per-plan hipRTC wave kernel batches this large run (light outputs; the
    // full-output variant runs the static kernel, fpf_wave.hip: launch_wave):
    // built here rather than inside the first solve (fpf_rtc.cpp: wave_rtc_function)
    if (kernel_for(f, max_scen) == FPF_KERNEL_WAVE && max_scen >= wave_rtc_min()) {
        const WaveDev &w = wave_dev_for(f, max_scen);
        if (w.spec && !w.coop && !w.has_mask && !w.has_lag && !(w.wps && w.has_rel))
            (void)wave_rtc_function(ctx->device, w, false);
    }
    const bool need_scratch = kernel_for(f, max_scen) == FPF_KERNEL_GENERIC;
    if (max_scen <= f->cap) {
        if (!need_scratch || (f->d_scratch && f->scratch_ld >= (size_t)max_scen)) return FPF_OK;
        (void)hipFree(f->d_scratch);
        f->d_scratch = nullptr;
        f->scratch_ld = 0;
        const size_t ld = ((size_t)max_scen + 63) & ~(size_t)63;
        const size_t per = (size_t)6 * (2 * f->dev.nl + 2 * f->dev.nn - 1);
        HIPCHK(ctx, hipMalloc(&f->d_scratch, sizeof(double) * per * ld));
        f->scratch_ld = ld;
        return FPF_OK;
    }
    (void)hipFree(f->d_iters);
    (void)hipFree(f->d_status);
    (void)hipFree(f->d_loss);
    (void)hipFree(f->d_vmin);
    (void)hipFree(f->d_vmax);
    (void)hipFree(f->d_scratch);
    f->d_iters = nullptr; f->d_status = nullptr; f->d_loss = f->d_vmin = f->d_vmax = nullptr;
    f->d_scratch = nullptr;
    f->cap = 0;
    HIPCHK(ctx, hipMalloc(&f->d_iters, sizeof(int32_t) * max_scen));
    HIPCHK(ctx, hipMalloc(&f->d_status, sizeof(int8_t) * max_scen));
    HIPCHK(ctx, hipMalloc(&f->d_loss, sizeof(double) * max_scen));
    HIPCHK(ctx, hipMalloc(&f->d_vmin, sizeof(double) * max_scen));
    HIPCHK(ctx, hipMalloc(&f->d_vmax, sizeof(double) * max_scen));
    if (need_scratch) {
        const size_t ld = ((size_t)max_scen + 63) & ~(size_t)63;
        const size_t per = (size_t)6 * (2 * f->dev.nl + 2 * f->dev.nn - 1);
        HIPCHK(ctx, hipMalloc(&f->d_scratch, sizeof(double) * per * ld));
        f->scratch_ld = ld;
    }
    f->cap = max_scen;
    return FPF_OK;
}

// device views of a batch's outputs; the per-scenario scalars the caller does
// not ask for go to the feeder's own buffers (the aggregate reads them)
static OutDev outdev_from(const fpf_feeder *f, const fpf_outputs &u, int layout) {
    OutDev o;
    std::memset(&o, 0, sizeof(o));
    o.vpolar = u.vpolar;
    o.pqb = u.pqb;
    o.pql = u.pql;
    o.v_re = u.v_re;
    o.v_im = u.v_im;
    o.iters = u.iters ? (int32_t *)u.iters : f->d_iters;
    o.status = u.status ? (int8_t *)u.status : f->d_status;
    o.loss = u.loss ? u.loss : f->d_loss;
    o.vmin = u.vmin ? u.vmin : f->d_vmin;
    o.vmax = u.vmax ? u.vmax : f->d_vmax;
    o.smaj = layout == FPF_LAYOUT_SCEN_MAJOR ? 1 : 0;
    o.errmx = u.errmx;
    o.guard = (int8_t *)u.guard;
    return o;
}

int fpf::fixup_batch_device(fpf_feeder *f, int n_scen, const double *d_pq, const fpf_outputs *d_out, double *d_agg,
                            void *stream, int layout) {
    fpf_ctx *ctx = f->ctx;
    if (!f->guard) return FPF_OK;
    fpf_outputs none;
    std::memset(&none, 0, sizeof(none));
    OutDev o = outdev_from(f, d_out ? *d_out : none, layout);
    o.agg = d_agg;
    o.flag_count = f->d_flag_count;
    o.flag_ids = f->d_flag_ids;
    HIPCHK(ctx, launch_fixup(f->dev, n_scen, d_pq, f->d_fix_scratch, fixup_scratch_ld(), o, (hipStream_t)stream));
    return FPF_OK;
}

// The paired kernel's sticky fault word (set by a launch whose exchange wait gave
// up; its scenarios have status FPF_EXCHANGE_FAILED): FPF_ERR_EXCHANGE once, then clear
int fpf::take_exchange_fault(fpf_feeder *f) {
    // (one read-and-clear: a launch on another stream that sets the word between a
    // separate load and store would lose its report)
    if (!f || !f->h_xerr || !__atomic_exchange_n(f->h_xerr, 0u, __ATOMIC_ACQ_REL)) return FPF_OK;
    return fail(f->ctx, FPF_ERR_EXCHANGE,
                "paired wave-block kernel: an exchange wait gave up (scenarios with status FPF_EXCHANGE_FAILED)");
}

extern "C" int fpf_feeder_check(fpf_feeder *f, void *stream) {
    if (!f) return FPF_ERR_ARG;
    fpf_ctx *ctx = f->ctx;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    HIPCHK(ctx, hipStreamSynchronize((hipStream_t)stream));
    return fpf::take_exchange_fault(f);
}

extern "C" int fpf_solve_batch_device(fpf_feeder *f, int n_scen, const double *d_pq, const fpf_outputs *d_out,
                                      double *d_agg, void *stream) {
    // an earlier launch's asynchronous fault is reported first (nothing enqueued)
    const int rc = fpf::take_exchange_fault(f);
    if (rc) return rc;
    return fpf::solve_batch_device_ex(f, n_scen, d_pq, d_out, d_agg, stream, nullptr, nullptr,
                                      f ? f->opts.layout : 0);
}

bool fpf::wave_hooks_supported(fpf_feeder *f, int n_scen) {
    if (kernel_for(f, n_scen) != FPF_KERNEL_WAVE || f->wdev.wps || f->wdev.coop) return false;
    const WaveDev w = wave_dev_for(f, n_scen);
    return !w.wps && !w.coop;
}

// the byte ranges of a batch's output arrays intersect (fpf_outputs: they must not --
// the fast kernels stash IL / Ib in pql / pqb before the final values)
static bool outputs_overlap(const fpf_outputs &u, int nn, int B) {
    const size_t b = (size_t)B, m6 = 6 * (size_t)nn * b * 8, m3 = 3 * (size_t)nn * b * 8;
    const std::pair<const void *, size_t> r[] = {
        {u.vpolar, m6}, {u.pqb, m6}, {u.pql, m6}, {u.v_re, m3}, {u.v_im, m3}, {u.iters, 4 * b}, {u.status, b},
        {u.loss, 8 * b}, {u.vmin, 8 * b}, {u.vmax, 8 * b}, {u.errmx, 8 * b}, {u.guard, b}};
    const size_t n = sizeof(r) / sizeof(r[0]);
    for (size_t i = 0; i < n; ++i)
        for (size_t j = i + 1; j < n; ++j) {
            if (!r[i].first || !r[j].first) continue;
            const uintptr_t a0 = (uintptr_t)r[i].first, a1 = a0 + r[i].second;
            const uintptr_t b0 = (uintptr_t)r[j].first, b1 = b0 + r[j].second;
            if (a0 < b1 && b0 < a1) return true;
        }
    return false;
}

int fpf::solve_batch_device_ex(fpf_feeder *f, int n_scen, const double *d_pq, const fpf_outputs *d_out, double *d_agg,
                               void *stream, const double *d_vsrc, double *d_s_in, int layout, unsigned *d_flag_out,
                               const int32_t *d_skip, const double *d_vinit_re, const double *d_vinit_im,
                               const AreaHook *d_hook, unsigned long long *d_move, const double *d_eps,
                               const AreaLink *d_check, unsigned *d_check_ticket) {
    if (!f || n_scen < 0 || (n_scen > 0 && !d_pq)) return fail(f ? f->ctx : nullptr, FPF_ERR_ARG, "bad arguments");
    fpf_ctx *ctx = f->ctx;
    if (n_scen == 0) return FPF_OK;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (n_scen > f->cap) {
        int rc = fpf_feeder_reserve(f, n_scen);
        if (rc) return rc;
    }
    hipStream_t st = (hipStream_t)stream;   // NULL = the default stream
    fpf_outputs none;
    std::memset(&none, 0, sizeof(none));
    const fpf_outputs &u = d_out ? *d_out : none;
    if (outputs_overlap(u, f->dev.nn, n_scen)) return fail(ctx, FPF_ERR_ARG, "output arrays overlap (fpf_outputs)");
    OutDev o = outdev_from(f, u, layout);
    o.vsrc = d_vsrc;
    o.s_in = d_s_in;
    o.skip = d_skip;
    o.vinit_re = d_vinit_re;
    o.vinit_im = d_vinit_im;
    o.hook = d_hook;
    o.move = d_move;
    o.eps_dev = d_eps;
    o.check = d_check;
    o.check_ticket = d_check_ticket;
    if ((d_hook || d_eps || d_check) && (!d_move || !d_skip || (d_check && !d_check_ticket) ||
                                         !wave_hooks_supported(f, n_scen)))
        return fail(ctx, FPF_ERR_UNSUPPORTED, "area hooks: the plain wave kernel only, with a move slot");
    if ((d_vinit_re != nullptr) != (d_vinit_im != nullptr) || (d_vinit_re && o.smaj))
        return fail(ctx, FPF_ERR_ARG, "warm start: both planes, scenario-fastest batches only");
    hipError_t e;
    bool agg_done = false;
    const int kern = kernel_for(f, n_scen);
    // the convergence guard: the fast kernel flags, the exact fixup kernel re-solves
    // (areas with per-scenario sources have no exact counterpart: no guard there);
    // without an aggregate the wave kernel re-solves its flagged scenarios in its
    // own LDS (local mode) where they fit
    const bool guarded = kern == FPF_KERNEL_WAVE && f->guard && !d_vsrc && !d_s_in;
    const bool local_fix = guarded && !d_agg && !f->wdev.wps &&
                           (size_t)96 * (f->dev.nl + f->dev.nn) <=
                               wave_lds_bytes(wave_dev_for(f, n_scen, u.vpolar || u.pqb || u.pql)) &&
                           (!f->lane_ok || (size_t)96 * (f->dev.nl + f->dev.nn) <= lane_lds_bytes(f->ldev));
    // launches that use state of the feeder -- the generic kernel's scratch, the
    // layout copies, an aggregate's partials and ticket, the guard's flag list and
    // fixup scratch, the paired kernel's exchange areas, the feeder's own
    // per-scenario buffers (NULL outputs) -- are ordered across streams: each waits
    // for the previous one (an event per feeder).  Wave-kernel solves that use none
    // of it overlap freely.
    const bool shared = kern != FPF_KERNEL_WAVE || d_agg || (guarded && !local_fix) || f->wdev.coop || !u.iters ||
                        !u.status || !u.loss || !u.vmin || !u.vmax;
    if (shared) HIPCHK(ctx, agg_before(f, st));
    // the generic and tiled kernels read and write [field][row][B] only: a
    // scenario-major batch goes through layout-0 copies (transposed in here,
    // the matrix outputs transposed back after the launch)
    const size_t nB = (size_t)n_scen, nnl = 6 * (size_t)f->dev.nl, nn6 = 6 * (size_t)f->dev.nn, nn3 = 3 * (size_t)f->dev.nn;
    struct Tr { double *user; double **dev; size_t rows; };
    Tr tr[5] = {{u.vpolar, &o.vpolar, nn6}, {u.pqb, &o.pqb, nn6}, {u.pql, &o.pql, nn6}, {u.v_re, &o.v_re, nn3},
                {u.v_im, &o.v_im, nn3}};
    const bool transpose = o.smaj && kern != FPF_KERNEL_WAVE;
    if (transpose) {
        size_t need = nnl * nB;
        for (const Tr &t : tr)
            if (t.user) need += t.rows * nB;
        if (need * sizeof(double) > f->lay_bytes) {
            (void)hipFree(f->d_lay);
            f->d_lay = nullptr;
            f->lay_bytes = 0;
            HIPCHK(ctx, hipMalloc(&f->d_lay, need * sizeof(double)));
            f->lay_bytes = need * sizeof(double);
        }
        double *q = f->d_lay;
        HIPCHK(ctx, launch_transpose(d_pq, q, nB, nnl, st));   // [B][6 Nl] -> [6 Nl][B]
        d_pq = q;
        q += nnl * nB;
        for (Tr &t : tr)
            if (t.user) {
                *t.dev = q;
                q += t.rows * nB;
            }
        o.smaj = 0;
    }
    static const bool fused_agg = !getenv("FPF_FUSED_AGG") || atoi(getenv("FPF_FUSED_AGG")) != 0;
    const bool fuses_agg = (kern == FPF_KERNEL_TILED && f->rtc) || kern == FPF_KERNEL_WAVE;
    const bool lane = kern == FPF_KERNEL_WAVE && lane_for(f, n_scen, o);
    if (d_agg && fused_agg && fuses_agg) {
        // the specialised and wave kernels reduce the batch aggregate in their last workgroup
        const int per = lane ? 64
                             : (kern == FPF_KERNEL_WAVE
                                    ? wave_scenarios_per_block(wave_dev_for(f, n_scen, o.vpolar || o.pqb || o.pql))
                                    : f->dev.tile);
        const size_t tiles = ((size_t)n_scen + per - 1) / per;
        if (tiles > f->partials_cap) {
            (void)hipFree(f->d_partials);
            f->d_partials = nullptr;
            f->partials_cap = 0;
            HIPCHK(ctx, hipMalloc(&f->d_partials, tiles * 8 * sizeof(double)));
            f->partials_cap = tiles;
        }
        o.agg = d_agg;
        o.partials = f->d_partials;
        o.ticket = f->d_ticket;
        agg_done = true;
    }
    if ((d_vsrc || d_s_in || d_skip || d_vinit_re) && kern != FPF_KERNEL_WAVE)
        return fail(ctx, FPF_ERR_UNSUPPORTED, "per-scenario source voltages need the wave kernel");
    if (guarded) {
        if (f->flag_cap < n_scen) {
            int rc = fpf_feeder_reserve(f, n_scen);
            if (rc) return rc;
        }
        o.flag_count = f->d_flag_count;
        o.flag_ids = f->d_flag_ids;
        o.flag_out = agg_done ? d_flag_out : nullptr;
        if (local_fix) {
            // no aggregate to recompute: every wave-kernel workgroup re-solves the
            // scenarios it flagged itself, in its LDS (no second launch, nothing
            // global on the common path)
            o.fix_dev = f->d_fixdev;
        }
    }
    if (kern == FPF_KERNEL_WAVE) {
        WaveDev w = f->wdev.wps ? f->wdev : wave_dev_for(f, n_scen, o.vpolar || o.pqb || o.pql);
        if (!guarded) w.guard_k = 0.0;
        if (lane) {
            LaneDev l = f->ldev;
            if (!guarded) l.guard_k = 0.0;
            e = launch_lane(l, n_scen, d_pq, o, st);
        } else {
            e = w.wps ? launch_wblk(w, n_scen, d_pq, o, st) : launch_wave(w, n_scen, d_pq, o, st);
        }
        // with an aggregate, the exact re-solve of flagged scenarios (and the
        // aggregate again) is a launch of its own after the fast solve (it exits at
        // once when none was flagged), unless the host API defers it until it has
        // read the count (d_flag_out)
        if (e == hipSuccess && guarded && !o.fix_dev && !(d_flag_out && agg_done))
            e = launch_fixup(f->dev, n_scen, d_pq, f->d_fix_scratch, fixup_scratch_ld(), o, st);
    } else if (kern == FPF_KERNEL_TILED) {
        if (f->rtc && o.pqb && !f->rtc_ib) {
            std::string err;
            if (rtc_build(ctx->device, f->rtc_spec, &f->rtc_kernel_ib, &err) != 0)
                return fail(ctx, FPF_ERR_HIP, "hipRTC build of the PQb variant: " + err);
            f->rtc_ib = true;
        }
        e = f->rtc ? rtc_launch(o.pqb ? f->rtc_kernel_ib : f->rtc_kernel, f->dev, n_scen, d_pq, o, st)
                   : launch_tiled(f->dev, n_scen, d_pq, o, st);
    } else {
        if (!f->d_scratch || f->scratch_ld < (size_t)n_scen) {
            int rc = fpf_feeder_reserve(f, n_scen);
            if (rc) return rc;
        }
        e = launch_generic(f->dev, n_scen, d_pq, f->d_scratch, f->scratch_ld, o, st);
    }
    if (e != hipSuccess) return fail(ctx, FPF_ERR_HIP, std::string("solve launch: ") + hipGetErrorString(e));
    if (transpose)
        for (const Tr &t : tr)
            if (t.user) HIPCHK(ctx, launch_transpose(*t.dev, t.user, t.rows, nB, st));   // [rows][B] -> [B][rows]
    if (d_agg && !agg_done) {
        e = launch_aggregate(n_scen, o.status, o.loss, o.vmin, o.vmax, f->dev.lb_v, f->dev.ub_v, d_agg, nullptr,
                             nullptr, st);
        if (e != hipSuccess) return fail(ctx, FPF_ERR_HIP, std::string("aggregate launch: ") + hipGetErrorString(e));
    }
    if (shared) HIPCHK(ctx, agg_after(f, st));
    return FPF_OK;
}

extern "C" int fpf_aggregate_device(fpf_feeder *f, int n_scen, const signed char *d_status, const double *d_loss,
                                    const double *d_vmin, const double *d_vmax, double *d_agg, void *stream) {
    if (!f || n_scen < 0 || !d_agg || (n_scen > 0 && (!d_status || !d_loss || !d_vmin || !d_vmax)))
        return fail(f ? f->ctx : nullptr, FPF_ERR_ARG, "fpf_aggregate_device: bad arguments");
    fpf_ctx *ctx = f->ctx;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    if (f->partials_cap < 256) {   // scratch of the multi-block form (shared with the fused aggregates)
        (void)hipFree(f->d_partials);
        f->d_partials = nullptr;
        f->partials_cap = 0;
        HIPCHK(ctx, hipMalloc(&f->d_partials, 256 * 8 * sizeof(double)));
        f->partials_cap = 256;
    }
    HIPCHK(ctx, agg_before(f, st));
    hipError_t e = launch_aggregate(n_scen, (const int8_t *)d_status, d_loss, d_vmin, d_vmax, f->dev.lb_v, f->dev.ub_v,
                                    d_agg, f->d_partials, f->d_ticket, st);
    if (e != hipSuccess) return fail(ctx, FPF_ERR_HIP, std::string("aggregate launch: ") + hipGetErrorString(e));
    HIPCHK(ctx, agg_after(f, st));
    return FPF_OK;
}

extern "C" int fpf_solve_batch(fpf_feeder *f, int n_scen, const double *pq, const fpf_outputs *out,
                               fpf_aggregate *agg) {
    return fpf::solve_batch_host(f, n_scen, pq, out, agg, f ? f->opts.layout : 0);
}

int fpf::solve_batch_host(fpf_feeder *f, int n_scen, const double *pq, const fpf_outputs *out, fpf_aggregate *agg,
                          int layout) {
    if (!f || n_scen < 0 || (n_scen > 0 && !pq)) return fail(f ? f->ctx : nullptr, FPF_ERR_ARG, "bad arguments");
    fpf_ctx *ctx = f->ctx;
    if (n_scen == 0) {
        if (agg) std::memset(agg, 0, sizeof(*agg));
        return 0;
    }
    HIPCHK(ctx, hipSetDevice(ctx->device));
    fpf_outputs none;
    std::memset(&none, 0, sizeof(none));
    const fpf_outputs &u = out ? *out : none;
    const size_t B = (size_t)n_scen, nn = (size_t)f->info.nn, nl = (size_t)f->info.nl;
    // staging layout: pq | vpolar | pqb | pql | v_re | v_im | iters | status | loss | vmin | vmax | errmx |
    // guard | aggregate | guard count (the count of scenarios the fast kernel flagged
    // for the exact re-solve comes back with the results: no extra launch or copy
    // when none was)
    constexpr int NP = 15;
    struct Part { void *host; size_t bytes; size_t off; };
    double h_agg[8];
    unsigned h_flag[2] = {0, 0};
    Part parts[NP] = {
        {(void *)pq, 6 * nl * B * 8, 0}, {u.vpolar, 6 * nn * B * 8, 0}, {u.pqb, 6 * nn * B * 8, 0},
        {u.pql, 6 * nn * B * 8, 0},      {u.v_re, 3 * nn * B * 8, 0},  {u.v_im, 3 * nn * B * 8, 0},
        {u.iters, 4 * B, 0},             {u.status, B, 0},             {u.loss, 8 * B, 0},
        {u.vmin, 8 * B, 0},              {u.vmax, 8 * B, 0},           {u.errmx, 8 * B, 0},
        {u.guard, B, 0},                 {h_agg, sizeof(h_agg), 0},    {h_flag, sizeof(h_flag), 0}};
    size_t total = 0;
    for (Part &p : parts) {
        if (!p.host) continue;
        p.off = total;
        total += (p.bytes + 255) & ~(size_t)255;
    }
    if (total > f->stage_bytes) {
        (void)hipFree(f->d_stage);
        f->d_stage = nullptr;
        f->stage_bytes = 0;
        HIPCHK(ctx, hipMalloc(&f->d_stage, total));
        f->stage_bytes = total;
    }
    char *sb = (char *)f->d_stage;
    auto dptr = [&](int i) -> void * { return parts[i].host ? (void *)(sb + parts[i].off) : nullptr; };
    HIPCHK(ctx, hipMemcpyAsync(dptr(0), pq, parts[0].bytes, hipMemcpyHostToDevice, ctx->stream));
    fpf_outputs d;
    d.vpolar = (double *)dptr(1);
    d.pqb = (double *)dptr(2);
    d.pql = (double *)dptr(3);
    d.v_re = (double *)dptr(4);
    d.v_im = (double *)dptr(5);
    d.iters = (int *)dptr(6);
    d.status = (signed char *)dptr(7);
    d.loss = (double *)dptr(8);
    d.vmin = (double *)dptr(9);
    d.vmax = (double *)dptr(10);
    d.errmx = (double *)dptr(11);
    d.guard = (signed char *)dptr(12);
    // the guard count: written by the fast kernel's aggregating workgroup (only a
    // guarded fast solve does; else it stays 0)
    const bool guarded = f->guard && kernel_for(f, n_scen) == FPF_KERNEL_WAVE;
    HIPCHK(ctx, hipMemsetAsync(dptr(14), 0, sizeof(h_flag), ctx->stream));
    int rc = fpf::solve_batch_device_ex(f, n_scen, (const double *)dptr(0), &d, (double *)dptr(13), (void *)ctx->stream,
                                        nullptr, nullptr, layout, guarded ? (unsigned *)dptr(14) : nullptr);
    if (rc) return rc;
    // the outputs are one contiguous region after pq: small ones (a VVC round's
    // solves, a batch's per-scenario scalars) come back in one copy into pinned
    // memory -- each copy costs tens of microseconds of latency -- large ones
    // straight into the caller's arrays
    size_t o0 = total;
    for (int i = 1; i < NP; ++i)
        if (parts[i].host) o0 = std::min(o0, parts[i].off);
    const size_t obytes = total - o0;
    auto bring_back = [&]() -> int {
        if (obytes <= (size_t)4 << 20) {
            if (obytes > f->h_stage_bytes) {
                (void)hipHostFree(f->h_stage);
                f->h_stage = nullptr;
                f->h_stage_bytes = 0;
                HIPCHK(ctx, hipHostMalloc(&f->h_stage, std::max(obytes, (size_t)1 << 16)));
                f->h_stage_bytes = std::max(obytes, (size_t)1 << 16);
            }
            HIPCHK(ctx, hipMemcpyAsync(f->h_stage, sb + o0, obytes, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
            for (int i = 1; i < NP; ++i)
                if (parts[i].host) std::memcpy(parts[i].host, (char *)f->h_stage + (parts[i].off - o0), parts[i].bytes);
        } else {
            for (int i = 1; i < NP; ++i)
                if (parts[i].host)
                    HIPCHK(ctx, hipMemcpyAsync(parts[i].host, dptr(i), parts[i].bytes, hipMemcpyDeviceToHost, ctx->stream));
            HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        }
        return FPF_OK;
    };
    rc = bring_back();
    if (rc) return rc;
    // the paired kernel's fault word (a hand-off wait that gave up: those scenarios
    // report FPF_EXCHANGE_FAILED, results are in place); the stream is synchronised
    rc = fpf::take_exchange_fault(f);
    if (rc) {
        if (agg) std::memcpy(agg, h_agg, sizeof(h_agg));
        return rc;
    }
    if (guarded && h_flag[0] > 0) {
        // some decisions fell within the guard band: re-solve those scenarios on the
        // exact kernel (results and aggregate in place), then bring everything back again
        rc = fpf::fixup_batch_device(f, n_scen, (const double *)dptr(0), &d, (double *)dptr(13), (void *)ctx->stream,
                                     layout);
        if (rc) return rc;
        rc = bring_back();
        if (rc) return rc;
    }
    if (agg) std::memcpy(agg, h_agg, sizeof(h_agg));
    return (int)h_agg[4];   // non-converged count
}

extern "C" long fpf_feeder_rtc_source(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
                                      const fpf_opts *opts, char *buf, size_t buf_size) {
    if (!dl || nl < 1 || ncols < 12 || z_rows < 0 || (z_rows > 0 && !z)) return FPF_ERR_ARG;
    fpf_opts o;
    if (opts) o = *opts;
    else fpf_opts_default(&o);
    HostFeeder h;
    h.nl = nl;
    h.ncols = ncols;
    h.dl.assign(dl, dl + (size_t)nl * ncols);
    std::string why = build_ops(h, z, z_rows, z_cols, o);
    if (why.empty()) why = build_lnum(h, z, z_rows, o);
    if (!why.empty()) return FPF_ERR_TOPOLOGY;
    analyse_tiled(h);
    RtcPlan plan;
    if (!wants_rtc(h, o) || !plan_rtc(h, o, &plan)) return FPF_ERR_UNSUPPORTED;
    RtcSpec sp = make_rtc_spec(h, plan, o);
    const char *kib = getenv("FPF_RTC_KEEP_IB");
    sp.keep_ib = kib && atoi(kib);   // default: the variant solves without PQb run
    const std::string src = rtc_source(sp);
    if (buf && buf_size > 0) {
        const size_t n = std::min(buf_size - 1, src.size());
        std::memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return (long)src.size() + 1;
}

extern "C" int fpf_feeder_wave_plan(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
                                    const fpf_opts *opts, int out[8]) {
    if (!dl || !out || nl < 1 || ncols < 12 || z_rows < 0 || (z_rows > 0 && !z)) return FPF_ERR_ARG;
    fpf_opts o;
    if (opts) o = *opts;
    else fpf_opts_default(&o);
    HostFeeder h;
    h.nl = nl;
    h.ncols = ncols;
    h.dl.assign(dl, dl + (size_t)nl * ncols);
    std::string why = build_ops(h, z, z_rows, z_cols, o);
    if (why.empty()) why = build_lnum(h, z, z_rows, o);
    if (!why.empty()) return FPF_ERR_TOPOLOGY;
    analyse_tiled(h);
    WaveHost wh;
    analyse_wave(h, wh);
    WaveDev w{};
    w.spw = wh.spw;
    w.C = wh.C;
    w.nl = nl;
    w.nblk = wh.nblk;
    w.bdepth = wh.bdepth;
    w.ncomp = wh.ncomp;
    w.wpb = wh.wpb;
    w.off_in_x = wh.off_in_x;
    w.temp_sym = wh.temp_sym;
    w.wps = wh.wps;
    w.coop = wh.coop;
    w.has_rel = wh.has_rel;
    w.ncode = h.ncode;
    const int lds = !wh.ok ? 0 : (int)wave_any_lds_bytes(w);
    const int v[8] = {wh.ok ? 1 : 0, wh.spw, wh.C, wh.wpb, lds, wh.ncomp, wh.nblk, wh.bdepth};
    std::memcpy(out, v, sizeof(v));
    return FPF_OK;
}

extern "C" int fpf_feeder_lane_plan(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols,
                                    const fpf_opts *opts, int out[8], int *slots, int slots_len, int *blk,
                                    int blk_len) {
    if (!dl || !out || nl < 1 || ncols < 12 || z_rows < 0 || (z_rows > 0 && !z)) return FPF_ERR_ARG;
    fpf_opts o;
    if (opts) o = *opts;
    else fpf_opts_default(&o);
    HostFeeder h;
    h.nl = nl;
    h.ncols = ncols;
    h.dl.assign(dl, dl + (size_t)nl * ncols);
    std::string why = build_ops(h, z, z_rows, z_cols, o);
    if (why.empty()) why = build_lnum(h, z, z_rows, o);
    if (!why.empty()) return FPF_ERR_TOPOLOGY;
    analyse_tiled(h);
    LaneHost lh;
    analyse_lane(h, o, lh);
    LaneDev l{};
    l.nE = lh.nE;
    l.nG = lh.nG;
    const int v[8] = {lh.ok ? 1 : 0, lh.ns, LANE_NW, lh.ok ? (int)lane_lds_bytes(l) : 0, lh.nE, lh.nG, lh.nblk, lh.n};
    std::memcpy(out, v, sizeof(v));
    if (slots && lh.ok)
        for (int i = 0; i < slots_len && i < (int)lh.slot.size(); ++i) slots[i] = lh.slot[i];
    if (blk && lh.ok)
        for (int i = 0; i < blk_len && i < (int)lh.blk.size(); ++i) blk[i] = lh.blk[i];
    return FPF_OK;
}

extern "C" long fpf_feeder_wave_rtc_source(const double *dl, int nl, int ncols, const double *z, int z_rows,
                                           int z_cols, const fpf_opts *opts, int big_batch, int full, char *buf,
                                           size_t buf_size) {
    if (!dl || nl < 1 || ncols < 12 || z_rows < 0 || (z_rows > 0 && !z)) return FPF_ERR_ARG;
    fpf_opts o;
    if (opts) o = *opts;
    else fpf_opts_default(&o);
    HostFeeder h;
    h.nl = nl;
    h.ncols = ncols;
    h.dl.assign(dl, dl + (size_t)nl * ncols);
    std::string why = build_ops(h, z, z_rows, z_cols, o);
    if (why.empty()) why = build_lnum(h, z, z_rows, o);
    if (!why.empty()) return FPF_ERR_TOPOLOGY;
    analyse_tiled(h);
    WaveHost wh;
    analyse_wave(h, wh);
    if (!wh.ok || wh.coop) return FPF_ERR_UNSUPPORTED;
    // the plan values fpf_feeder_create puts in the launch's WaveDev
    WaveDev w{};
    w.nn = h.nn;
    w.nl = nl;
    w.spw = wh.spw;
    w.C = wh.C;
    w.nblk = wh.nblk;
    w.bdepth = wh.bdepth;
    w.ncomp = wh.ncomp;
    w.has_rel = wh.has_rel;
    w.has_mask = wh.has_mask;
    w.wpb = big_batch ? wh.wpb_big_batch : wh.wpb;
    w.off_in_x = wh.off_in_x;
    w.temp_sym = wh.temp_sym;
    w.mxitr = o.mxitr;
    w.wps = wh.wps;
    w.ncode = h.ncode;
    if (!w.wps) {
        std::vector<int32_t> a, b;
        w.stage_u = wave_stage_tables(w, a, b);
        w.out_u = wave_out_tables(w, a, b);
        wave_io_units(w);
    }
    std::string name;
    const std::string src = wave_rtc_source(w, full != 0, &name);
    if (buf && buf_size > 0) {
        const size_t n = std::min(buf_size - 1, src.size());
        std::memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return (long)src.size() + 1;
}
