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
    // topology-specialised tiled kernel (hipRTC), if built
    bool rtc = false;
    RtcKernel rtc_kernel{};
};

static int fail(fpf_ctx *ctx, int code, const std::string &msg) {
    if (ctx) ctx->err = msg;
    return code;
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
    h.node.assign(nn, NodeOp{-1, -1, -1, 0, -1});
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

// tile for the tiled kernel; *nt / *maxt describe the specialised build's geometry
int choose_tile(const HostFeeder &h, const fpf_opts &o, int *nt = nullptr, int *maxt = nullptr) {
    if (!h.wf) return 0;
    FeederDev probe{};
    probe.nn = h.nn;
    probe.n_taps = h.n_taps;
    int tmax, n = 0, m = 0;
    if (wants_rtc(h, o)) {
        tmax = rtc_tile(probe, &n, &m);
        if (tmax < 1) tmax = tiled_max_tile(probe);
    } else {
        tmax = tiled_max_tile(probe);
    }
    if (nt) *nt = n;
    if (maxt) *maxt = m;
    return o.tile > 0 ? std::min(o.tile, tmax) : tmax;
}

RtcSpec make_rtc_spec(const HostFeeder &h, int tile, int nt, int maxt) {
    RtcSpec sp;
    sp.tile = tile;
    sp.nn = h.nn;
    sp.n_taps = h.n_taps;
    sp.nt = nt;
    sp.maxt = maxt;
    sp.min_waves = std::max(1, 4 * 256 / nt);   // <= 128 VGPRs: 4 waves per SIMD
    if (const char *g = getenv("FPF_RTC_GEOM")) {
        int n = 0, m = 0, w = 0;
        if (sscanf(g, "%d,%d,%d", &n, &m, &w) == 3 && w >= 1 && w <= 8) sp.min_waves = w;
    }
    for (const auto &op : h.bwi) sp.bw.push_back({op.k, op.a, op.p});
    for (const auto &op : h.fwi) sp.fw.push_back({op.dst, op.src, op.mask});
    return sp;
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

    HostFeeder h;
    h.nl = nl;
    h.ncols = ncols;
    h.dl.assign(dl, dl + (size_t)nl * ncols);
    std::string why = build_ops(h, z, z_rows, z_cols, o);
    if (why.empty()) why = build_lnum(h, z, z_rows, o);
    if (!why.empty()) return fail(ctx, FPF_ERR_TOPOLOGY, "feeder rejected (the reference would throw): " + why);
    analyse_tiled(h);

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

    // tile of the tiled kernel (the sequential programs are built for it)
    const int tile = choose_tile(h, o);
    if (tile >= 1) build_seq_programs(h, tile);
    // upload all tables as one blob
    std::vector<char> blob;
    const size_t o_tz = push_blob(blob, h.tz);
    const size_t o_il = push_blob(blob, h.il);
    const size_t o_bw = push_blob(blob, h.bw);
    const size_t o_fw = push_blob(blob, h.fw);
    const size_t o_node = push_blob(blob, h.node);
    const size_t o_sbw = push_blob(blob, h.seq_bw);
    const size_t o_sfw = push_blob(blob, h.seq_fw);
    hipError_t e = hipSetDevice(ctx->device);
    if (e == hipSuccess) e = hipMalloc(&f->d_tables, blob.size());
    if (e == hipSuccess) e = hipMemcpy(f->d_tables, blob.data(), blob.size(), hipMemcpyHostToDevice);
    e = e == hipSuccess ? hipMalloc(&f->d_agg, 8 * sizeof(double)) : e;
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
    d.fw_ops = (const FwOp *)(base + o_fw);
    d.node_ops = (const NodeOp *)(base + o_node);
    d.seq_bw = (const SeqBw *)(base + o_sbw);
    d.seq_fw = (const SeqFw *)(base + o_sfw);
    d.n_seq_bw = (int)h.seq_bw.size();
    d.n_seq_fw = (int)h.seq_fw.size();
    d.tile = tile;
    d.prog_lds = 1;
    if (tile >= 1 && tiled_lds_bytes(d, tile) > 160 * 1024) d.prog_lds = 0;   // programs stay in HBM/L2

    // kernel choice
    int kern = o.kernel;
    if (kern == FPF_KERNEL_AUTO) kern = (h.wf && tile >= 1) ? FPF_KERNEL_TILED : FPF_KERNEL_GENERIC;
    if (kern == FPF_KERNEL_TILED && (!h.wf || tile < 1)) {
        fpf_feeder_destroy(f);
        return fail(ctx, FPF_ERR_UNSUPPORTED,
                    "tiled kernel needs a well-formed feeder that fits in LDS: " + (h.wf ? std::string("too large") : h.wf_why));
    }
    in.kernel = kern;
    in.tile = kern == FPF_KERNEL_TILED ? tile : 0;
    int rtc_nt = 0, rtc_maxt = 0;
    (void)choose_tile(h, o, &rtc_nt, &rtc_maxt);
    // an explicit tile above the default geometry takes more tasks per lane
    while (rtc_nt > 0 && rtc_maxt < 4 && tile * (h.nn - 1) > rtc_nt * rtc_maxt) ++rtc_maxt;
    while (rtc_nt > 256 && tile * (h.nn - 1) <= (rtc_nt / 2) * rtc_maxt) rtc_nt /= 2;
    if (kern == FPF_KERNEL_TILED && wants_rtc(h, o) && rtc_nt > 0 && tile * (h.nn - 1) <= rtc_nt * rtc_maxt) {
        const RtcSpec sp = make_rtc_spec(h, tile, rtc_nt, rtc_maxt);
        if (tiled_lds_bytes_rtc(d, tile) <= 160 * 1024) {
            std::string err;
            if (rtc_build(ctx->device, sp, &f->rtc_kernel, &err) == 0) {
                f->rtc = true;
            } else {
                ctx->err = err;   // not fatal: the interpreted tiled kernel runs instead
            }
        }
    }
    in.specialized = f->rtc ? 1 : 0;
    *out = f;
    return FPF_OK;
}

extern "C" void fpf_feeder_destroy(fpf_feeder *f) {
    if (!f) return;
    (void)hipSetDevice(f->ctx->device);
    (void)hipFree(f->d_tables);
    (void)hipFree(f->d_scratch);
    (void)hipFree(f->d_iters);
    (void)hipFree(f->d_status);
    (void)hipFree(f->d_loss);
    (void)hipFree(f->d_vmin);
    (void)hipFree(f->d_vmax);
    (void)hipFree(f->d_stage);
    (void)hipFree(f->d_agg);
    delete f;
}

extern "C" int fpf_feeder_get_info(const fpf_feeder *f, fpf_feeder_info *info) {
    if (!f || !info) return FPF_ERR_ARG;
    *info = f->info;
    return FPF_OK;
}

extern "C" int fpf_feeder_reserve(fpf_feeder *f, int max_scen) {
    if (!f || max_scen < 0) return FPF_ERR_ARG;
    fpf_ctx *ctx = f->ctx;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (max_scen <= f->cap) return FPF_OK;
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
    if (f->info.kernel == FPF_KERNEL_GENERIC) {
        const size_t ld = ((size_t)max_scen + 63) & ~(size_t)63;
        const size_t per = (size_t)6 * (2 * f->dev.nl + 2 * f->dev.nn - 1);
        HIPCHK(ctx, hipMalloc(&f->d_scratch, sizeof(double) * per * ld));
        f->scratch_ld = ld;
    }
    f->cap = max_scen;
    return FPF_OK;
}

extern "C" int fpf_solve_batch_device(fpf_feeder *f, int n_scen, const double *d_pq, const fpf_outputs *d_out,
                                      double *d_agg, void *stream) {
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
    OutDev o;
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
    hipError_t e;
    if (f->info.kernel == FPF_KERNEL_TILED) {
        e = f->rtc ? rtc_launch(f->rtc_kernel, f->dev, n_scen, d_pq, o, st) : launch_tiled(f->dev, n_scen, d_pq, o, st);
    } else {
        if (!f->d_scratch || f->scratch_ld < (size_t)n_scen) {
            int rc = fpf_feeder_reserve(f, n_scen);
            if (rc) return rc;
        }
        e = launch_generic(f->dev, n_scen, d_pq, f->d_scratch, f->scratch_ld, o, st);
    }
    if (e != hipSuccess) return fail(ctx, FPF_ERR_HIP, std::string("solve launch: ") + hipGetErrorString(e));
    if (d_agg) {
        e = launch_aggregate(n_scen, o.status, o.loss, o.vmin, o.vmax, f->dev.lb_v, f->dev.ub_v, d_agg, st);
        if (e != hipSuccess) return fail(ctx, FPF_ERR_HIP, std::string("aggregate launch: ") + hipGetErrorString(e));
    }
    return FPF_OK;
}

extern "C" int fpf_aggregate_device(fpf_feeder *f, int n_scen, const signed char *d_status, const double *d_loss,
                                    const double *d_vmin, const double *d_vmax, double *d_agg, void *stream) {
    if (!f || n_scen < 0 || !d_agg || (n_scen > 0 && (!d_status || !d_loss || !d_vmin || !d_vmax)))
        return fail(f ? f->ctx : nullptr, FPF_ERR_ARG, "fpf_aggregate_device: bad arguments");
    fpf_ctx *ctx = f->ctx;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t st = (hipStream_t)stream;
    hipError_t e = launch_aggregate(n_scen, (const int8_t *)d_status, d_loss, d_vmin, d_vmax, f->dev.lb_v, f->dev.ub_v,
                                    d_agg, st);
    if (e != hipSuccess) return fail(ctx, FPF_ERR_HIP, std::string("aggregate launch: ") + hipGetErrorString(e));
    return FPF_OK;
}

extern "C" int fpf_solve_batch(fpf_feeder *f, int n_scen, const double *pq, const fpf_outputs *out,
                               fpf_aggregate *agg) {
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
    // staging layout: pq | vpolar | pqb | pql | v_re | v_im | iters | status | loss | vmin | vmax
    struct Part { void *host; size_t bytes; size_t off; };
    Part parts[11] = {
        {(void *)pq, 6 * nl * B * 8, 0}, {u.vpolar, 6 * nn * B * 8, 0}, {u.pqb, 6 * nn * B * 8, 0},
        {u.pql, 6 * nn * B * 8, 0},      {u.v_re, 3 * nn * B * 8, 0},  {u.v_im, 3 * nn * B * 8, 0},
        {u.iters, 4 * B, 0},             {u.status, B, 0},             {u.loss, 8 * B, 0},
        {u.vmin, 8 * B, 0},              {u.vmax, 8 * B, 0}};
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
    int rc = fpf_solve_batch_device(f, n_scen, (const double *)dptr(0), &d, f->d_agg, (void *)ctx->stream);
    if (rc) return rc;
    for (int i = 1; i < 11; ++i)
        if (parts[i].host)
            HIPCHK(ctx, hipMemcpyAsync(parts[i].host, dptr(i), parts[i].bytes, hipMemcpyDeviceToHost, ctx->stream));
    double h_agg[8];
    HIPCHK(ctx, hipMemcpyAsync(h_agg, f->d_agg, sizeof(h_agg), hipMemcpyDeviceToHost, ctx->stream));
    HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
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
    const int tile = choose_tile(h, o);
    if (tile < 1) return FPF_ERR_UNSUPPORTED;
    FeederDev d{};
    d.nn = h.nn;
    d.n_taps = h.n_taps;
    int nt = 0, maxt = 0;
    (void)choose_tile(h, o, &nt, &maxt);
    if (nt == 0) return FPF_ERR_UNSUPPORTED;
    const std::string src = rtc_source(make_rtc_spec(h, tile, nt, maxt));
    if (buf && buf_size > 0) {
        const size_t n = std::min(buf_size - 1, src.size());
        std::memcpy(buf, src.data(), n);
        buf[n] = 0;
    }
    return (long)src.size() + 1;
}
