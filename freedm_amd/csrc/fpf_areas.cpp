// fpf_areas.cpp -- the multi-area solve (BASELINE config 5: the Broker_s1..s3
// feeder areas).  The reference splits the feeder by SST ownership across
// three slave DGIs (Broker_s1/src/vvc/VoltVarCtrl.cpp:327-395: s1 = SST2-4,
// s2 = SST1, s3 = SST5-7 -- the rows of the master's SST map,
// Broker/src/vvc/VoltVarCtrl.cpp:442-1135) but the slaves never solve a power
// flow; this is the "per-area batched solves with boundary-voltage exchange"
// of SURVEY.md 8(d) config 5 -- an algorithm with no reference counterpart,
// checked against the monolithic solve.
//
// Each area is a connected subtree of the feeder.  Its own Dl table (rebuilt
// with local node numbers, chain-first blocks) is fed from its boundary bus:
// local node 0 is the bus of the parent area its top branch hangs off.  One
// outer iteration, batched over all scenarios on the GPU:
//   for each area, parents before children:
//     loads  = the area's own loads + at every bus a child hangs off, the power
//              the child drew at its source in the previous iteration (PQb row 0);
//     source = V0 for the root area, else the parent's voltage at the boundary
//              bus from this iteration;
//     a full DPF solve of the area (wave kernel, the caller's eps / mxitr).
// until no boundary voltage moves by more than `tol` (p.u.).  At the fixed
// point every area satisfies the monolithic equations (constant-power loads,
// the same branch impedances), so V equals the monolithic solution to the
// solver tolerance: the areas' eps and `tol` near 1e-12 give 1e-10 agreement
// with a monolithic solve run to the same eps (tests/test_areas.py).
#include "../../include/freedm_pf.h"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "fpf_internal.h"

namespace fpf {
hipError_t areas_setup(const double *src, int nl, const int32_t *map, int rows, int B, double *dst, int n_areas,
                       const int32_t *sub_off, const int32_t *sub_rows, double *s_in, int32_t *ctl, double *last,
                       unsigned long long *move, double *eps_dev, double eps_first, hipStream_t st);
hipError_t areas_link(const AreaLink &L, int B, int32_t *ctl, hipStream_t st);
hipError_t areas_scatter_nodes(const double *src, int nn, int k0, const int32_t *mono, int nn_dst, int B, double *dst,
                               hipStream_t st);
hipError_t areas_fold_results(int B, const AreaFold &F, double *o_loss, double *o_vmin, double *o_vmax,
                              int8_t *o_status, hipStream_t st);
}  // namespace fpf

using namespace fpf;

namespace {
struct Area {
    int parent = -1;             // parent area, -1: the root (fed from the substation)
    int bus = 0;                 // monolithic bus it is fed from (root: 0)
    int lb = 0;                  // that bus's local node in the parent area
    std::vector<double> dl;      // local Dl, nl x ncols column-major
    int nl = 0, nn = 0;
    std::vector<int32_t> row_of_local;   // local Dl row -> monolithic row (-1: separator)
    std::vector<int32_t> mono;           // local node -> monolithic node (local 0 -> bus)
    std::vector<int> local_of;           // monolithic node -> local node (-1: not here)
    std::vector<std::pair<int, int>> kids;   // (local row carrying the bus's load, child area)
    std::vector<int32_t> sub_rows;       // monolithic rows of the area's whole subtree (its own and its descendants')
    fpf_feeder *feeder = nullptr;
    // device buffers
    int32_t *d_mono = nullptr;
    size_t roff = 0;             // the area's first line in fpf_areas::d_base / d_work
    double *d_base = nullptr, *d_work = nullptr;   // [6][nl][B] in fpf_areas::d_base / d_work (not owned)
    double *d_vsrc = nullptr;
    double *d_sin = nullptr;   // [6][B] in fpf_areas::d_sin (not owned)
    double *d_vre = nullptr, *d_vim = nullptr, *d_loss = nullptr, *d_vmin = nullptr, *d_vmax = nullptr;
    int32_t *d_iters = nullptr;
    int8_t *d_status = nullptr;
};
}  // namespace

struct fpf_areas {
    fpf_ctx *ctx = nullptr;
    int nl = 0, ncols = 0, nn = 0;
    double lb_v = 0.96, ub_v = 1.05;   // the hosting counters of the aggregate (fpf_opts)
    double eps = 1e-4;                 // the areas' inner eps (fpf_opts)
    // inexact outer iterations (with hooks, more than one area): the first
    // iteration's solves run to eps_first, each later one to inexact x the
    // previous boundary move, never looser than eps_first nor tighter than eps --
    // the early iterations' areas stop sweeping once they are as accurate as
    // their boundary is; the loop stops only after an iteration solved to eps.
    // FPF_AREAS_INEXACT (0: off) / FPF_AREAS_EPS_FIRST
    double inexact = 1e-4, eps_first = 1e-6;
    bool warm = true;                  // warm-started area solves (FPF_AREAS_WARM=0: flat V0 each time)
    int last_outer = 0;                // the previous solve's outer iterations (the first chunk's size)
    std::vector<Area> area;      // index = area id, parents before children
    std::vector<int> order;      // solve order
    int cap = 0, vcap = 0;
    hipStream_t stream = nullptr;
    // when some area has more than one child area: one stream and one "solved"
    // event per area -- within an outer iteration an area waits only for its
    // parent (its source voltage), so siblings (and their subtrees) run
    // concurrently; the check joins them all.  Otherwise (a chain of areas, where
    // nothing can overlap) everything on `stream`: the cross-stream waits cost
    // about 11 us each (profiles/r04h_c5).  FPF_AREAS_STREAMS=0 / 1 forces either.
    std::vector<hipStream_t> astream;
    std::vector<hipEvent_t> aev;
    hipEvent_t ev_start = nullptr;
    double *d_pq = nullptr;
    double *d_sin = nullptr;                       // [area][6][B] children's source powers
    unsigned long long *d_move = nullptr;          // [2] the iteration's boundary move (by parity, link_kernel)
    int32_t *d_sub_off = nullptr, *d_sub_rows = nullptr;   // Area::sub_rows of every area, CSR
    // the links folded into the area solves (AreaHook, one per area; the plain wave
    // kernel for every area, at most AREA_MAX_KIDS children each): an outer
    // iteration is then its n_areas solves and one stop-test launch.
    // FPF_AREAS_HOOKS=0: separate link launches (A/B)
    AreaHook *d_hook = nullptr;
    bool hooks_env = true;
    // every area's loads, one block: [sum of 6 nl][B] (gathered from the feeder's
    // batch by d_gmap in one launch), and the working copy of the link launches
    double *d_base = nullptr, *d_work = nullptr;
    int32_t *d_gmap = nullptr;
    int n_gmap = 0;
    // the stop test fused into the last area's solve (OutDev::check): its
    // arguments by iteration parity, and the workgroups' ticket
    AreaLink h_check[2] = {};
    AreaLink *d_check = nullptr;
    unsigned *d_ticket = nullptr;
    // the whole-feeder results, one block so that one copy brings them back:
    // [ctl: done, outer, 2 pad (int32)][last move][loss B][vmin B][vmax B][status B (int8)]
    char *d_res = nullptr, *h_res = nullptr;   // h_res: pinned
    double *d_vre = nullptr, *d_vim = nullptr;  // [3][Nn][B] in the feeder's numbering (when V is asked for)
    std::string err;
};

namespace {
constexpr size_t RES_HEAD = 32;   // ctl (16 bytes) + the last boundary move (8) + the inexact inner eps (8)
size_t res_bytes(size_t B) { return RES_HEAD + 24 * B + ((B + 7) & ~(size_t)7); }
}  // namespace

namespace {
int afail(fpf_areas *a, int code, const std::string &msg) {
    if (a) a->err = msg;
    return code;
}
#define AHIP(a, expr)                                                                                  \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess) return afail(a, FPF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

void free_area_buffers(Area &ar) {
    (void)hipFree(ar.d_vsrc);
    (void)hipFree(ar.d_vre);
    (void)hipFree(ar.d_vim);
    (void)hipFree(ar.d_loss);
    (void)hipFree(ar.d_vmin);
    (void)hipFree(ar.d_vmax);
    (void)hipFree(ar.d_iters);
    (void)hipFree(ar.d_status);
    ar.d_base = ar.d_work = ar.d_vsrc = ar.d_sin = ar.d_vre = ar.d_vim = nullptr;
    ar.d_loss = ar.d_vmin = ar.d_vmax = nullptr;
    ar.d_iters = nullptr;
    ar.d_status = nullptr;
}
}  // namespace

extern "C" void fpf_areas_destroy(fpf_areas *a) {
    if (!a) return;
    if (a->ctx) (void)hipSetDevice(ctx_device(a->ctx));
    for (Area &ar : a->area) {
        free_area_buffers(ar);
        (void)hipFree(ar.d_mono);
        fpf_feeder_destroy(ar.feeder);
    }
    (void)hipFree(a->d_pq);
    (void)hipFree(a->d_sin);
    (void)hipFree(a->d_move);
    (void)hipFree(a->d_hook);
    (void)hipFree(a->d_base);
    (void)hipFree(a->d_work);
    (void)hipFree(a->d_gmap);
    (void)hipFree(a->d_check);
    (void)hipFree(a->d_ticket);
    (void)hipFree(a->d_sub_off);
    (void)hipFree(a->d_sub_rows);
    (void)hipFree(a->d_res);
    (void)hipHostFree(a->h_res);
    (void)hipFree(a->d_vre);
    (void)hipFree(a->d_vim);
    for (hipEvent_t e : a->aev) (void)hipEventDestroy(e);
    for (hipStream_t s : a->astream) (void)hipStreamDestroy(s);
    if (a->ev_start) (void)hipEventDestroy(a->ev_start);
    if (a->stream) (void)hipStreamDestroy(a->stream);
    delete a;
}

extern "C" const char *fpf_areas_last_error(const fpf_areas *a) { return a ? a->err.c_str() : "null context"; }

extern "C" int fpf_areas_create(fpf_ctx *ctx, const double *dl, int nl, int ncols, const double *z, int z_rows,
                                int z_cols, const int *node_area, int nn, const fpf_opts *opts, fpf_areas **out) {
    if (!ctx || !dl || !node_area || !out || nl < 1 || ncols < 12 || nn < 2) return FPF_ERR_ARG;
    *out = nullptr;
    if (hipSetDevice(ctx_device(ctx)) != hipSuccess) return FPF_ERR_HIP;
    auto at = [&](int r, int c) { return dl[(size_t)c * nl + r]; };
    // the feeder tree: row of each node, parent bus
    std::vector<int> row_of(nn, -1), par(nn, -1);
    int nb = 0;
    for (int m = 0; m < nl; ++m) {
        if (at(m, 0) == 0) continue;
        const int k = (int)at(m, 2), s = m == 0 ? 0 : (int)at(m, 1);
        if (k < 1 || k >= nn || s < 0 || s >= nn || row_of[k] >= 0) return FPF_ERR_TOPOLOGY;
        row_of[k] = m;
        par[k] = s;
        ++nb;
    }
    if (nb != nn - 1) return FPF_ERR_TOPOLOGY;
    int n_areas = 0;
    for (int k = 1; k < nn; ++k) {
        if (node_area[k] < 0) return FPF_ERR_ARG;
        n_areas = std::max(n_areas, node_area[k] + 1);
    }
    fpf_areas *a = new fpf_areas();
    a->ctx = ctx;
    a->nl = nl;
    a->ncols = ncols;
    a->nn = nn;
    a->area.resize(n_areas);
    // each area: exactly one top node (parent outside the area)
    std::vector<int> top(n_areas, -1);
    for (int k = 1; k < nn; ++k) {
        const int ar = node_area[k];
        if (par[k] == 0 || node_area[par[k]] != ar) {
            if (top[ar] >= 0) {
                fpf_areas_destroy(a);
                return FPF_ERR_TOPOLOGY;   // area not connected
            }
            top[ar] = k;
        }
    }
    for (int ar = 0; ar < n_areas; ++ar)
        if (top[ar] < 0) {
            fpf_areas_destroy(a);
            return FPF_ERR_ARG;   // empty area id
        }
    // children of every node, in monolithic row order
    std::vector<std::vector<int>> kids(nn);
    for (int m = 0; m < nl; ++m)
        if (at(m, 0) != 0) {
            const int k = (int)at(m, 2);
            kids[par[k]].push_back(k);
        }
    for (int ar = 0; ar < n_areas; ++ar) {
        Area &A = a->area[ar];
        const int t = top[ar];
        A.bus = par[t];
        A.parent = A.bus == 0 ? -1 : node_area[A.bus];
        A.local_of.assign(nn, -1);
        A.mono.push_back(A.bus);
        A.local_of[A.bus] = 0;
        // rows: chain-first blocks, laterals (within the area) after separators
        std::vector<std::vector<double>> rows;   // each ncols wide
        std::vector<int32_t> mrow;
        std::vector<std::pair<int, int>> queue = {{A.bus, t}};
        for (size_t qi = 0; qi < queue.size(); ++qi) {
            int u = queue[qi].first, v = queue[qi].second;
            if (qi > 0) {
                rows.push_back(std::vector<double>(ncols, 0.0));
                mrow.push_back(-1);
            }
            while (v >= 0) {
                const int lv = (int)A.mono.size();
                A.mono.push_back(v);
                A.local_of[v] = lv;
                std::vector<double> r(ncols);
                for (int c = 0; c < ncols; ++c) r[c] = at(row_of[v], c);
                r[1] = A.local_of[u];
                r[2] = lv;
                rows.push_back(r);
                mrow.push_back(row_of[v]);
                int next = -1;
                for (int w : kids[v])
                    if (node_area[w] == ar) {
                        if (next < 0) next = w;
                        else queue.push_back({v, w});
                    }
                u = v;
                v = next;
            }
        }
        // DPF_return7 indexes V by receiving bus in a field of Nl entries
        // (DPF_return7.cpp:92-96, 113), so a table without a separator row
        // cannot hold its last bus: such an area gets a zero-length, unloaded
        // lateral (its bus repeats its tap's voltage and carries no current)
        if (std::find(mrow.begin(), mrow.end(), -1) == mrow.end()) {
            rows.push_back(std::vector<double>(ncols, 0.0));
            mrow.push_back(-1);
            std::vector<double> r(ncols, 0.0);
            r[0] = 1;
            r[1] = 1;
            r[2] = (double)A.mono.size();
            r[3] = rows[0][3];
            r[4] = 0.0;
            r[5] = rows[0][5];
            rows.push_back(r);
            mrow.push_back(-2);
            A.mono.push_back(-1);
        }
        A.nl = (int)rows.size();
        A.nn = (int)A.mono.size();
        A.dl.assign((size_t)A.nl * ncols, 0.0);
        int ln = 0;
        for (int r = 0; r < A.nl; ++r) {
            for (int c = 0; c < ncols; ++c) A.dl[(size_t)c * A.nl + r] = rows[r][c];
            if (mrow[r] != -1) A.dl[r] = ++ln;
        }
        for (auto &m : mrow) m = m < 0 ? -1 : m;   // the pad row gathers no loads
        A.row_of_local = mrow;
    }
    // children of each area: the local row whose receiving bus is the boundary bus
    for (int ar = 0; ar < n_areas; ++ar) {
        Area &A = a->area[ar];
        if (A.parent < 0) continue;
        Area &P = a->area[A.parent];
        A.lb = P.local_of[A.bus];
        int lrow = -1;
        for (int r = 0; r < P.nl; ++r)
            if (P.row_of_local[r] == row_of[A.bus]) lrow = r;
        if (A.lb < 1 || lrow < 0) {
            fpf_areas_destroy(a);
            return FPF_ERR_TOPOLOGY;
        }
        P.kids.push_back({lrow, ar});
    }
    // every non-root area's subtree rows (the first iteration's source-power estimate)
    for (int ar = 0; ar < n_areas; ++ar)
        for (int d = ar; d >= 0 && a->area[d].parent >= 0; d = a->area[d].parent)
            for (int32_t m : a->area[ar].row_of_local)
                if (m >= 0) a->area[d].sub_rows.push_back(m);
    // solve order: parents first
    std::vector<int> depth(n_areas, 0);
    for (int ar = 0; ar < n_areas; ++ar)
        for (int p = a->area[ar].parent; p >= 0; p = a->area[p].parent) ++depth[ar];
    a->order.resize(n_areas);
    for (int ar = 0; ar < n_areas; ++ar) a->order[ar] = ar;
    std::stable_sort(a->order.begin(), a->order.end(), [&](int x, int y) { return depth[x] < depth[y]; });
    if (a->area[a->order[0]].parent >= 0) {
        fpf_areas_destroy(a);
        return FPF_ERR_TOPOLOGY;
    }
    // one feeder per area: the wave kernel (fast mode; per-scenario source voltage)
    fpf_opts o;
    if (opts) o = *opts;
    else fpf_opts_default(&o);
    a->lb_v = o.lb_v;
    a->eps = o.eps;
    if (const char *e = getenv("FPF_AREAS_INEXACT")) a->inexact = atof(e);
    if (const char *e = getenv("FPF_AREAS_EPS_FIRST")) a->eps_first = atof(e);
    a->ub_v = o.ub_v;
    if (const char *e = getenv("FPF_AREAS_WARM")) a->warm = atoi(e) != 0;   // (A/B, tests)
    if (const char *e = getenv("FPF_AREAS_HOOKS")) a->hooks_env = atoi(e) != 0;

    if (hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking) != hipSuccess) {
        fpf_areas_destroy(a);
        return FPF_ERR_HIP;
    }
    bool branching = false;
    for (const Area &A : a->area) branching = branching || A.kids.size() > 1;
    if (const char *e = getenv("FPF_AREAS_STREAMS")) branching = atoi(e) != 0;
    if (a->area.size() > 1 && branching) {
        bool ok = hipEventCreateWithFlags(&a->ev_start, hipEventDisableTiming) == hipSuccess;
        for (size_t i = 0; ok && i < a->area.size(); ++i) {
            hipStream_t s = nullptr;
            hipEvent_t e = nullptr;
            ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
            if (ok) a->astream.push_back(s);
            ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
            if (ok) a->aev.push_back(e);
        }
        if (!ok) {
            fpf_areas_destroy(a);
            return FPF_ERR_HIP;
        }
    }
    o.kernel = FPF_KERNEL_WAVE;
    o.exact = 0;
    o.layout = FPF_LAYOUT_SCEN_FASTEST;   // fpf_areas_solve's arrays are [field][row][B] (include/freedm_pf.h)
    {
        // the areas' lines of the feeder's batch: area after area, [field][local row]
        std::vector<int32_t> gmap;
        for (Area &A : a->area) {
            A.roff = gmap.size();
            for (int f = 0; f < 6; ++f)
                for (int r = 0; r < A.nl; ++r)
                    gmap.push_back(A.row_of_local[r] < 0 ? -1 : f * nl + A.row_of_local[r]);
        }
        a->n_gmap = (int)gmap.size();
        if (hipMalloc(&a->d_gmap, sizeof(int32_t) * gmap.size()) != hipSuccess ||
            hipMalloc(&a->d_check, 2 * sizeof(AreaLink)) != hipSuccess ||
            hipMalloc(&a->d_ticket, sizeof(unsigned)) != hipSuccess ||
            hipMemset(a->d_ticket, 0, sizeof(unsigned)) != hipSuccess ||
            hipMemcpy(a->d_gmap, gmap.data(), sizeof(int32_t) * gmap.size(), hipMemcpyHostToDevice) != hipSuccess) {
            fpf_areas_destroy(a);
            return FPF_ERR_HIP;
        }
    }
    {
        std::vector<int32_t> off(1, 0), rows;
        for (const Area &A : a->area) {
            rows.insert(rows.end(), A.sub_rows.begin(), A.sub_rows.end());
            off.push_back((int32_t)rows.size());
        }
        if (rows.empty()) rows.push_back(0);
        if (hipMalloc(&a->d_sub_off, sizeof(int32_t) * off.size()) != hipSuccess ||
            hipMalloc(&a->d_sub_rows, sizeof(int32_t) * rows.size()) != hipSuccess ||
            hipMalloc(&a->d_move, 2 * sizeof(unsigned long long)) != hipSuccess ||
            hipMalloc(&a->d_hook, sizeof(AreaHook) * a->area.size()) != hipSuccess ||
            hipMemcpy(a->d_sub_off, off.data(), sizeof(int32_t) * off.size(), hipMemcpyHostToDevice) != hipSuccess ||
            hipMemcpy(a->d_sub_rows, rows.data(), sizeof(int32_t) * rows.size(), hipMemcpyHostToDevice) != hipSuccess) {
            fpf_areas_destroy(a);
            return FPF_ERR_HIP;
        }
    }
    for (Area &A : a->area) {
        const int rc = fpf_feeder_create(ctx, A.dl.data(), A.nl, ncols, z, z_rows, z_cols, &o, &A.feeder);
        if (rc != FPF_OK) {
            a->err = fpf_last_error(ctx);
            fpf_areas_destroy(a);
            return rc;
        }
        if (hipMalloc(&A.d_mono, sizeof(int32_t) * A.nn) != hipSuccess ||
            hipMemcpy(A.d_mono, A.mono.data(), sizeof(int32_t) * A.nn, hipMemcpyHostToDevice) != hipSuccess) {
            fpf_areas_destroy(a);
            return FPF_ERR_HIP;
        }
    }
    *out = a;
    return FPF_OK;
}

extern "C" int fpf_areas_info(const fpf_areas *a, int *n_areas, int *area_nodes, int *area_parent) {
    if (!a || !n_areas) return FPF_ERR_ARG;
    *n_areas = (int)a->area.size();
    for (size_t i = 0; i < a->area.size(); ++i) {
        if (area_nodes) area_nodes[i] = a->area[i].nn - 1;
        if (area_parent) area_parent[i] = a->area[i].parent;
    }
    return FPF_OK;
}

static int areas_reserve(fpf_areas *a, int B, bool want_v) {
    const size_t b = (size_t)B;
    if (B > a->cap) {
        for (Area &A : a->area) free_area_buffers(A);
        (void)hipFree(a->d_pq);
        (void)hipFree(a->d_sin);
        (void)hipFree(a->d_base);
        (void)hipFree(a->d_work);
        (void)hipFree(a->d_res);
        (void)hipHostFree(a->h_res);
        a->d_pq = a->d_sin = a->d_base = a->d_work = nullptr;
        a->d_res = a->h_res = nullptr;
        a->cap = 0;
        AHIP(a, hipMalloc(&a->d_pq, sizeof(double) * 6 * a->nl * b));
        AHIP(a, hipMalloc(&a->d_sin, sizeof(double) * 6 * b * a->area.size()));
        AHIP(a, hipMalloc(&a->d_res, res_bytes(b)));
        AHIP(a, hipHostMalloc((void **)&a->h_res, res_bytes(b) + 16, hipHostMallocDefault));   // + the flag slots
        AHIP(a, hipMalloc(&a->d_base, sizeof(double) * a->n_gmap * b));
        AHIP(a, hipMalloc(&a->d_work, sizeof(double) * a->n_gmap * b));
        for (size_t ar = 0; ar < a->area.size(); ++ar) {
            Area &A = a->area[ar];
            A.d_sin = a->d_sin + ar * 6 * b;
            A.d_base = a->d_base + A.roff * b;
            A.d_work = a->d_work + A.roff * b;
        }
        for (Area &A : a->area) {
            AHIP(a, hipMalloc(&A.d_vsrc, sizeof(double) * 6 * b));
            AHIP(a, hipMalloc(&A.d_vre, sizeof(double) * 3 * A.nn * b));
            AHIP(a, hipMalloc(&A.d_vim, sizeof(double) * 3 * A.nn * b));
            AHIP(a, hipMalloc(&A.d_loss, sizeof(double) * b));
            AHIP(a, hipMalloc(&A.d_vmin, sizeof(double) * b));
            AHIP(a, hipMalloc(&A.d_vmax, sizeof(double) * b));
            AHIP(a, hipMalloc(&A.d_iters, sizeof(int32_t) * b));
            AHIP(a, hipMalloc(&A.d_status, sizeof(int8_t) * b));
        }
        // the hooks point at the buffers just allocated
        std::vector<AreaHook> hk(a->area.size());
        for (size_t ar = 0; ar < a->area.size(); ++ar) {
            const Area &A = a->area[ar];
            AreaHook &h = hk[ar];
            std::memset(&h, 0, sizeof(h));
            for (size_t j = 0; j < A.kids.size() && j < (size_t)AREA_MAX_KIDS; ++j) {
                const Area &Ch = a->area[A.kids[j].second];
                h.pre_lrow[j] = A.kids[j].first;
                h.pre_sin[j] = Ch.d_sin;
                h.post_lb[j] = Ch.lb;
                h.post_vsrc[j] = Ch.d_vsrc;
            }
            h.pre_n = h.post_n = (int)std::min(A.kids.size(), (size_t)AREA_MAX_KIDS);
        }
        AHIP(a, hipMemcpy(a->d_hook, hk.data(), sizeof(AreaHook) * hk.size(), hipMemcpyHostToDevice));
        a->cap = B;
    }
    if (want_v && B > a->vcap) {
        (void)hipFree(a->d_vre);
        (void)hipFree(a->d_vim);
        a->d_vre = a->d_vim = nullptr;
        a->vcap = 0;
        AHIP(a, hipMalloc(&a->d_vre, sizeof(double) * 3 * a->nn * b));
        AHIP(a, hipMalloc(&a->d_vim, sizeof(double) * 3 * a->nn * b));
        a->vcap = B;
    }
    return FPF_OK;
}

// pq: host [6][Nl][B] of the whole feeder; out (host): v_re / v_im [3][Nn][B]
// in the feeder's node numbering, iters = outer iterations, status (worst
// area; FPF_NONCONVERGED also when the outer loop did not reach tol), loss
// (sum over areas), vmin / vmax (over areas).  vpolar / pqb / pql must be NULL.
//
// Schedule: no host round trip inside the outer loop.  The convergence test is a
// device flag (link_kernel's stop test: ctl[0]);
// every kernel of an iteration enqueued after it is set does nothing.  The host
// enqueues iterations in chunks and looks at the flag of chunk c (an 8-byte
// copy into pinned memory) only after chunk c + 1 is enqueued, so the GPU never
// waits for the host; at most two chunks of no-op launches follow convergence.
// The scalar results and the flag come back in one copy.
extern "C" int fpf_areas_solve(fpf_areas *a, int n_scen, const double *pq, double tol, int max_outer,
                               const fpf_outputs *out, fpf_aggregate *agg) {
    if (!a || n_scen < 0 || (n_scen > 0 && !pq) || !(tol > 0) || max_outer < 1)
        return afail(a, FPF_ERR_ARG, "fpf_areas_solve: bad arguments");
    fpf_outputs none;
    std::memset(&none, 0, sizeof(none));
    const fpf_outputs &u = out ? *out : none;
    if (u.vpolar || u.pqb || u.pql || u.errmx || u.guard)
        return afail(a, FPF_ERR_UNSUPPORTED, "fpf_areas_solve: Vpolar / PQb / PQL / errmx / guard not produced");
    if (n_scen == 0) {
        if (agg) fpf_aggregate_fold(nullptr, 0, agg);
        return 0;
    }
    const int B = n_scen;
    const size_t b = (size_t)B;
    const bool want_v = u.v_re || u.v_im;
    AHIP(a, hipSetDevice(ctx_device(a->ctx)));
    int rc = areas_reserve(a, B, want_v);
    if (rc) return rc;
    hipStream_t st = a->stream;
    int32_t *ctl = (int32_t *)a->d_res;
    double *last = (double *)(a->d_res + 16);
    double *r_loss = (double *)(a->d_res + RES_HEAD), *r_vmin = r_loss + b, *r_vmax = r_vmin + b;
    int8_t *r_status = (int8_t *)(r_vmax + b);
    AHIP(a, hipMemcpyAsync(a->d_pq, pq, sizeof(double) * 6 * a->nl * b, hipMemcpyHostToDevice, st));
    const bool par = !a->astream.empty();
    const int single = a->area.size() == 1 ? 1 : 0;
    // the areas' loads and their working copies (the rows a child hangs off are
    // rewritten every iteration, every other row of d_work is the base, copied
    // once), and the first iteration's source powers: each child's subtree load
    bool hooks = a->hooks_env;
    for (Area &A : a->area) hooks = hooks && A.kids.size() <= (size_t)AREA_MAX_KIDS && wave_hooks_supported(A.feeder, B);
    // (the inexact iterations' inner eps, RES_HEAD's last 8 bytes, set by that launch)
    const bool inexact = hooks && !single && a->inexact > 0 && a->eps_first > a->eps;
    double *eps_dev = inexact ? (double *)(a->d_res + 24) : nullptr;
    // (also the loop's state in the result head and the move slots)
    AHIP(a, areas_setup(a->d_pq, a->nl, a->d_gmap, a->n_gmap, B, a->d_base, (int)a->area.size(), a->d_sub_off,
                        a->d_sub_rows, a->d_sin, ctl, last, a->d_move, eps_dev, a->eps_first, st));
    if (!hooks)
        AHIP(a, hipMemcpyAsync(a->d_work, a->d_base, sizeof(double) * a->n_gmap * b, hipMemcpyDeviceToDevice, st));
    // the stop test's arguments for iteration `it`
    auto fill_check = [&](AreaLink &L, int it) {
        L.move_acc = a->d_move + (it & 1);
        L.move_chk = a->d_move + (it & 1);
        L.move_clr = a->d_move + ((it + 1) & 1);
        L.last = last;
        L.tol = tol;
        L.single = single;
        L.eps_dev = eps_dev;
        L.eps = a->eps;
        L.eps_first = a->eps_first;
        L.inexact = a->inexact;
    };
    // one stream with hooks: the stop test runs in the last area's solve
    const bool fused_check = hooks && !par;
    if (fused_check) {
        AreaLink hc[2];
        for (int p = 0; p < 2; ++p) {
            std::memset(&hc[p], 0, sizeof(AreaLink));
            fill_check(hc[p], p);
            hc[p].check = 1;
        }
        if (std::memcmp(hc, a->h_check, sizeof(hc)) != 0) {   // (the same as the previous solve's: no copy)
            std::memcpy(a->h_check, hc, sizeof(hc));
            AHIP(a, hipMemcpyAsync(a->d_check, a->h_check, sizeof(a->h_check), hipMemcpyHostToDevice, st));
        }
    }
    // one link launch (link_kernel): the children's source voltages after `post`'s
    // solve, the child rows of `pre` before its solve, the stop test of iteration
    // `it` (AREA_MAX_KIDS children of each at a time)
    auto link = [&](const Area *post, const Area *pre, bool check, int it, hipStream_t s) -> int {
        const size_t np = post ? post->kids.size() : 0, nq = pre ? pre->kids.size() : 0;
        const size_t n = std::max<size_t>(std::max((np + AREA_MAX_KIDS - 1) / AREA_MAX_KIDS,
                                                   (nq + AREA_MAX_KIDS - 1) / AREA_MAX_KIDS), check ? 1 : 0);
        for (size_t c = 0; c < n; ++c) {
            AreaLink L{};
            if (post) {
                L.v_re = post->d_vre;
                L.v_im = post->d_vim;
                L.nn = post->nn;
                for (size_t j = c * AREA_MAX_KIDS; j < np && L.post.n < AREA_MAX_KIDS; ++j, ++L.post.n) {
                    const Area &Ch = a->area[post->kids[j].second];
                    L.post.lrow[L.post.n] = Ch.lb;
                    L.post.ptr[L.post.n] = Ch.d_vsrc;
                }
            }
            if (pre) {
                L.work = pre->d_work;
                L.base = pre->d_base;
                L.nl = pre->nl;
                for (size_t j = c * AREA_MAX_KIDS; j < nq && L.pre.n < AREA_MAX_KIDS; ++j, ++L.pre.n) {
                    L.pre.lrow[L.pre.n] = pre->kids[j].first;
                    L.pre.ptr[L.pre.n] = a->area[pre->kids[j].second].d_sin;
                }
            }
            fill_check(L, it);
            // the stop test reads the move once every post of the iteration is done:
            // in its own launch after them (the last area in the order has no children)
            L.check = check && c + 1 == n ? 1 : 0;
            if (L.check && L.post.n > 0) return afail(a, FPF_ERR_TOPOLOGY, "areas: stop test fused with a post link");
            AHIP(a, areas_link(L, B, ctl, s));
        }
        return FPF_OK;
    };
    auto solve_area = [&](Area &A, bool warm, int it, hipStream_t s, bool check) -> int {
        fpf_outputs o;
        std::memset(&o, 0, sizeof(o));
        o.v_re = A.d_vre;
        o.v_im = A.d_vim;
        o.iters = A.d_iters;
        o.status = (signed char *)A.d_status;
        o.loss = A.d_loss;
        o.vmin = A.d_vmin;
        o.vmax = A.d_vmax;
        const size_t ai = (size_t)(&A - a->area.data());
        const int r = solve_batch_device_ex(A.feeder, B, hooks ? A.d_base : A.d_work, &o, nullptr, (void *)s,
                                            A.parent >= 0 ? A.d_vsrc : nullptr, A.d_sin, FPF_LAYOUT_SCEN_FASTEST,
                                            nullptr, ctl, warm ? A.d_vre : nullptr, warm ? A.d_vim : nullptr,
                                            hooks ? a->d_hook + ai : nullptr, hooks ? a->d_move + (it & 1) : nullptr,
                                            eps_dev, check ? a->d_check + (it & 1) : nullptr,
                                            check ? a->d_ticket : nullptr);
        if (r < 0) return afail(a, r, std::string("area solve: ") + fpf_last_error(a->ctx));
        static const bool dbg = getenv("FPF_AREAS_DEBUG") && atoi(getenv("FPF_AREAS_DEBUG")) != 0;
        if (dbg) {   // (diagnostics: every area solve's sweeps; synchronises)
            std::vector<int32_t> h(b);
            AHIP(a, hipMemcpyAsync(h.data(), A.d_iters, sizeof(int32_t) * b, hipMemcpyDeviceToHost, s));
            AHIP(a, hipStreamSynchronize(s));
            long sum = 0;
            int mx = 0;
            for (int32_t x : h) sum += x, mx = std::max(mx, (int)x);
            double mv = 0.0;
            if (check) AHIP(a, hipMemcpy(&mv, last, 8, hipMemcpyDeviceToHost));
            fprintf(stderr, "areas it %d area %d: sweeps mean %.2f max %d%s%.3e\n", it, (int)ai, (double)sum / B, mx,
                    check ? ", boundary move " : "", check ? mv : 0.0);
        }
        return FPF_OK;
    };
    // from the second outer iteration on, every area solve starts from its own V of
    // the previous one (a warm start: its sweeps then only follow the boundary's
    // move, instead of ~10 sweeps from the flat V0 to the inner tolerance).
    // With hooks: the solves (each its links folded in), then the stop test --
    // on one stream, or each area on its stream after its parent's.  Without:
    // one stream: solve, link(post this, pre next), ..., the last link also the
    // stop test and the root's rows of the next iteration -- n_areas solves and
    // n_areas links per iteration; per-area streams: each area's pre link, solve
    // and post link on its stream after its parent's; the stop test joins them.
    auto enqueue_iteration = [&](int it, bool warm) -> int {
        int r = FPF_OK;
        if (fused_check) {
            for (size_t i = 0; !r && i < a->order.size(); ++i)
                r = solve_area(a->area[a->order[i]], warm, it, st, i + 1 == a->order.size());
            return r;
        }
        if (!par) {
            if (it == 0) r = link(nullptr, &a->area[a->order[0]], false, it, st);
            for (size_t i = 0; !r && i < a->order.size(); ++i) {
                Area &A = a->area[a->order[i]];
                r = solve_area(A, warm, it, st, false);
                const bool last_area = i + 1 == a->order.size();
                if (!r) r = link(&A, &a->area[a->order[last_area ? 0 : i + 1]], last_area, it, st);
            }
            return r;
        }
        AHIP(a, hipEventRecord(a->ev_start, st));
        for (int ar : a->order) {
            Area &A = a->area[ar];
            const hipStream_t sa = a->astream[ar];
            AHIP(a, hipStreamWaitEvent(sa, A.parent >= 0 ? a->aev[A.parent] : a->ev_start, 0));
            if (!hooks && !A.kids.empty()) r = link(nullptr, &A, false, it, sa);
            if (!r) r = solve_area(A, warm, it, sa, false);
            if (!r && !hooks && !A.kids.empty()) r = link(&A, nullptr, false, it, sa);
            if (r) return r;
            AHIP(a, hipEventRecord(a->aev[ar], sa));
        }
        for (size_t ar = 0; ar < a->area.size(); ++ar) AHIP(a, hipStreamWaitEvent(st, a->aev[ar], 0));
        return link(nullptr, nullptr, true, it, st);
    };
    // results in the feeder's numbering; whole-feeder loss / extremes / status.
    // Without V they are enqueued after every chunk (before its flag is looked
    // at): the chunk that ends the loop then needs no further launch
    auto enqueue_results = [&](bool with_v) -> int {
        AreaFold F{};
        F.first = 1;
        for (size_t i = 0; i < a->order.size(); ++i) {
            const Area &A = a->area[a->order[i]];
            F.loss[F.n] = A.d_loss;
            F.vmin[F.n] = A.d_vmin;
            F.vmax[F.n] = A.d_vmax;
            F.status[F.n] = A.d_status;
            if (++F.n == AREA_MAX_FOLD || i + 1 == a->order.size()) {
                AHIP(a, areas_fold_results(B, F, r_loss, r_vmin, r_vmax, r_status, st));
                F.n = 0;
                F.first = 0;
            }
        }
        for (int ar : a->order) {
            Area &A = a->area[ar];
            if (with_v) {
                // the root area's local node 0 is the substation (monolithic node 0)
                const int k0 = A.parent < 0 ? 0 : 1;
                AHIP(a, areas_scatter_nodes(A.d_vre, A.nn, k0, A.d_mono, a->nn, B, a->d_vre, st));
                AHIP(a, areas_scatter_nodes(A.d_vim, A.nn, k0, A.d_mono, a->nn, B, a->d_vim, st));
            }
        }
        AHIP(a, hipMemcpyAsync(a->h_res, a->d_res, res_bytes(b), hipMemcpyDeviceToHost, st));
        return FPF_OK;
    };
    // chunks of K iterations; the flag of chunk c is read after chunk c + 1 is enqueued
    const int K = 2;
    int32_t *const h_flag = (int32_t *)(a->h_res + res_bytes(b));
    int32_t *h_ctl[2] = {h_flag, h_flag + 2};   // two 8-byte slots after the pinned results
    hipEvent_t ev[2] = {nullptr, nullptr};
    AHIP(a, hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    AHIP(a, hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    // the first chunk is as long as the previous solve's loop (repeated studies of
    // one feeder converge in about as many outer iterations), and its flag is read
    // at once: a solve that needs no more then enqueues no no-op iterations
    const int first_chunk = a->last_outer >= K ? std::min(a->last_outer, max_outer) : 0;
    int enq = 0, chunk = 0;
    bool stop = false;
    while (!stop && enq < max_outer) {
        const int n_it = chunk == 0 && first_chunk ? first_chunk : K;
        for (int i = 0; i < n_it && enq < max_outer; ++i, ++enq) {
            rc = enqueue_iteration(enq, enq > 0 && a->warm);
            if (rc) break;
        }
        if (rc) break;
        // (the first chunk's flag, read at once, comes back with the results when
        // those are enqueued after every chunk: no copy of its own)
        const bool flag_in_res = chunk == 0 && first_chunk && !want_v;
        if (!flag_in_res) AHIP(a, hipMemcpyAsync(h_ctl[chunk & 1], ctl, 8, hipMemcpyDeviceToHost, st));
        if (!want_v) {
            rc = enqueue_results(false);
            if (rc) break;
        }
        AHIP(a, hipEventRecord(ev[chunk & 1], st));
        if (chunk == 0 && first_chunk) {
            AHIP(a, hipEventSynchronize(ev[0]));
            stop = (flag_in_res ? ((const int32_t *)a->h_res)[0] : h_ctl[0][0]) != 0;
        } else if (chunk > 0) {
            AHIP(a, hipEventSynchronize(ev[(chunk - 1) & 1]));
            stop = stop || h_ctl[(chunk - 1) & 1][0] != 0;
        }
        ++chunk;
    }
    (void)hipEventDestroy(ev[0]);
    (void)hipEventDestroy(ev[1]);
    if (rc) {
        (void)hipStreamSynchronize(st);
        return rc;
    }
    if (want_v) {
        rc = enqueue_results(true);
        if (rc) return rc;
    }
    if (u.v_re) AHIP(a, hipMemcpyAsync(u.v_re, a->d_vre, sizeof(double) * 3 * a->nn * b, hipMemcpyDeviceToHost, st));
    if (u.v_im) AHIP(a, hipMemcpyAsync(u.v_im, a->d_vim, sizeof(double) * 3 * a->nn * b, hipMemcpyDeviceToHost, st));
    AHIP(a, hipStreamSynchronize(st));
    for (int ar : a->order) {   // a paired-kernel area whose exchange gave up (FPF_EXCHANGE_FAILED)
        const int fr = take_exchange_fault(a->area[ar].feeder);
        if (fr) {
            a->err = "area " + std::to_string(ar) + ": " + fpf_last_error(a->ctx);
            return fr;
        }
    }
    const int32_t *h_c = (const int32_t *)a->h_res;
    const bool conv = h_c[0] != 0;
    const int outer = h_c[1];
    a->last_outer = outer;
    double h_last;
    std::memcpy(&h_last, a->h_res + 16, 8);
    const double *h_loss = (const double *)(a->h_res + RES_HEAD), *h_vmin = h_loss + b, *h_vmax = h_vmin + b;
    const int8_t *h_status = (const int8_t *)(h_vmax + b);
    auto status_of = [&](int s) -> int8_t { return conv ? h_status[s] : (int8_t)FPF_NONCONVERGED; };
    if (u.iters)
        for (int s = 0; s < B; ++s) u.iters[s] = outer;
    if (u.status)
        for (int s = 0; s < B; ++s) u.status[s] = status_of(s);
    if (u.loss) std::memcpy(u.loss, h_loss, sizeof(double) * b);
    if (u.vmin) std::memcpy(u.vmin, h_vmin, sizeof(double) * b);
    if (u.vmax) std::memcpy(u.vmax, h_vmax, sizeof(double) * b);
    // the aggregate as every fpf_aggregate producer forms it (converged scenarios;
    // n_over / n_under by the hosting bounds)
    int n_nonconv = 0;
    fpf_aggregate g;
    std::memset(&g, 0, sizeof(g));
    g.vmin = INFINITY;
    g.vmax = -INFINITY;
    for (int s = 0; s < B; ++s) {
        if (status_of(s) == FPF_CONVERGED) {
            g.loss_sum += h_loss[s];
            g.vmin = std::min(g.vmin, h_vmin[s]);
            g.vmax = std::max(g.vmax, h_vmax[s]);
            g.n_conv += 1;
            if (h_vmax[s] > a->ub_v) g.n_over += 1;
            if (h_vmin[s] < a->lb_v) g.n_under += 1;
        } else {
            g.n_nonconv += 1;
            ++n_nonconv;
        }
    }
    g.n_scen = B;
    if (agg) *agg = g;
    a->err = "outer iterations " + std::to_string(outer) + ", last boundary move " + std::to_string(h_last);
    return n_nonconv;
}
