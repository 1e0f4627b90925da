// fpf_multi.cpp -- one process driving n GPUs of a node (include/freedm_pf.h,
// "Multi-GPU study"): the scenario batch is cut into contiguous shards, one
// per device (shard_range of freedm_amd/dist.py), every device solves its
// shard on its own stream with its own copy of the feeder tables, and the
// per-device batch aggregates are combined by RCCL over xGMI -- the path's
// only collective: one all-gather of every device's 8
// aggregate doubles, folded in device order on the host (fpf_aggregate_fold,
// the fold of the one-process-per-GPU form, dist.py: bit-identical aggregates).
// Per-scenario results never cross devices; they
// return to the caller's host arrays at their global scenario index.
//
// The reference caller is single-threaded C++ (VoltVarCtrl.cpp:1141 on the
// Broker's io_service thread, CBroker.cpp:582-612), so this is the form a
// Broker linking libfreedm_pf can use more than one GPU through -- from one
// host thread, so the devices only run concurrently if nothing in the issue
// loop blocks.  Copies to and from the caller's pageable arrays would (HIP
// completes them synchronously), so every transfer goes through pinned
// staging (hipHostMalloc) in chunks, double-buffered per device, in the order
// of multi_schedule(): chunk round r of every device is issued (host packing
// into its pinned slot, H2D, solve, D2H into the pinned slot; nothing waits)
// before round r - 1 of any device is collected (wait for its event, unpack
// into the caller's arrays).  The host packs device d + 1's chunk while device
// d computes, and unpacks round r - 1 while round r runs everywhere.
#include "../../include/freedm_pf.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

namespace {
// one chunk of one device: scenarios [lo, hi) of the batch, staging slot
struct Op {
    int kind;   // 0 = issue, 1 = collect
    int dev, slot;
    long lo, hi;
};

// The issue / collect order (see the file comment): shard of device d cut into
// chunks of at most `chunk` scenarios; round r issues chunk r of every device,
// then collects round r - 1; the last round is collected at the end.
std::vector<Op> multi_schedule(int n_gpus, long n_scen, long chunk) {
    std::vector<Op> ops;
    std::vector<long> lo(n_gpus), hi(n_gpus);
    long rounds = 0;
    for (int d = 0; d < n_gpus; ++d) {
        fpf_multi_shard(d, n_gpus, n_scen, &lo[d], &hi[d]);
        rounds = std::max(rounds, (hi[d] - lo[d] + chunk - 1) / chunk);
    }
    auto chunk_of = [&](int d, long r, long *a, long *b) {
        *a = lo[d] + r * chunk;
        *b = std::min(hi[d], *a + chunk);
        return *a < *b;
    };
    for (long r = 0; r <= rounds; ++r) {
        if (r < rounds)
            for (int d = 0; d < n_gpus; ++d) {
                long a, b;
                if (chunk_of(d, r, &a, &b)) ops.push_back({0, d, (int)(r & 1), a, b});
            }
        if (r >= 1)
            for (int d = 0; d < n_gpus; ++d) {
                long a, b;
                if (chunk_of(d, r - 1, &a, &b)) ops.push_back({1, d, (int)((r - 1) & 1), a, b});
            }
    }
    return ops;
}

long default_chunk() {
    const char *e = getenv("FPF_MULTI_CHUNK");   // experiments / tests
    const long c = e ? atol(e) : 0;
    return c > 0 ? c : 65536;
}
}  // namespace

struct fpf_multi {
    int n = 0;
    std::vector<fpf_ctx *> ctx;
    std::vector<fpf_feeder *> feeder;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    // per device: d_agg[8 + 8 n] = the shard's aggregate (8) | every device's, gathered
    // in device order (8 n) by the one collective
    std::vector<double *> d_agg;
    // per device: the shard's per-scenario scalars (the aggregate reads status /
    // loss / vmin / vmax; iters, errmx, guard as asked) and their pinned copy
    std::vector<char *> d_scal, h_scal;
    std::vector<size_t> scal_cap;
    // per device and slot: device staging (loads in, matrix outputs out) and its
    // pinned host twin, the event that marks the slot's D2H done
    std::vector<char *> d_slot[2], h_slot[2];
    std::vector<size_t> slot_cap[2];
    std::vector<hipEvent_t> ev[2];
    int nn = 0, nl = 0;
    int layout = FPF_LAYOUT_SCEN_FASTEST;   // fpf_opts.layout of the host arrays
    std::string err;
};

namespace {
int mfail(fpf_multi *m, int code, const std::string &msg) {
    if (m) m->err = msg;
    return code;
}
#define MHIP(m, expr)                                                                                 \
    do {                                                                                              \
        hipError_t e_ = (expr);                                                                       \
        if (e_ != hipSuccess) return mfail(m, FPF_ERR_HIP, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)
#define MNCCL(m, expr)                                                                                \
    do {                                                                                              \
        ncclResult_t r_ = (expr);                                                                     \
        if (r_ != ncclSuccess) return mfail(m, FPF_ERR_HIP, std::string(#expr ": ") + ncclGetErrorString(r_)); \
    } while (0)

// grow a device buffer and its pinned host twin to `bytes`
hipError_t grow(char **d, char **h, size_t *cap, size_t bytes) {
    if (bytes <= *cap) return hipSuccess;
    (void)hipFree(*d);
    (void)hipHostFree(*h);
    *d = *h = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc((void **)d, bytes);
    if (e == hipSuccess) e = hipHostMalloc((void **)h, bytes);
    if (e == hipSuccess) *cap = bytes;
    return e;
}
}  // namespace

extern "C" int fpf_multi_shard(int rank, int n_gpus, long n_total, long *lo, long *hi) {
    if (n_gpus < 1 || rank < 0 || rank >= n_gpus || n_total < 0 || !lo || !hi) return FPF_ERR_ARG;
    const long base = n_total / n_gpus, extra = n_total % n_gpus;
    *lo = rank * base + std::min<long>(rank, extra);
    *hi = *lo + base + (rank < extra ? 1 : 0);
    return FPF_OK;
}

extern "C" long fpf_multi_schedule(int n_gpus, long n_scen, long chunk, long *ops, long max_ops) {
    if (n_gpus < 1 || n_scen < 0 || chunk < 1 || (max_ops > 0 && !ops)) return FPF_ERR_ARG;
    const std::vector<Op> v = multi_schedule(n_gpus, n_scen, chunk);
    for (long i = 0; i < (long)v.size() && i < max_ops; ++i) {
        ops[4 * i + 0] = v[i].kind;
        ops[4 * i + 1] = v[i].dev;
        ops[4 * i + 2] = v[i].lo;
        ops[4 * i + 3] = v[i].hi;
    }
    return (long)v.size();
}

// collective calls fpf_multi_solve has issued in this process (one per solve)
static std::atomic<long> g_multi_collectives{0};
extern "C" long fpf_multi_collectives(void) { return g_multi_collectives.load(); }

extern "C" void fpf_aggregate_fold(const fpf_aggregate *parts, int n, fpf_aggregate *out) {
    if (!out) return;
    fpf_aggregate a;
    std::memset(&a, 0, sizeof(a));
    a.vmin = INFINITY;
    a.vmax = -INFINITY;
    for (int i = 0; parts && i < n; ++i) {
        const fpf_aggregate &p = parts[i];
        a.loss_sum += p.loss_sum;
        a.vmin = std::min(a.vmin, p.vmin);
        a.vmax = std::max(a.vmax, p.vmax);
        a.n_conv += p.n_conv;
        a.n_nonconv += p.n_nonconv;
        a.n_over += p.n_over;
        a.n_under += p.n_under;
        a.n_scen += p.n_scen;
    }
    *out = a;
}

extern "C" void fpf_multi_destroy(fpf_multi *m) {
    if (!m) return;
    for (int d = 0; d < m->n; ++d) {
        if (d < (int)m->comm.size() && m->comm[d]) (void)ncclCommDestroy(m->comm[d]);
        (void)hipSetDevice(d);
        if (d < (int)m->d_agg.size()) (void)hipFree(m->d_agg[d]);
        if (d < (int)m->d_scal.size()) (void)hipFree(m->d_scal[d]);
        if (d < (int)m->h_scal.size()) (void)hipHostFree(m->h_scal[d]);
        for (int k = 0; k < 2; ++k) {
            if (d < (int)m->d_slot[k].size()) (void)hipFree(m->d_slot[k][d]);
            if (d < (int)m->h_slot[k].size()) (void)hipHostFree(m->h_slot[k][d]);
            if (d < (int)m->ev[k].size() && m->ev[k][d]) (void)hipEventDestroy(m->ev[k][d]);
        }
        if (d < (int)m->stream.size() && m->stream[d]) (void)hipStreamDestroy(m->stream[d]);
        if (d < (int)m->feeder.size()) fpf_feeder_destroy(m->feeder[d]);
        if (d < (int)m->ctx.size()) fpf_ctx_destroy(m->ctx[d]);
    }
    delete m;
}

// why the calling thread's last fpf_multi_create failed (there is no handle to carry it)
static thread_local std::string g_create_err = "no error";

extern "C" const char *fpf_multi_last_error(const fpf_multi *m) { return m ? m->err.c_str() : g_create_err.c_str(); }

extern "C" int fpf_multi_create(int n_gpus, const double *dl, int nl, int ncols, const double *z, int z_rows,
                                int z_cols, const fpf_opts *opts, fpf_multi **out) {
    if (!out || n_gpus < 1) {
        g_create_err = "fpf_multi_create: out is NULL or n_gpus < 1";
        return FPF_ERR_ARG;
    }
    *out = nullptr;
    int avail = 0;
    if (hipGetDeviceCount(&avail) != hipSuccess || avail < n_gpus) {
        g_create_err = "fpf_multi_create: " + std::to_string(n_gpus) + " devices requested, " + std::to_string(avail) +
                       " visible";
        return FPF_ERR_ARG;
    }
    fpf_multi *m = new fpf_multi();
    m->n = n_gpus;
    m->ctx.assign(n_gpus, nullptr);
    m->feeder.assign(n_gpus, nullptr);
    m->comm.assign(n_gpus, nullptr);
    m->stream.assign(n_gpus, nullptr);
    m->d_agg.assign(n_gpus, nullptr);
    m->d_scal.assign(n_gpus, nullptr);
    m->h_scal.assign(n_gpus, nullptr);
    m->scal_cap.assign(n_gpus, 0);
    for (int k = 0; k < 2; ++k) {
        m->d_slot[k].assign(n_gpus, nullptr);
        m->h_slot[k].assign(n_gpus, nullptr);
        m->slot_cap[k].assign(n_gpus, 0);
        m->ev[k].assign(n_gpus, nullptr);
    }
    for (int d = 0; d < n_gpus; ++d) {
        int rc = fpf_ctx_create(d, &m->ctx[d]);
        if (rc == FPF_OK) rc = fpf_feeder_create(m->ctx[d], dl, nl, ncols, z, z_rows, z_cols, opts, &m->feeder[d]);
        if (rc != FPF_OK) {
            g_create_err = "fpf_multi_create: device " + std::to_string(d) + ": " +
                           (m->ctx[d] ? fpf_last_error(m->ctx[d]) : "context creation failed");
            fpf_multi_destroy(m);
            return rc;
        }
        if (hipSetDevice(d) != hipSuccess || hipStreamCreateWithFlags(&m->stream[d], hipStreamNonBlocking) != hipSuccess ||
            hipMalloc(&m->d_agg[d], (8 + 8 * (size_t)n_gpus) * sizeof(double)) != hipSuccess ||
            hipEventCreateWithFlags(&m->ev[0][d], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&m->ev[1][d], hipEventDisableTiming) != hipSuccess) {
            g_create_err = "fpf_multi_create: device " + std::to_string(d) + ": stream / buffer allocation failed";
            fpf_multi_destroy(m);
            return FPF_ERR_HIP;
        }
    }
    std::vector<int> devs(n_gpus);
    for (int d = 0; d < n_gpus; ++d) devs[d] = d;
    if (const ncclResult_t nr = ncclCommInitAll(m->comm.data(), n_gpus, devs.data()); nr != ncclSuccess) {
        g_create_err = std::string("fpf_multi_create: ncclCommInitAll: ") + ncclGetErrorString(nr);
        m->comm.assign(n_gpus, nullptr);
        fpf_multi_destroy(m);
        return FPF_ERR_HIP;
    }
    fpf_feeder_info in;
    fpf_feeder_get_info(m->feeder[0], &in);
    m->nn = in.nn;
    m->nl = in.nl;
    m->layout = opts ? opts->layout : FPF_LAYOUT_SCEN_FASTEST;
    g_create_err = "no error";
    *out = m;
    return FPF_OK;
}

extern "C" int fpf_multi_get_feeder(fpf_multi *m, int device, fpf_feeder **out) {
    if (!m || !out || device < 0 || device >= m->n) return FPF_ERR_ARG;
    *out = m->feeder[device];
    return FPF_OK;
}

// Every pointer of `out` and pq is host memory laid out for the whole batch
// ([rows][n_scen], or [n_scen][rows] scenario-major); device d handles the
// scenarios [lo_d, hi_d) of multi_schedule's chunks.
extern "C" int fpf_multi_solve(fpf_multi *m, int n_scen, const double *pq, const fpf_outputs *out,
                               fpf_aggregate *agg) {
    if (!m || n_scen < 0 || (n_scen > 0 && !pq)) return mfail(m, FPF_ERR_ARG, "fpf_multi_solve: bad arguments");
    fpf_outputs none;
    std::memset(&none, 0, sizeof(none));
    const fpf_outputs &u = out ? *out : none;
    const size_t B = (size_t)n_scen, nn = (size_t)m->nn, nl = (size_t)m->nl;
    const bool smaj = m->layout == FPF_LAYOUT_SCEN_MAJOR;
    // matrix outputs (chunked through the slots): host pointer, rows per scenario
    struct Mat { double *host; size_t rows; };
    const Mat mats[5] = {{u.vpolar, 6 * nn}, {u.pqb, 6 * nn}, {u.pql, 6 * nn}, {u.v_re, 3 * nn}, {u.v_im, 3 * nn}};
    // per-scenario scalars (device-resident for the shard): host pointer, element bytes;
    // status / loss / vmin / vmax always (the shard's aggregate reads them)
    struct Scal { void *host; size_t esz; };
    const Scal scal[7] = {{u.iters, 4}, {u.status, 1}, {u.loss, 8}, {u.vmin, 8}, {u.vmax, 8}, {u.errmx, 8}, {u.guard, 1}};
    const bool need_scal[7] = {u.iters != nullptr, true, true, true, true, u.errmx != nullptr, u.guard != nullptr};
    const long chunk = default_chunk();
    const size_t CH = (size_t)std::min<long>(chunk, std::max(1, n_scen));
    // slot layout: loads [CH][6 Nl] | each requested matrix output [CH][rows]
    size_t moff[6], slot_bytes = ((6 * nl * CH * 8) + 255) & ~(size_t)255;
    for (int i = 0; i < 5; ++i) {
        moff[i] = slot_bytes;
        if (mats[i].host) slot_bytes += (mats[i].rows * CH * 8 + 255) & ~(size_t)255;
    }
    std::vector<long> lo(m->n), hi(m->n);
    std::vector<size_t> soff(8);
    for (int d = 0; d < m->n; ++d) fpf_multi_shard(d, m->n, n_scen, &lo[d], &hi[d]);
    // scalar block per device: each array [shard], 256-byte aligned
    auto scal_layout = [&](size_t nd) {
        size_t t = 0;
        for (int i = 0; i < 7; ++i) {
            soff[i] = t;
            if (need_scal[i]) t += (scal[i].esz * std::max<size_t>(nd, 1) + 255) & ~(size_t)255;
        }
        soff[7] = t;
        return t;
    };
    static const double ident[8] = {0.0, INFINITY, -INFINITY, 0, 0, 0, 0, 0};
    for (int d = 0; d < m->n; ++d) {
        MHIP(m, hipSetDevice(d));
        const size_t nd = (size_t)(hi[d] - lo[d]);
        const size_t sb = scal_layout(nd);
        if (sb > m->scal_cap[d]) {
            (void)hipFree(m->d_scal[d]);
            (void)hipHostFree(m->h_scal[d]);
            m->d_scal[d] = m->h_scal[d] = nullptr;
            m->scal_cap[d] = 0;
            MHIP(m, hipMalloc((void **)&m->d_scal[d], sb));
            MHIP(m, hipHostMalloc((void **)&m->h_scal[d], sb));
            m->scal_cap[d] = sb;
        }
        for (int k = 0; k < 2; ++k) MHIP(m, grow(&m->d_slot[k][d], &m->h_slot[k][d], &m->slot_cap[k][d], slot_bytes));
        if (nd > 0) {
            const int rc = fpf_feeder_reserve(m->feeder[d], (int)std::min(nd, CH));
            if (rc < 0) return mfail(m, rc, std::string("device ") + std::to_string(d) + ": " + fpf_last_error(m->ctx[d]));
        }
    }
    // scenarios [a, b) of a [rows][B] (or [B][rows]) host array <-> a packed [rows][b - a]
    // (or [b - a][rows]) chunk
    auto pack = [&](double *dst, const double *src, size_t rows, long a, long b) {
        const size_t n = (size_t)(b - a);
        if (smaj) std::memcpy(dst, src + (size_t)a * rows, n * rows * 8);
        else
            for (size_t r = 0; r < rows; ++r) std::memcpy(dst + r * n, src + r * B + a, n * 8);
    };
    auto unpack = [&](double *dst, const double *src, size_t rows, long a, long b) {
        const size_t n = (size_t)(b - a);
        if (smaj) std::memcpy(dst + (size_t)a * rows, src, n * rows * 8);
        else
            for (size_t r = 0; r < rows; ++r) std::memcpy(dst + r * B + a, src + r * n, n * 8);
    };
    for (const Op &op : multi_schedule(m->n, n_scen, (long)CH)) {
        const int d = op.dev, k = op.slot;
        const size_t n = (size_t)(op.hi - op.lo), off = (size_t)(op.lo - lo[d]);
        char *ds = m->d_slot[k][d], *hs = m->h_slot[k][d];
        MHIP(m, hipSetDevice(d));
        hipStream_t st = m->stream[d];
        if (op.kind == 0) {
            // issue: pack the loads into the pinned slot, copy in, solve, copy the matrix
            // outputs back into the pinned slot, mark the slot; nothing here waits
            pack((double *)hs, pq, 6 * nl, op.lo, op.hi);
            MHIP(m, hipMemcpyAsync(ds, hs, 6 * nl * n * 8, hipMemcpyHostToDevice, st));
            fpf_outputs o;
            std::memset(&o, 0, sizeof(o));
            double **mp[5] = {&o.vpolar, &o.pqb, &o.pql, &o.v_re, &o.v_im};
            for (int i = 0; i < 5; ++i)
                if (mats[i].host) *mp[i] = (double *)(ds + moff[i]);
            char *sc = m->d_scal[d];
            if (need_scal[0]) o.iters = (int *)(sc + soff[0]) + off;
            o.status = (signed char *)(sc + soff[1]) + off;
            o.loss = (double *)(sc + soff[2]) + off;
            o.vmin = (double *)(sc + soff[3]) + off;
            o.vmax = (double *)(sc + soff[4]) + off;
            if (need_scal[5]) o.errmx = (double *)(sc + soff[5]) + off;
            if (need_scal[6]) o.guard = (signed char *)(sc + soff[6]) + off;
            // a shard of one chunk takes its aggregate from the solve itself (the same
            // reduction as fpf_solve_batch); longer shards reduce their scalars at the end
            const bool whole = op.lo == lo[d] && op.hi == hi[d];
            const int rc = fpf_solve_batch_device(m->feeder[d], (int)n, (const double *)ds, &o, whole ? m->d_agg[d] : nullptr,
                                                  (void *)st);
            if (rc < 0) return mfail(m, rc, std::string("device ") + std::to_string(d) + ": " + fpf_last_error(m->ctx[d]));
            for (int i = 0; i < 5; ++i)
                if (mats[i].host)
                    MHIP(m, hipMemcpyAsync(hs + moff[i], ds + moff[i], mats[i].rows * n * 8, hipMemcpyDeviceToHost, st));
            MHIP(m, hipEventRecord(m->ev[k][d], st));
        } else {
            // collect: the slot's outputs into the caller's arrays
            MHIP(m, hipEventSynchronize(m->ev[k][d]));
            for (int i = 0; i < 5; ++i)
                if (mats[i].host) unpack(mats[i].host, (const double *)(hs + moff[i]), mats[i].rows, op.lo, op.hi);
        }
    }
    // per device: the shard's aggregate over its scalars, the scalars back (pinned)
    for (int d = 0; d < m->n; ++d) {
        MHIP(m, hipSetDevice(d));
        hipStream_t st = m->stream[d];
        const size_t nd = (size_t)(hi[d] - lo[d]);
        scal_layout(nd);
        if (nd == 0) {   // an empty shard still joins the all-gather, with the identity
            MHIP(m, hipMemcpyAsync(m->d_agg[d], ident, sizeof(ident), hipMemcpyHostToDevice, st));
            continue;
        }
        char *sc = m->d_scal[d];
        if (nd > CH) {
            const int rc = fpf_aggregate_device(m->feeder[d], (int)nd, (const signed char *)(sc + soff[1]),
                                                (const double *)(sc + soff[2]), (const double *)(sc + soff[3]),
                                                (const double *)(sc + soff[4]), m->d_agg[d], (void *)st);
            if (rc < 0) return mfail(m, rc, std::string("device ") + std::to_string(d) + ": " + fpf_last_error(m->ctx[d]));
        }
        MHIP(m, hipMemcpyAsync(m->h_scal[d], sc, soff[7], hipMemcpyDeviceToHost, st));
    }
    // the one collective: an all-gather of every device's 8-double aggregate (one
    // ncclAllGather per communicator rank, grouped), folded on the host in device
    // order by fpf_aggregate_fold -- the same rows and the same fold as the
    // one-process-per-GPU form (dist.py: gather_aggregates + fold_aggregates), so
    // the two forms give bit-identical aggregates
    MNCCL(m, ncclGroupStart());
    for (int d = 0; d < m->n; ++d) {
        MHIP(m, hipSetDevice(d));
        MNCCL(m, ncclAllGather(m->d_agg[d], m->d_agg[d] + 8, 8, ncclDouble, m->comm[d], m->stream[d]));
    }
    MNCCL(m, ncclGroupEnd());
    g_multi_collectives.fetch_add(1);
    std::vector<fpf_aggregate> rows((size_t)m->n);
    MHIP(m, hipSetDevice(0));
    MHIP(m, hipMemcpyAsync(rows.data(), m->d_agg[0] + 8, 8 * sizeof(double) * (size_t)m->n, hipMemcpyDeviceToHost,
                           m->stream[0]));
    for (int d = 0; d < m->n; ++d) {
        MHIP(m, hipSetDevice(d));
        MHIP(m, hipStreamSynchronize(m->stream[d]));
        const size_t nd = (size_t)(hi[d] - lo[d]);
        scal_layout(nd);
        for (int i = 0; i < 7; ++i)
            if (scal[i].host && nd > 0)
                std::memcpy((char *)scal[i].host + (size_t)lo[d] * scal[i].esz, m->h_scal[d] + soff[i], nd * scal[i].esz);
    }
    for (int d = 0; d < m->n; ++d) {   // a paired-kernel exchange that gave up (FPF_EXCHANGE_FAILED)
        const int fr = fpf_feeder_check(m->feeder[d], (void *)m->stream[d]);
        if (fr) return mfail(m, fr, std::string("device ") + std::to_string(d) + ": " + fpf_last_error(m->ctx[d]));
    }
    fpf_aggregate a;
    fpf_aggregate_fold(rows.data(), m->n, &a);
    if (agg) *agg = a;
    return (int)a.n_nonconv;
}
