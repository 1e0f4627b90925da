// fpf_multi.cpp -- one process driving n GPUs of a node (include/freedm_pf.h,
// "Multi-GPU study"): the scenario batch is cut into contiguous shards, one
// per device (shard_range of freedm_amd/dist.py), every device solves its
// shard on its own stream with its own copy of the feeder tables, and the
// per-device batch aggregates are combined by RCCL over xGMI -- the path's
// only collective: a sum of the 8 aggregate doubles, a min
// of vmin and a max of vmax.  Per-scenario results never cross devices; they
// return to the caller's host arrays at their global scenario index.
//
// The reference caller is single-threaded C++ (VoltVarCtrl.cpp:1141 on the
// Broker's io_service thread, CBroker.cpp:582-612), so this is the form a
// Broker linking libfreedm_pf can use more than one GPU through.
#include "../../include/freedm_pf.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>
#include <vector>

struct fpf_multi {
    int n = 0;
    std::vector<fpf_ctx *> ctx;
    std::vector<fpf_feeder *> feeder;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> stream;
    // per device: d_agg[16] = aggregate (8) | summed (8); d_mm[4] = vmin, vmax reduced
    std::vector<double *> d_agg;
    std::vector<char *> d_stage;
    std::vector<size_t> stage_bytes;
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
}  // namespace

extern "C" int fpf_multi_shard(int rank, int n_gpus, long n_total, long *lo, long *hi) {
    if (n_gpus < 1 || rank < 0 || rank >= n_gpus || n_total < 0 || !lo || !hi) return FPF_ERR_ARG;
    const long base = n_total / n_gpus, extra = n_total % n_gpus;
    *lo = rank * base + std::min<long>(rank, extra);
    *hi = *lo + base + (rank < extra ? 1 : 0);
    return FPF_OK;
}

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
        if (d < (int)m->d_stage.size()) (void)hipFree(m->d_stage[d]);
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
    m->d_stage.assign(n_gpus, nullptr);
    m->stage_bytes.assign(n_gpus, 0);
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
            hipMalloc(&m->d_agg[d], 20 * sizeof(double)) != hipSuccess) {
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

// Every pointer of `out` and pq is host memory laid out for the whole batch;
// device d reads and writes scenarios [lo_d, hi_d) of it: the columns of
// [field][row][n_scen] (2-D copies) or one contiguous block of
// [n_scen][field][row] (the scenario-major layout).
extern "C" int fpf_multi_solve(fpf_multi *m, int n_scen, const double *pq, const fpf_outputs *out,
                               fpf_aggregate *agg) {
    if (!m || n_scen < 0 || (n_scen > 0 && !pq)) return mfail(m, FPF_ERR_ARG, "fpf_multi_solve: bad arguments");
    fpf_outputs none;
    std::memset(&none, 0, sizeof(none));
    const fpf_outputs &u = out ? *out : none;
    const size_t B = (size_t)n_scen, nn = (size_t)m->nn, nl = (size_t)m->nl;
    // matrix outputs: (host pointer, rows = fields * rows-per-field, element bytes)
    struct Mat { void *host; size_t rows, esz; };
    const Mat mats[10] = {{u.vpolar, 6 * nn, 8}, {u.pqb, 6 * nn, 8}, {u.pql, 6 * nn, 8}, {u.v_re, 3 * nn, 8},
                          {u.v_im, 3 * nn, 8},  {u.iters, 1, 4},     {u.status, 1, 1},  {u.loss, 1, 8},
                          {u.vmin, 1, 8},       {u.vmax, 1, 8}};
    static const double ident[8] = {0.0, INFINITY, -INFINITY, 0, 0, 0, 0, 0};
    for (int d = 0; d < m->n; ++d) {
        long lo = 0, hi = 0;
        fpf_multi_shard(d, m->n, n_scen, &lo, &hi);
        const size_t nd = (size_t)(hi - lo);
        MHIP(m, hipSetDevice(d));
        hipStream_t st = m->stream[d];
        if (nd == 0) {   // an empty shard still joins the all-reduce, with the identity
            MHIP(m, hipMemcpyAsync(m->d_agg[d], ident, sizeof(ident), hipMemcpyHostToDevice, st));
            continue;
        }
        // staging: pq slice, then each requested output, 256-byte aligned
        size_t offs[11], total = 0;
        offs[0] = 0;
        total = (6 * nl * nd * 8 + 255) & ~(size_t)255;
        for (int i = 0; i < 10; ++i) {
            offs[i + 1] = total;
            if (mats[i].host) total += (mats[i].rows * nd * mats[i].esz + 255) & ~(size_t)255;
        }
        if (total > m->stage_bytes[d]) {
            (void)hipFree(m->d_stage[d]);
            m->d_stage[d] = nullptr;
            m->stage_bytes[d] = 0;
            MHIP(m, hipMalloc(&m->d_stage[d], total));
            m->stage_bytes[d] = total;
        }
        char *sb = m->d_stage[d];
        // scenarios [lo, lo + nd) of a [rows][B] (or, scenario-major, [B][rows]) host array
        auto copy = [&](void *dst, const void *src, size_t rows, size_t esz, hipMemcpyKind kind, bool to_host) {
            if (m->layout == FPF_LAYOUT_SCEN_MAJOR || rows == 1) {
                const size_t off = (size_t)lo * rows * esz, n = nd * rows * esz;
                return to_host ? hipMemcpyAsync((char *)dst + off, src, n, kind, st)
                               : hipMemcpyAsync(dst, (const char *)src + off, n, kind, st);
            }
            return to_host ? hipMemcpy2DAsync((char *)dst + lo * esz, B * esz, src, nd * esz, nd * esz, rows, kind, st)
                           : hipMemcpy2DAsync(dst, nd * esz, (const char *)src + lo * esz, B * esz, nd * esz, rows, kind, st);
        };
        MHIP(m, copy(sb, pq, 6 * nl, 8, hipMemcpyHostToDevice, false));
        void *dp[10];
        for (int i = 0; i < 10; ++i) dp[i] = mats[i].host ? (void *)(sb + offs[i + 1]) : nullptr;
        fpf_outputs o;
        o.vpolar = (double *)dp[0];
        o.pqb = (double *)dp[1];
        o.pql = (double *)dp[2];
        o.v_re = (double *)dp[3];
        o.v_im = (double *)dp[4];
        o.iters = (int *)dp[5];
        o.status = (signed char *)dp[6];
        o.loss = (double *)dp[7];
        o.vmin = (double *)dp[8];
        o.vmax = (double *)dp[9];
        const int rc = fpf_solve_batch_device(m->feeder[d], (int)nd, (const double *)sb, &o, m->d_agg[d], (void *)st);
        if (rc < 0) return mfail(m, rc, std::string("device ") + std::to_string(d) + ": " + fpf_last_error(m->ctx[d]));
        for (int i = 0; i < 10; ++i)
            if (mats[i].host) MHIP(m, copy(mats[i].host, dp[i], mats[i].rows, mats[i].esz, hipMemcpyDeviceToHost, true));
    }
    // the one collective: [loss_sum .. n_scen] summed, vmin min'd, vmax max'd
    MNCCL(m, ncclGroupStart());
    for (int d = 0; d < m->n; ++d) {
        MHIP(m, hipSetDevice(d));
        MNCCL(m, ncclAllReduce(m->d_agg[d], m->d_agg[d] + 8, 8, ncclDouble, ncclSum, m->comm[d], m->stream[d]));
        MNCCL(m, ncclAllReduce(m->d_agg[d] + 1, m->d_agg[d] + 16, 1, ncclDouble, ncclMin, m->comm[d], m->stream[d]));
        MNCCL(m, ncclAllReduce(m->d_agg[d] + 2, m->d_agg[d] + 17, 1, ncclDouble, ncclMax, m->comm[d], m->stream[d]));
    }
    MNCCL(m, ncclGroupEnd());
    double h[20];
    MHIP(m, hipSetDevice(0));
    MHIP(m, hipMemcpyAsync(h, m->d_agg[0], sizeof(h), hipMemcpyDeviceToHost, m->stream[0]));
    for (int d = 0; d < m->n; ++d) {
        MHIP(m, hipSetDevice(d));
        MHIP(m, hipStreamSynchronize(m->stream[d]));
    }
    fpf_aggregate a;
    a.loss_sum = h[8];
    a.vmin = h[16];
    a.vmax = h[17];
    a.n_conv = h[11];
    a.n_nonconv = h[12];
    a.n_over = h[13];
    a.n_under = h[14];
    a.n_scen = h[15];
    if (agg) *agg = a;
    return (int)a.n_nonconv;
}
