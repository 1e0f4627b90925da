/*
 * fpf_broker.h -- the Broker-side glue core for libfreedm_pf (C++98, header
 * only, no Armadillo): what Broker/src/vvc/DPF_hip.cpp wraps.
 *
 * Replaces, in the FREEDM DGI Broker (vmuthuk2/FREEDM):
 *   VPQ DPF_return7(arma::mat Dl, arma::cx_mat Z)   Broker/src/vvc/fun_return.h:53,
 *                                                  defined DPF_return7.cpp:8-263
 * and adds the batched form DPF_batch the VVC line search needs
 * (VoltVarCtrl.cpp:1330-1542: every step is an independent DPF).
 *
 * Everything is plain column-major double buffers -- an arma::mat's memptr()
 * -- so the Armadillo-facing wrapper (DPF_hip.cpp) is a few lines of
 * marshalling.  Compiles with g++ -std=c++98 -pedantic (the Broker's flags,
 * Broker/CMakeLists.txt:55); tests/test_integration.py builds it that way and
 * runs it on the GPU against the oracle.
 *
 * Errors: the reference throws std::logic_error out of Armadillo where a
 * feeder is malformed or a solve does not converge (DPF_return7.cpp:100-101,
 * 242); the glue throws the same type at the same points, and
 * std::runtime_error for a HIP failure (the reference has none).
 * Threading: one Engine per thread (the Broker calls from its single
 * io_service thread, CBroker.cpp:582-612).
 */
#ifndef FPF_BROKER_H
#define FPF_BROKER_H

#include <freedm_pf.h>

#include <cstring>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

namespace fpf_broker {

/* One DPF_return7 result (fun_return.h:43-51): Nn x 6 column-major matrices,
 * row 0 = substation (DPF_return7.cpp:236-252 order). */
struct Vpq {
    int nn;
    std::vector<double> vpolar, pqb, pql;
    int iters;
    bool converged;
    double loss, vmin, vmax;   /* the VVC reductions (VoltVarCtrl.cpp:1152-1161, 1201-1207) */
};

class Engine {
public:
    /* exact = 1: the reference's roundings (bit-identical V / PQb / PQL);
       0: fast mode (1e-10 on V, same iteration counts) */
    explicit Engine(int device = 0, int exact = 1)
        : ctx_(0), feeder_(0), nl_(0), ncols_(0), z_rows_(0), z_cols_(0), log_(0) {
        if (fpf_ctx_create(device, &ctx_) != FPF_OK) throw std::runtime_error("libfreedm_pf: no HIP device");
        fpf_opts_default(&opts_);
        opts_.exact = exact;
        std::memset(&info_, 0, sizeof(info_));
    }
    ~Engine() {
        fpf_feeder_destroy(feeder_);
        fpf_ctx_destroy(ctx_);
    }

    /* The device feeder for Dl's topology (columns 0..5) and Z (complex,
       interleaved re/im, column-major): uploaded on first use and again only
       when the topology or Z change -- the loads (columns 6..11) travel per call. */
    fpf_feeder *feeder(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols) {
        const size_t zn = (size_t)2 * z_rows * z_cols;
        if (feeder_ && nl == nl_ && ncols == ncols_ && z_rows == z_rows_ && z_cols == z_cols_ &&
            std::memcmp(dl, &topo_[0], sizeof(double) * 6 * nl) == 0 &&
            (zn == 0 || std::memcmp(z, &z_[0], sizeof(double) * zn) == 0))
            return feeder_;
        fpf_feeder_destroy(feeder_);
        feeder_ = 0;
        if (fpf_feeder_create(ctx_, dl, nl, ncols, z, z_rows, z_cols, &opts_, &feeder_) != FPF_OK)
            throw std::logic_error(std::string("DPF_return7: ") + fpf_last_error(ctx_));   /* Armadillo throws here */
        topo_.assign(dl, dl + (size_t)6 * nl);
        z_.assign(z, z + zn);
        nl_ = nl;
        ncols_ = ncols;
        z_rows_ = z_rows;
        z_cols_ = z_cols;
        fpf_feeder_get_info(feeder_, &info_);
        return feeder_;
    }

    const fpf_feeder_info &info() const { return info_; }

    /* The reference's console lines (DPF_return7.cpp:38 "Run DPF on <Nn> Nodes
       System" and :206 " DPF converged!") per solved scenario, in the order K
       sequential calls would print them (0: silent, the default here;
       Broker/src/vvc/DPF_hip.cpp sets std::cout, as the reference prints). */
    void set_log(std::ostream *os) { log_ = os; }
    const char *last_error() const { return fpf_last_error(ctx_); }

    /* DPF_return7(Dl, Z): one scenario; throws std::logic_error where the
       reference would (no convergence within mxitr sweeps). */
    Vpq dpf_return7(const double *dl, int nl, int ncols, const double *z, int z_rows, int z_cols) {
        std::vector<const double *> one(1, dl);
        std::vector<Vpq> r = dpf_batch(one, nl, ncols, z, z_rows, z_cols, true);
        return r[0];
    }

    /* DPF_batch: K Dl tables that share one topology and Z (the candidates of
       the line search), solved as ONE batch.  Each Dl must match dls[0] in
       columns 0..5.  throw_nonconv: throw like K sequential DPF_return7 calls
       would at the first non-converged one; otherwise report it in Vpq. */
    std::vector<Vpq> dpf_batch(const std::vector<const double *> &dls, int nl, int ncols, const double *z,
                               int z_rows, int z_cols, bool throw_nonconv) {
        const int K = (int)dls.size();
        std::vector<Vpq> out(K);
        if (K == 0) return out;
        fpf_feeder *f = feeder(dls[0], nl, ncols, z, z_rows, z_cols);
        for (int s = 1; s < K; ++s)
            if (std::memcmp(dls[s], dls[0], sizeof(double) * 6 * nl) != 0)
                throw std::invalid_argument("DPF_batch: every Dl must share the topology columns 0..5");
        const int nn = info_.nn;
        /* [6][Nl][K] scenario fastest: field c of row j of scenario s = Dl_s(j, 6 + c) */
        std::vector<double> pq((size_t)6 * nl * K);
        for (int s = 0; s < K; ++s)
            for (int c = 0; c < 6; ++c)
                for (int j = 0; j < nl; ++j) pq[((size_t)c * nl + j) * K + s] = dls[s][(size_t)(6 + c) * nl + j];
        std::vector<double> vp((size_t)6 * nn * K), pb((size_t)6 * nn * K), pl((size_t)6 * nn * K);
        std::vector<double> loss(K), vmin(K), vmax(K);
        std::vector<int> iters(K);
        std::vector<signed char> status(K);
        fpf_outputs o;
        std::memset(&o, 0, sizeof(o));
        o.vpolar = &vp[0];
        o.pqb = &pb[0];
        o.pql = &pl[0];
        o.iters = &iters[0];
        o.status = &status[0];
        o.loss = &loss[0];
        o.vmin = &vmin[0];
        o.vmax = &vmax[0];
        const int rc = fpf_solve_batch(f, K, &pq[0], &o, 0);
        if (rc < 0) throw std::runtime_error(std::string("libfreedm_pf: ") + fpf_last_error(ctx_));
        for (int s = 0; s < K; ++s) {
            if (log_) *log_ << "Run DPF on " << nn << " Nodes System" << std::endl;
            /* (a non-converged solve prints nothing more: the reference's :210 test
               i >= mxitr is never true inside its loop, and :242 throws) */
            if (throw_nonconv && status[s] != FPF_CONVERGED)
                throw std::logic_error("DPF_return7: no convergence");   /* DPF_return7.cpp:100-101,242 */
            if (log_ && status[s] == FPF_CONVERGED) *log_ << " DPF converged!" << std::endl;
            Vpq &r = out[s];
            r.nn = nn;
            r.vpolar.resize((size_t)6 * nn);
            r.pqb.resize((size_t)6 * nn);
            r.pql.resize((size_t)6 * nn);
            /* [col][row][K] -> column-major Nn x 6 */
            for (int c = 0; c < 6; ++c)
                for (int k = 0; k < nn; ++k) {
                    const size_t src = ((size_t)c * nn + k) * K + s, dst = (size_t)c * nn + k;
                    r.vpolar[dst] = vp[src];
                    r.pqb[dst] = pb[src];
                    r.pql[dst] = pl[src];
                }
            r.iters = iters[s];
            r.converged = status[s] == FPF_CONVERGED;
            r.loss = loss[s];
            r.vmin = vmin[s];
            r.vmax = vmax[s];
        }
        return out;
    }

private:
    Engine(const Engine &);
    Engine &operator=(const Engine &);
    fpf_ctx *ctx_;
    fpf_feeder *feeder_;
    fpf_opts opts_;
    fpf_feeder_info info_;
    std::vector<double> topo_, z_;
    int nl_, ncols_, z_rows_, z_cols_;
    std::ostream *log_;
};

}  // namespace fpf_broker

#endif /* FPF_BROKER_H */
