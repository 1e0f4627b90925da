// Broker/src/vvc/DPF_hip.cpp -- DPF_return7 on libfreedm_pf (C++98, in the Broker tree).
//
// Replaces Broker/src/vvc/DPF_return7.cpp in BROKER_FILES (Broker/src/CMakeLists.txt:29-47);
// same declaration (fun_return.h:53), same VPQ record (fun_return.h:43-51), same
// std::logic_error where the reference's Armadillo code throws.  Adds DPF_batch for
// the VVC step-size search (VoltVarCtrl.cpp:1330-1542): its 2m+1 sequential
// DPF_return7 calls become one batched solve.  The marshalling lives in
// fpf_broker.h (no Armadillo), which tests/test_integration.py compiles as C++98
// and runs on the GPU; this file only moves arma::mat memory in and out and
// needs the Broker's Armadillo to build (not present in this repository's image).
#include "fun_return_hip.h"   // fun_return.h + the DPF_batch declaration

#include <iostream>
#include <vector>

#include "fpf_broker.h"

namespace {
fpf_broker::Engine &engine() {
    static fpf_broker::Engine e(0, 1);   // device 0, exact mode: the reference's roundings
    static bool init = false;
    if (!init) {
        e.set_log(&std::cout);           // DPF_return7.cpp:38,206 print on every call
        init = true;
    }
    return e;
}

VPQ to_vpq(const fpf_broker::Vpq &r, const arma::mat &Dl) {
    VPQ v;
    v.Vpolar = arma::mat(&r.vpolar[0], r.nn, 6);
    v.PQb = arma::mat(&r.pqb[0], r.nn, 6);
    v.PQL = arma::mat(&r.pql[0], r.nn, 6);
    v.Qset_a = Dl.col(7);   // DPF_return7.cpp:259-261
    v.Qset_b = Dl.col(9);
    v.Qset_c = Dl.col(11);
    return v;               // Ib / IL are declared but never set by the reference either
}
}  // namespace

VPQ DPF_return7(arma::mat Dl, arma::cx_mat Z) {
    const fpf_broker::Vpq r = engine().dpf_return7(Dl.memptr(), (int)Dl.n_rows, (int)Dl.n_cols,
                                                   reinterpret_cast<const double *>(Z.memptr()),
                                                   (int)Z.n_rows, (int)Z.n_cols);
    return to_vpq(r, Dl);
}

// K candidate Dl tables of one topology as one batch (each result as DPF_return7
// would return it); throws at the first non-converged candidate like K
// sequential calls would.
std::vector<VPQ> DPF_batch(const std::vector<arma::mat> &Dls, const arma::cx_mat &Z) {
    std::vector<const double *> ptrs;
    for (size_t s = 0; s < Dls.size(); ++s) ptrs.push_back(Dls[s].memptr());
    std::vector<VPQ> out;
    if (Dls.empty()) return out;
    const std::vector<fpf_broker::Vpq> r =
        engine().dpf_batch(ptrs, (int)Dls[0].n_rows, (int)Dls[0].n_cols, reinterpret_cast<const double *>(Z.memptr()),
                           (int)Z.n_rows, (int)Z.n_cols, true);
    for (size_t s = 0; s < r.size(); ++s) out.push_back(to_vpq(r[s], Dls[s]));
    return out;
}
