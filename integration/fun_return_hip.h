// Broker/src/vvc/fun_return_hip.h -- the one declaration DPF_hip.cpp adds to the
// Broker beside fun_return.h:53 (VPQ DPF_return7(arma::mat Dl, arma::cx_mat Z)):
// DPF_batch, K Dl tables of one topology (columns 0..5) and one Z solved as one
// batch on libfreedm_pf, each result as DPF_return7 would return it.  Include it
// after fun_return.h where a caller (VoltVarCtrl.cpp's step-size search,
// :1330-1542) batches its candidates; fun_return.h itself stays unchanged.
#ifndef FUN_RETURN_HIP_H
#define FUN_RETURN_HIP_H

#include <vector>

#include "fun_return.h"

std::vector<VPQ> DPF_batch(const std::vector<arma::mat> &Dls, const arma::cx_mat &Z);

#endif
