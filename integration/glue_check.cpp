// glue_check.cpp -- drives the Broker glue core (fpf_broker.h) the way
// DPF_hip.cpp does, from plain files, so tests/test_integration.py can compile
// it as C++98 and check it on the GPU against the oracle.
//
//   glue_check in.bin out.bin [log.txt]
// in.bin : int32 nl, ncols, z_rows, z_cols, K, exact; Dl (nl x ncols col-major f64);
//          Z (z_rows x z_cols complex, interleaved re/im, col-major); then K load
//          sets, each the 6 Dl columns 6..11 (nl x 6 col-major f64)
// out.bin: int32 nn, K; then per scenario: int32 iters, int32 converged,
//          f64 loss, vmin, vmax, vpolar[nn*6], pqb[nn*6], pql[nn*6] (col-major);
//          then int32 single_ok (DPF_return7 of scenario 0 equals batch[0]) and
//          int32 threw (DPF_return7 threw std::logic_error on a non-converged scenario, -1: none)
// log.txt: the reference's console lines of the K single DPF_return7 calls
#include <cstdio>
#include <cstring>
#include <fstream>
#include <stdexcept>
#include <vector>

#include "fpf_broker.h"

static bool rd(FILE *f, void *p, size_t n) { return std::fread(p, 1, n, f) == n; }

int main(int argc, char **argv) {
    if (argc != 3 && argc != 4) return 2;
    FILE *in = std::fopen(argv[1], "rb");
    if (!in) return 2;
    int hdr[6];
    if (!rd(in, hdr, sizeof(hdr))) return 2;
    const int nl = hdr[0], ncols = hdr[1], zr = hdr[2], zc = hdr[3], K = hdr[4], exact = hdr[5];
    std::vector<double> dl((size_t)nl * ncols), z((size_t)2 * zr * zc + 2), loads((size_t)K * nl * 6);
    if (!rd(in, &dl[0], dl.size() * 8) || !rd(in, &z[0], (size_t)2 * zr * zc * 8) || !rd(in, &loads[0], loads.size() * 8))
        return 2;
    std::fclose(in);
    // K full Dl tables: the topology of dl, the loads of set s
    std::vector<std::vector<double> > dls(K, dl);
    std::vector<const double *> ptrs;
    for (int s = 0; s < K; ++s) {
        std::memcpy(&dls[s][(size_t)6 * nl], &loads[(size_t)s * nl * 6], sizeof(double) * nl * 6);
        ptrs.push_back(&dls[s][0]);
    }
    fpf_broker::Engine eng(0, exact);
    std::vector<fpf_broker::Vpq> r = eng.dpf_batch(ptrs, nl, ncols, &z[0], zr, zc, false);
    int single_ok = 0, threw = -1;
    std::ofstream log;
    if (argc == 4) {
        log.open(argv[3]);
        eng.set_log(&log);
    }
    for (int s = 0; s < K; ++s) {
        try {
            fpf_broker::Vpq one = eng.dpf_return7(ptrs[s], nl, ncols, &z[0], zr, zc);
            if (s == 0) single_ok = one.vpolar == r[0].vpolar && one.pqb == r[0].pqb && one.pql == r[0].pql &&
                                    one.iters == r[0].iters;
        } catch (const std::logic_error &) {
            if (threw < 0) threw = s;
        }
    }
    FILE *out = std::fopen(argv[2], "wb");
    if (!out) return 2;
    const int nn = eng.info().nn;
    std::fwrite(&nn, 4, 1, out);
    std::fwrite(&K, 4, 1, out);
    for (int s = 0; s < K; ++s) {
        const int it = r[s].iters, cv = r[s].converged ? 1 : 0;
        std::fwrite(&it, 4, 1, out);
        std::fwrite(&cv, 4, 1, out);
        std::fwrite(&r[s].loss, 8, 1, out);
        std::fwrite(&r[s].vmin, 8, 1, out);
        std::fwrite(&r[s].vmax, 8, 1, out);
        std::fwrite(&r[s].vpolar[0], 8, (size_t)nn * 6, out);
        std::fwrite(&r[s].pqb[0], 8, (size_t)nn * 6, out);
        std::fwrite(&r[s].pql[0], 8, (size_t)nn * 6, out);
    }
    std::fwrite(&single_ok, 4, 1, out);
    std::fwrite(&threw, 4, 1, out);
    std::fclose(out);
    return 0;
}
