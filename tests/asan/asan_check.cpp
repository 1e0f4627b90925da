// asan_check.cpp -- host sanitizer run (-fsanitize=address,undefined)
// over the C ABI's host code and the oracle.  Built by tests/asan/Makefile with
// the host objects of libfreedm_pf compiled host-only under ASan/UBSan (the
// kernels are linked unsanitised: GPU sanitizers are not available), run by
// tests/test_sanitize.py on CPU -- no device is touched: it exercises the
// no-device entry points (feeder analysis, wave plan, hipRTC source generation,
// shard / fold arithmetic, error paths) and the oracle's solve, batch and VVC
// round on every feeder file given on the command line.
//
// Feeder file: int32 nl, ncols, z_rows, z_cols; then Dl (nl x ncols, f64,
// column-major); then Z (z_rows x z_cols complex, re/im interleaved, column-major).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "freedm_pf.h"
extern "C" {
#include "ref_dpf.h"
}

static bool read_feeder(const char *path, int hdr[4], std::vector<double> &dl, std::vector<double> &z) {
    FILE *f = fopen(path, "rb");
    if (!f) return false;
    bool ok = fread(hdr, sizeof(int), 4, f) == 4;
    if (ok) {
        dl.resize((size_t)hdr[0] * hdr[1]);
        z.resize((size_t)2 * hdr[2] * hdr[3] + 2);
        ok = fread(dl.data(), sizeof(double), dl.size(), f) == dl.size() &&
             fread(z.data(), sizeof(double), (size_t)2 * hdr[2] * hdr[3], f) == (size_t)2 * hdr[2] * hdr[3];
    }
    fclose(f);
    return ok;
}

int main(int argc, char **argv) {
    int failures = 0;
    fpf_opts o;
    fpf_opts_default(&o);
    printf("abi %d\n", fpf_abi_version());
    // shard / fold arithmetic
    long lo = 0, hi = 0, total = 0;
    for (int r = 0; r < 8; ++r) {
        if (fpf_multi_shard(r, 8, 1000003, &lo, &hi) != FPF_OK) ++failures;
        total += hi - lo;
    }
    if (total != 1000003) ++failures;
    fpf_aggregate parts[3];
    std::memset(parts, 0, sizeof(parts));
    for (int i = 0; i < 3; ++i) {
        parts[i].loss_sum = i;
        parts[i].vmin = 0.9 + 0.01 * i;
        parts[i].vmax = 1.0 + 0.01 * i;
        parts[i].n_scen = 10;
    }
    fpf_aggregate all;
    fpf_aggregate_fold(parts, 3, &all);
    if (all.n_scen != 30 || all.vmin != 0.9) ++failures;
    // error paths without a device
    fpf_ctx *ctx = nullptr;
    if (fpf_ctx_create(0, &ctx) == FPF_OK) fpf_ctx_destroy(ctx);   // no GPU here: an error code
    fpf_multi *m = nullptr;
    if (fpf_multi_create(4096, nullptr, 0, 0, nullptr, 0, 0, &o, &m) >= 0) ++failures;
    printf("multi create: %s\n", fpf_multi_last_error(nullptr));

    for (int a = 1; a < argc; ++a) {
        int h[4];
        std::vector<double> dl, z;
        if (!read_feeder(argv[a], h, dl, z)) {
            printf("%s: unreadable\n", argv[a]);
            ++failures;
            continue;
        }
        const int nl = h[0], nc = h[1], zr = h[2], zc = h[3];
        int plan[8];
        const int rp = fpf_feeder_wave_plan(dl.data(), nl, nc, z.data(), zr, zc, &o, plan);
        int lplan[8];
        std::vector<int> lslots(8 * 16 * 4), lblk(4096 * 17);
        const int rl = fpf_feeder_lane_plan(dl.data(), nl, nc, z.data(), zr, zc, &o, lplan, lslots.data(), (int)lslots.size(),
                                            lblk.data(), (int)lblk.size());
        const long need = fpf_feeder_rtc_source(dl.data(), nl, nc, z.data(), zr, zc, &o, nullptr, 0);
        std::vector<char> src(need > 0 ? (size_t)need : 1);
        const long got = need > 0 ? fpf_feeder_rtc_source(dl.data(), nl, nc, z.data(), zr, zc, &o, src.data(), src.size()) : need;
        // the oracle: one solve, a 4-scenario batch on 2 threads
        ref_opts ro;
        ref_opts_default(&ro);
        ref_out out;
        std::memset(&out, 0, sizeof(out));
        const int rs = ref_dpf_solve(dl.data(), nl, nc, z.data(), zr, zc, &ro, &out);
        const int B = 4, nn = ref_count_nodes(dl.data(), nl, nc);
        int rb = -99;
        if (nn > 0) {
            std::vector<double> pq((size_t)6 * nl * B), vre((size_t)3 * nn * B), vim((size_t)3 * nn * B), loss(B), vmin(B), vmax(B);
            for (int c = 0; c < 6; ++c)
                for (int r = 0; r < nl; ++r)
                    for (int s = 0; s < B; ++s) pq[((size_t)c * nl + r) * B + s] = dl[(size_t)(6 + c) * nl + r] * (0.8 + 0.1 * s);
            std::vector<int> it(B);
            std::vector<signed char> st(B);
            rb = ref_dpf_batch(dl.data(), nl, nc, z.data(), zr, zc, &ro, B, pq.data(), nullptr, nullptr, nullptr,
                               vre.data(), vim.data(), it.data(), st.data(), loss.data(), vmin.data(), vmax.data(), 2);
        }
        int rv = -99;
        if (nl <= 200 && rs == 0) {   // the VVC round on the small feeders
            const int ld = nl, mm = 30;
            std::vector<double> g(3 * ld), nodes(3 * ld), lf(mm + 1), lr(mm + 1), dlo(dl.size()), res(13);
            int nloads[3];
            rv = ref_vvc_main(dl.data(), nl, nc, z.data(), zr, zc, &ro, 0.1, 1.1, mm, ld, g.data(), nodes.data(), nloads,
                              lf.data(), lr.data(), dlo.data(), res.data());
        }
        printf("%s: nl %d plan rc %d ok %d lane %d/%d | rtc src %ld/%ld | ref solve %d batch %d vvc %d\n", argv[a], nl, rp,
               rp == 0 ? plan[0] : -1, rl, rl == 0 ? lplan[0] : -1, got, need, rs, rb, rv);
    }
    printf(failures ? "FAILURES %d\n" : "asan_check ok\n", failures);
    return failures ? 1 : 0;
}
