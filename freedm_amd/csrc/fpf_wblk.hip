// fpf_wblk.hip -- the wave-block kernel (fast mode, fpf_opts.exact = 0) for
// feeders of 257..2048 branches (BASELINE config 3: the 2048-bus feeder): every
// sweep of DPF_return7 (Broker/src/vvc/DPF_return7.cpp:104-217) as data-parallel
// work over one workgroup of W wavefronts per scenario.
//
// The per-wavefront wave kernel (fpf_wave.hip) holds a scenario in one segment
// of a wavefront; a 2048-bus scenario needs W = 8 wavefronts (512 lanes x C = 4
// slots).  The layout is the same: the feeder tree in the depth-first order that
// keeps every subtree and every block contiguous, node at position q in slot
// q % C of lane q / C (lane = the workgroup's thread id), V in registers for the
// whole solve.  What changes:
//   * the two prefix scans per sweep (the backward sweep's subtree sums of IL,
//     :134-160; the forward sweep's path sums of the drops, :163-195) are a DPP
//     scan inside each wavefront plus a scan of the W wavefront totals (through
//     LDS, one barrier) that every wave computes alike, so Ib(0) and with it the
//     convergence test (:199-217) are the same in every wave of the workgroup;
//   * LDS holds the scenario's loads (Sld, 3 x (Nl + 1) complex, ~105 KB for
//     2048 buses: one workgroup per CU, 8 wavefronts = 2 per SIMD), the gathered
//     scan values, the block offsets and the per-code impedances;
//   * TEMP = lng * Zl(code) is factorised: a slot keeps its branch's lng in a
//     register and reads Zl of its line code from a small LDS table (the 2048
//     per-slot TEMP blocks would not fit next to Sld), one real scaling per
//     phase more than the wave kernel's precomputed TEMP;
//   * scenario s = blockIdx.x in XCD-aware order (the workgroups one XCD runs
//     take consecutive scenarios, so the [row][B] lines of pq and V that
//     neighbouring scenarios share meet in that XCD's L2).
// Zeroed phases (line codes with a zero self-impedance, :180-192) as in the
// wave kernel: V = 0 on the phase, the path restarting below a zeroed ancestor,
// the loss over PQL and the general V_abc_list extremes (full-output variant).
//
// Arithmetic: as the wave kernel (prefix sums instead of the sequential chains,
// FMA products, one-reciprocal division, Sld scaled by 1/(bkva/3)), checked at
// the north-star bar (1e-10 relative on V, identical iteration counts) against
// the oracle and the exact generic kernel in tests/test_gpu_wblk.py.
#include <array>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <set>

#include "fpf_internal.h"
#include "fpf_wblk_body.h"

namespace fpf {

size_t wblk_lds_bytes(const WaveDev &w) {
    const size_t ntz = w.temp_sym ? 4 : 9, xc = (size_t)w.ncomp + 1, nt = 64 * (size_t)w.wps;
    const size_t zc = 16 * (size_t)w.ncode * ntz;
    const size_t rest = 16 * (3 * ((size_t)w.nl + 1) + 3 * xc + 3 * (size_t)w.nblk * (w.has_rel ? 2 : 1) + 4 + 3 * (size_t)w.nlag) +
                        8 * 16 * (size_t)w.wps + 64 +
                        4 * 2 * (size_t)w.bdepth * w.nblk;
    return zc + std::max(rest, 8 * 8 * nt);   // the last workgroup's fold reuses the space after zc
}

bool wblk_geometry(int n, int *wps, int *c) {
    // C = 4 slots per lane, 2 wavefronts per SIMD; FPF_WBLK_C=8 (experiments):
    // 8 slots per lane, half the wavefronts, 1 per SIMD (AGPRs hold the rest)
    // FPF_WBLK_C=2 (experiments): 2 slots per lane, up to 16 wavefronts = 4 per SIMD
    // (the per-plan build only: no static instantiation)
    const char *e = getenv("FPF_WBLK_C");
    *c = (e && atoi(e) == 8) ? 8 : (e && atoi(e) == 2) ? 2 : WB_C;
    for (int w = 2; w <= (*c == 2 ? 16 : 8); w *= 2)
        if (n <= 64 * w * *c) {
            *wps = w;
            return true;
        }
    return false;
}

namespace {
typedef void (*WblkKernel)(WaveDev, int, const double *, OutDev);
template <int W, int C>
WblkKernel pick_wblk(bool full, bool seg, int gx) {
    // (a live phase below a zeroed one implies zeroed phases: the full variant)
    // The lean full variant for a tree feeder without zeroed phases (GX 0: no VGPR
    // spills); every general path in one instantiation otherwise (GX 3): the
    // zeroed-phase-only one crashes the compiler's register allocator
    if (seg) return dpf_wblk_kernel<W, true, C, true, 1>;
    if (!full) return dpf_wblk_kernel<W, false, C, false, 0>;
    return gx == 0 ? dpf_wblk_kernel<W, true, C, false, 0> : dpf_wblk_kernel<W, true, C, false, 3>;
}
}  // namespace

hipError_t launch_wblk(const WaveDev &w, int n_scen, const double *pq, const OutDev &o, hipStream_t st) {
    if (w.coop) return launch_wcoop(w, n_scen, pq, o, st);   // 2049..4096 branches: fpf_wcoop.hip
    // the full-output variant keeps IL and Ib of the last sweep (Vpolar / PQb /
    // PQL), and the zeroed-phase paths
    // (the tables of a feeder with a live phase below a zeroed one are built for
    // the segmented forward scan: fpf_api.cpp analyse_wave)
    const bool full = o.vpolar || o.pqb || o.pql || w.has_mask || w.has_lag, seg = w.has_rel != 0;   // (has_lag: FULL only)
    // the full variant's general paths only where the plan has them (fpf_wblk_body.h: GX)
    const int gx = w.has_lag ? 2 : (w.has_mask || w.has_rel ? 1 : 0);
    WblkKernel k = nullptr;
    if (w.C == WB_C)
        k = w.wps == 2 ? pick_wblk<2, WB_C>(full, seg, gx)
                       : (w.wps == 4 ? pick_wblk<4, WB_C>(full, seg, gx) : (w.wps == 8 ? pick_wblk<8, WB_C>(full, seg, gx) : nullptr));
    else if (w.C == 8) k = w.wps == 2 ? pick_wblk<2, 8>(full, seg, gx) : (w.wps == 4 ? pick_wblk<4, 8>(full, seg, gx) : nullptr);
    // dynamic LDS above the default 64 KiB: a per-device setting, once per (device, variant)
    static std::mutex mu;
    static std::set<std::array<int, 3>> attr_done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    if (k) {
        std::lock_guard<std::mutex> lk(mu);
        const std::array<int, 3> key = {dev, w.wps * 16 + w.C, (int)full + 2 * (int)seg + 4 * (full ? gx : 0)};
        if (!attr_done.count(key)) {
            hipFuncAttributes fa{};
            hipError_t e = hipFuncGetAttributes(&fa, (const void *)k);
            if (e == hipSuccess)
                e = hipFuncSetAttribute((const void *)k, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        160 * 1024 - (int)fa.sharedSizeBytes);
            if (e != hipSuccess) return e;
            attr_done.insert(key);
        }
    }
#if !defined(FPF_WBLK_ABL) && !defined(FPF_WBLK_NO_GUARD_CODE) && !defined(FPF_STAMPS)
    // launches of at least wave_rtc_min() scenarios: the per-plan hipRTC build
    // (fpf_rtc.cpp), identical results; a failed build runs the static kernel
    if (w.spec && !full && !seg && n_scen >= wave_rtc_min()) {   // (the light variant only, as launch_wave)
        if (hipFunction_t fn = wave_rtc_function(dev, w, false)) {
            WaveDev wa = w;
            OutDev oa = o;
            int b = n_scen;
            const double *p = pq;
            void *args[] = {&wa, &b, &p, &oa};
            return hipModuleLaunchKernel(fn, (unsigned)n_scen, 1, 1, 64u * w.wps, 1, 1, (unsigned)wblk_lds_bytes(w), st,
                                         args, nullptr);
        }
    }
#endif
    if (!k) return hipErrorInvalidValue;   // (FPF_WBLK_C=2: no static build)
    hipLaunchKernelGGL(k, dim3((unsigned)n_scen), dim3(64 * w.wps), wblk_lds_bytes(w), st, w, n_scen, pq, o);
    return hipGetLastError();
}

}  // namespace fpf
