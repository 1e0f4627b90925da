// fpf_wave.hip -- the wave kernel (fast mode, fpf_opts.exact = 0): every sweep
// of DPF_return7 (Broker/src/vvc/DPF_return7.cpp:104-217) as data-parallel work
// over a segment of L = 64/SPW lanes per scenario, SPW scenarios per wavefront.
//
// The feeder tree (node k's parent = sbus of its row; for the feeders this
// kernel accepts this is also the node that receives Ib(k) in the backward
// sweep, :134-160) is laid out in a depth-first order that visits a node's
// in-block child before its laterals, so
//   * every subtree is a contiguous range of positions  -> the backward sweep
//       Ib(k) = sum of IL over the subtree of k = Einc[last(k)] - Eexc[pos(k)]
//     is one segment-wide prefix scan E of IL plus one gather;
//   * every block (Dl row run between separator rows) is a contiguous range
//     -> the forward sweep V(k) = V(src) - drop(k) (:163-195), i.e.
//       V(k) = V0 - A(k), A(k) = sum of drops on the path 1..k,
//     is one prefix scan G of the drops: A(k) = Ginc[pos(k)] + off(block(k)),
//     off(b) = sum over b's block-ancestor chain of (Ginc[tap] - Ginc[first-1]),
//     resolved by one lane per block.
// Phase zeroing (:180-192): V(k,p) = 0 on a zeroed phase, and below a zeroed
// ancestor m the path restarts from 0: V(k,p) = A(m) - A(k).
//
// Node at position q lives in slot c = q % C of segment lane q / C; its state
// (Sld, V, IL, Ib) stays in registers for the whole solve.  LDS holds, per
// scenario, the scan array (X, [3][L*C+1] complex, slot-major so a lane's
// stores are conflict-free; entry L*C is a permanent zero) and the block
// offsets, and once per workgroup the TEMP blocks (lng * Z/Zb, 9 complex per
// branch) and the block-chain table.  Scans are DPP row shifts (+ row
// broadcasts for L = 32, 64) on the fp64 halves; segments never read each
// other's lanes.  A scenario's outputs are written in the sweep it converges
// in (or its 20th); its lanes then idle along until the wave's last scenario
// is done.
//
// Arithmetic: the quantities of the reference with a different association
// (prefix sums instead of the sequential chains, FMA products, one-reciprocal
// division, Sld scaled by 1/(bkva/3)): a few ulp per operation, checked at the
// north-star bar (1e-10 relative on V, identical iteration counts) in
// tests/test_gpu_parity.py.  Voltages are per-unit: |V|^2 must stay a normal
// double (a solve that diverges past 1e+-150 p.u. gets non-finite values; its
// status is NONCONVERGED either way).
#include <algorithm>
#include <array>
#include <cstdio>
#include <mutex>
#include <set>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "fpf_internal.h"
#include "fpf_wave_body.h"

namespace fpf {

// STG double index of pq element (field fq, row r) of the workgroup's scenario j
static int stg_double(int fq, int r, int j, int nl, int srow) {
    return 2 * (((fq >> 1) * (swz_row(nl) + 1) + swz_row(r)) * srow + j) + (fq & 1);
}

int wave_out_tables(const WaveDev &w, std::vector<int32_t> &smaj, std::vector<int32_t> &l0) {
    const int spb = w.wpb * w.spw, nt = w.wpb * 64, nl = w.nl, nn = w.nn, srow = spb + 1;
    const int ntot = spb * 3 * nn, U = (ntot + nt - 1) / nt;
    if (U > WAVE_STAGE_U || (spb & (spb - 1))) return 0;
    const int pstr = (swz_row(nl) + 1) * srow, xc = w.ncomp + 1, noff = w.off_in_x ? 0 : 3 * w.nblk;
    const int rs = (3 * xc + noff + 4 + REGION_EXTRA + 3 * w.nlag) | 1;
    auto at = [&](int j, int p, int k) { return k == 0 ? 3 * pstr + j * rs + 3 * xc + noff + p : p * pstr + swz_row(k - 1) * srow + j; };
    smaj.assign((size_t)U * nt, 0);
    l0.assign((size_t)U * nt, 0);
    for (int i = 0; i < ntot; ++i) {
        smaj[i] = at(i / (3 * nn), (i % (3 * nn)) / nn, i % nn);
        l0[i] = at(i % spb, (i / spb) / nn, (i / spb) % nn);
    }
    return U;
}

int wave_stage_tables(const WaveDev &w, std::vector<int32_t> &smaj, std::vector<int32_t> &l0) {
    const int spb = w.wpb * w.spw, nt = w.wpb * 64, nl = w.nl, srow = spb + 1;
    const int nchunk = spb * 3 * nl, U = (nchunk + nt - 1) / nt;
    if (U > WAVE_STAGE_U || spb % 2) return 0;
    smaj.assign((size_t)2 * U * nt, 0);
    l0.assign((size_t)2 * U * nt, 0);
    const int H = spb / 2;
    for (int u = 0; u < U; ++u)
        for (int t = 0; t < nt; ++t) {
            const int c = u * nt + t;
            int32_t *a = &smaj[2 * (size_t)c], *b = &l0[2 * (size_t)c];
            if (c >= nchunk) continue;
            // scenario major: elements e = 2c, 2c + 1 of the tile's [spb][6][nl] block
            const int e = 2 * c, j = e / (6 * nl), rem = e % (6 * nl), fq = rem / nl, r = rem % nl;
            a[0] = stg_double(fq, r, j, nl, srow);
            a[1] = r + 1 < nl ? stg_double(fq, r + 1, j, nl, srow) : stg_double(fq + 1, 0, j, nl, srow);
            // scenario fastest: line fr of [6 nl][B], the scenario pair 2 (t % H), 2 (t % H) + 1
            const int fr = t / H + u * (nt / H), jj = 2 * (t % H);
            b[0] = fr;
            b[1] = fr < 6 * nl ? stg_double(fr / nl, fr % nl, jj, nl, srow) : 0;
        }
    return U;
}

void wave_io_units(WaveDev &w) {
    w.stage_uw = w.out_uw = 0;
    if (getenv("FPF_WAVE_WG_IO")) return;   // (experiments: the workgroup's IO)
    const int suw = (w.spw * 3 * w.nl + 63) / 64, ouw = (w.spw * 3 * w.nn + 63) / 64;
    if (w.stage_u > 0 && w.out_u > 0 && suw <= WAVE_STAGE_U && ouw <= WAVE_STAGE_U) {
        w.stage_uw = suw;
        w.out_uw = ouw;
    }
}

// (experiments) the per-plan builds read TEMP through the vector memory pipe
// (FPF_WAVE_RTC_DEFS names FPF_WAVE_TEMP_VMEM): no TEMP block in LDS.  Only
// launches that run the per-plan build may be sized so (FPF_WAVE_WPB=2 has no
// static kernel)
static bool rtc_temp_vmem() {
    static const bool on = [] {
        const char *d = getenv("FPF_WAVE_RTC_DEFS");
        return d && strstr(d, "FPF_WAVE_TEMP_VMEM");
    }();
    return on;
}

// the dynamic LDS of one launch: temp_in_lds is the launched build's own choice
// (the static kernels always stage TEMP in LDS; a per-plan build compiled with
// FPF_WAVE_TEMP_VMEM does not)
static size_t wave_lds_bytes_as(const WaveDev &w, bool temp_in_lds) {
    const size_t L = 64 / (size_t)w.spw, xc = (size_t)w.ncomp + 1, spb = (size_t)w.wpb * w.spw;
    const size_t pairs = ((2 * (size_t)w.bdepth * w.nblk + 3) & ~(size_t)3) * 4 + 4 * (size_t)w.C * L;
    const size_t regions = 16 * spb * ((3 * xc + (w.off_in_x ? 0 : 3 * (size_t)w.nblk) + 4 + REGION_EXTRA + 3 * (size_t)w.nlag) | 1);
    const size_t stage = 16 * 3 * ((size_t)swz_row(w.nl) + 1) * (spb + 1);   // STG: Sld in place, then V
    const size_t agg = 8 * 8 * (size_t)w.wpb * 64;                     // the last workgroup's fold
    const size_t temp = temp_in_lds ? 16 * ((w.temp_sym ? 4 : 9) * (size_t)w.C * L) : 0;
    return temp + pairs + std::max(stage + regions, agg);
}

// the plan's figure (the large launches' build: the per-plan one when the
// experiment switch moves TEMP out of LDS)
size_t wave_lds_bytes(const WaveDev &w) { return wave_lds_bytes_as(w, TEMP_IN_LDS && !rtc_temp_vmem()); }

int wave_scenarios_per_block(const WaveDev &w) { return w.wps ? 1 : w.wpb * w.spw; }   // wps: fpf_wblk.hip

// the waves-per-workgroup choices each geometry is built for
bool wave_wpb_supported(int spw, int c, int wpb) {
    // (2: experiments, FPF_WAVE_WPB=2 with FPF_WAVE_TEMP_VMEM -- per-plan build only)
    return spw * c <= 2 ? (wpb == 16 || wpb == 8) : (wpb == 8 || wpb == 4 || (wpb == 2 && rtc_temp_vmem()));
}

namespace {
typedef void (*WaveKernel)(WaveDev, int, const double *, OutDev);
template <int SPW, int C, int WPB>
WaveKernel pick_w(bool full, int gx) {
    if (!full) return dpf_wave_kernel<SPW, C, false, WPB, 0>;
    if (gx == 2) return dpf_wave_kernel<SPW, C, true, WPB, 2>;
    if (gx == 0) return dpf_wave_kernel<SPW, C, true, WPB, 0>;
    // (the 1-scenario, 2-slot geometry -- FPF_WAVE_GEOM experiments only -- has no
    // zeroed-phase instantiation: the compiler's register allocator crashes on it)
    if constexpr (SPW == 1 && C == 2) return nullptr;
    else if (gx == 3) return dpf_wave_kernel<SPW, C, true, WPB, 3>;   // sequential order with zeroed phases
    else return dpf_wave_kernel<SPW, C, true, WPB, 1>;
}
template <int SPW, int C>
WaveKernel pick(bool full, int gen, int wpb) {
    if constexpr (SPW * C <= 2) {
        if (wpb == 16) return pick_w<SPW, C, 16>(full, gen);
        if (wpb == 8) return pick_w<SPW, C, 8>(full, gen);
    } else {
        if (wpb == 8) return pick_w<SPW, C, 8>(full, gen);
        if (wpb == 4) return pick_w<SPW, C, 4>(full, gen);
    }
    return nullptr;
}
}  // namespace

hipError_t launch_wave(const WaveDev &w, int n_scen, const double *pq, const OutDev &o, hipStream_t st) {
    const int per_block = wave_scenarios_per_block(w);
    const unsigned grid = (unsigned)((n_scen + per_block - 1) / per_block);
    // (the static kernels' size; the per-plan build's below)
    const size_t lds = wave_lds_bytes_as(w, TEMP_IN_LDS);
    // FULL keeps IL and Ib of the last sweep for Vpolar/PQb/PQL, and for the
    // loss of a feeder with zeroed phases (reference formula over PQL)
    const bool full = o.vpolar || o.pqb || o.pql || w.has_mask || w.has_lag;   // (the sequential-order plan: FULL only)
    // the general paths only where the plan has them (fpf_wave_body.h: GX): zeroed
    // phases (bit 0), the sequential-order plan (bit 1)
    const int gen = (w.has_lag ? 2 : 0) | (w.has_mask || w.has_rel ? 1 : 0);
    WaveKernel k = nullptr;
    int id = -1;
    if (w.spw == 4 && w.C == 1) { k = pick<4, 1>(full, gen, w.wpb); id = 0; }
    else if (w.spw == 4 && w.C == 2) { k = pick<4, 2>(full, gen, w.wpb); id = 1; }
    else if (w.spw == 4 && w.C == 4) { k = pick<4, 4>(full, gen, w.wpb); id = 2; }
    else if (w.spw == 2 && w.C == 4) { k = pick<2, 4>(full, gen, w.wpb); id = 3; }
    else if (w.spw == 1 && w.C == 4) { k = pick<1, 4>(full, gen, w.wpb); id = 4; }
    else if (w.spw == 1 && w.C == 2) { k = pick<1, 2>(full, gen, w.wpb); id = 5; }
    else if (w.spw == 2 && w.C == 2) { k = pick<2, 2>(full, gen, w.wpb); id = 6; }
    // dynamic LDS above the default 64 KiB (gfx950: 160 KiB per CU, minus the
    // static part) -- a per-device setting, done once per (device, variant)
    static std::mutex mu;
    static std::set<std::array<int, 4>> attr_done;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorInvalidDevice;
    if (k) {
        std::lock_guard<std::mutex> lk(mu);
        const std::array<int, 4> key = {dev, id, (int)full + 2 * (full ? gen : 0), w.wpb};
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
    WaveDev wl = w;
    wl.stag_lo = wl.stag_hi = wl.stag_n = 0;
    if (getenv("FPF_PRINT_WAVEDEV"))   // (diagnostic: the uniform plan values of a launch)
        fprintf(stderr, "wavedev spw %d C %d wpb %d nl %d nn %d nblk %d bdepth %d ncomp %d temp_sym %d off_in_x %d "
                "stage_u %d out_u %d has_mask %d has_rel %d mxitr %d\n", w.spw, w.C, w.wpb, w.nl, w.nn, w.nblk, w.bdepth,
                w.ncomp, (int)w.temp_sym, (int)w.off_in_x, w.stage_u, w.out_u, (int)w.has_mask, (int)w.has_rel, w.mxitr);
    if (const char *e = getenv("FPF_WAVE_WG_STAGGER")) {   // experiments: "lo,hi,n"
        if (sscanf(e, "%d,%d,%d", &wl.stag_lo, &wl.stag_hi, &wl.stag_n) != 3) wl.stag_lo = wl.stag_hi = wl.stag_n = 0;
    }
#if !defined(FPF_STAMPS) && !defined(FPF_WAVE_ABL) && !defined(FPF_WAVE_ABLATE)
    // launches of at least wave_rtc_min() scenarios run the per-plan hipRTC build
    // (fpf_rtc.cpp: ~2.5 s to compile, once per plan and variant in a process);
    // smaller ones, and a failed or non-resident build, the static kernel --
    // identical results (the light variant only: the full-output variants --
    // Vpolar / PQb / PQL, zeroed phases, lag -- keep the static build, which is
    // spill-free for them since the round-5 restructure)
    if (w.spec && !full && n_scen >= wave_rtc_min()) {
        if (hipFunction_t fn = wave_rtc_function(dev, w, full)) {
            OutDev oa = o;
            int b = n_scen;
            const double *p = pq;
            void *args[] = {&wl, &b, &p, &oa};
            const size_t lds_rtc = wave_lds_bytes_as(w, TEMP_IN_LDS && !rtc_temp_vmem());
            hipError_t e = hipModuleLaunchKernel(fn, grid, 1, 1, (unsigned)w.wpb * 64, 1, 1, (unsigned)lds_rtc, st,
                                                 args, nullptr);
            return e;
        }
    }
#endif
    if (!k) return hipErrorInvalidValue;   // (FPF_WAVE_WPB=2: no static build)
    hipLaunchKernelGGL(k, dim3(grid), dim3(w.wpb * 64), lds, st, wl, n_scen, pq, o);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess && getenv("FPF_DEBUG")) {
        hipFuncAttributes fa{};
        (void)hipFuncGetAttributes(&fa, (const void *)k);
        fprintf(stderr, "launch_wave: %s grid %u block %d dyn lds %zu static %zu maxdyn %d regs %d local %zu\n",
                hipGetErrorString(e), grid, w.wpb * 64, lds, fa.sharedSizeBytes, fa.maxDynamicSharedSizeBytes,
                fa.numRegs, fa.localSizeBytes);
    }
    return e;
}

// the (scenarios per wave, slots per lane) geometry for n branches
bool wave_geometry(int n, int *spw, int *c) {
    static const int cfg[5][2] = {{4, 1}, {4, 2}, {2, 2}, {2, 4}, {1, 4}};
    if (const char *e = getenv("FPF_WAVE_GEOM")) {   // experiments: "spw,c"
        int a = 0, b = 0;
        if (sscanf(e, "%d,%d", &a, &b) == 2 && n <= (64 / std::max(a, 1)) * b) {
            *spw = a;
            *c = b;
            return true;
        }
    }
    for (const auto &g : cfg)
        if (n <= (64 / g[0]) * g[1]) {
            *spw = g[0];
            *c = g[1];
            return true;
        }
    return false;
}

}  // namespace fpf
