// fpf_tiled.hip -- AOT instantiations of the tiled kernel (fpf_tiled_body.h)
// with the LDS-program sequential stages, plus sizing and launch helpers.
// Feeders small enough for hipRTC get a topology-specialised build instead
// (fpf_rtc.cpp); this one runs any well-formed feeder that fits in LDS.
#include "fpf_tiled_body.h"

#include <cstdio>
#include <cstdlib>

namespace fpf {

template <int NT>
__global__ __launch_bounds__(NT, 2) void dpf_tiled_kernel(FeederDev f, int B, const double *__restrict__ pq,
                                                          OutDev o) {
    tiled_body<NT, AOT_MAXT, RuntimeProg>(f, B, pq, o);
}

namespace {
template <int NT>
hipError_t launch_nt(const FeederDev &f, int n_scen, const double *pq, const OutDev &o, hipStream_t st) {
    const size_t lds = tiled_lds_bytes(f, f.tile);
    static bool attr_done = false;
    if (!attr_done) {
        hipError_t e = hipFuncSetAttribute((const void *)dpf_tiled_kernel<NT>,
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr_done = true;
    }
    const int grid = (n_scen + f.tile - 1) / f.tile;
    hipLaunchKernelGGL(dpf_tiled_kernel<NT>, dim3(grid), dim3(NT), lds, st, f, n_scen, pq, o);
    return hipGetLastError();
}

}  // namespace

int tiled_threads(const FeederDev &f, int tile) {
    const int tasks = tile * (f.nn - 1);
    if (tasks <= 256 * AOT_MAXT) return 256;
    if (tasks <= 512 * AOT_MAXT) return 512;
    return 1024;
}
namespace {
int threads_for(const FeederDev &f, int tile) { return tiled_threads(f, tile); }
}  // namespace

// Geometry of the specialised build.  The sequential stages cost ~45 cycles per
// row per wave whatever the number of active lanes (each LDS wave-instruction
// has a fixed issue cost), so one sequential wave should carry as many
// scenarios as possible: up to 16 scenarios (48 lanes) per workgroup, two tasks
// per lane, 1024 threads at <= 128 VGPRs -- one workgroup per CU, and a
// 4096-scenario batch is exactly one wave of workgroups on 256 CUs.
int rtc_tile(const FeederDev &f, int *nt, int *maxt) {
    const int nb = f.nn - 1;
    int m = 2, n = 1024;
    int t = std::min(MAX_SEQ_TILE, n * m / nb);
    if (t == 0) return 0;
    // diagnostic override of the geometry: FPF_RTC_GEOM="nt,maxt[,min_waves]"
    if (const char *g = getenv("FPF_RTC_GEOM")) {
        int gn = 0, gm = 0;
        if (sscanf(g, "%d,%d", &gn, &gm) == 2 && (gn == 256 || gn == 512 || gn == 1024) && gm >= 1 && gm <= 4) {
            n = gn;
            m = gm;
            t = std::min(MAX_SEQ_TILE, n * m / nb);
        }
    }
    while (t > 0 && tiled_lds_bytes_rtc(f, t) > 160 * 1024) --t;
    // small feeders: the fewest threads that hold the tile's tasks
    while (n > 256 && t * nb <= (n / 2) * m) n /= 2;
    *nt = n;
    *maxt = m;
    return t;
}

size_t tiled_lds_bytes_rtc(const FeederDev &f, int tile) {
    return sizeof(double2) * 3 * (size_t)tile * (size_t)(f.nn + 2 + f.n_taps + 2) + sizeof(Flags);
}

size_t tiled_lds_bytes(const FeederDev &f, int tile) {
    const size_t state = tiled_lds_bytes_rtc(f, tile);
    const size_t progs = sizeof(SeqBw) * (size_t)f.n_seq_bw + sizeof(SeqFw) * (size_t)f.n_seq_fw;
    return f.prog_lds ? state + progs : state;
}

int tiled_max_tile(const FeederDev &f) {
    const int nb = f.nn - 1;
    int t = std::min(MAX_SEQ_TILE, (512 * AOT_MAXT) / nb);
    if (t == 0) t = std::min(MAX_SEQ_TILE, (1024 * AOT_MAXT) / nb);
    while (t > 0 && tiled_lds_bytes_rtc(f, t) > 160 * 1024) --t;
    return t;
}

hipError_t launch_tiled(const FeederDev &f, int n_scen, const double *pq, const OutDev &o, hipStream_t st) {
    switch (threads_for(f, f.tile)) {
        case 256: return launch_nt<256>(f, n_scen, pq, o, st);
        case 512: return launch_nt<512>(f, n_scen, pq, o, st);
        default: return launch_nt<1024>(f, n_scen, pq, o, st);
    }
}

#ifdef FPF_STAMPS
extern "C" int fpf_debug_set_stamp_buffer(void *dptr) {
    unsigned long long *p = (unsigned long long *)dptr;
    return hipMemcpyToSymbol(HIP_SYMBOL(fpf_stamp_buf), &p, sizeof(p)) == hipSuccess ? 0 : -3;
}
#endif

}  // namespace fpf
