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

size_t tiled_lds_bytes_rtc(const FeederDev &f, int tile) {
    const size_t slot = f.slot_bytes > 0 ? (size_t)f.slot_bytes : sizeof(double2) * 3 * (size_t)tile;
    const size_t state = (slot * (size_t)f.n_slots + sizeof(Flags) + 15) & ~(size_t)15;
    // + the TEMP blocks staged in LDS; after the sweeps the same bytes hold the
    // tile's aggregate rows (8 doubles per scenario)
    return state + std::max(f.temp_lds ? 144 * (size_t)f.n_fw : 0, (size_t)64 * MAX_SEQ_TILE);
}

size_t tiled_lds_bytes(const FeederDev &f, int tile) {
    const size_t state = sizeof(double2) * 3 * (size_t)tile * (size_t)(f.nn + 2 + f.n_taps + 2) + sizeof(Flags);
    const size_t progs = sizeof(SeqBw) * (size_t)f.n_seq_bw + sizeof(SeqFw) * (size_t)f.n_seq_fw;
    return f.prog_lds ? state + progs : state;
}

int tiled_max_tile(const FeederDev &f) {
    const int nb = f.nn - 1;
    int t = std::min(MAX_SEQ_TILE, (512 * AOT_MAXT) / nb);
    if (t == 0) t = std::min(MAX_SEQ_TILE, (1024 * AOT_MAXT) / nb);
    FeederDev g = f;
    g.prog_lds = 0;
    while (t > 0 && tiled_lds_bytes(g, t) > 160 * 1024) --t;
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
