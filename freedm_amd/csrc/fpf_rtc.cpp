// fpf_rtc.cpp -- topology-specialised tiled kernel via hipRTC.
//
// The tiled kernel's sequential stages are the feeder's backward/forward
// programs (one op per Dl row).  Interpreted from LDS (RuntimeProg) each op
// pays for descriptor loads and address arithmetic; here the programs are
// emitted as straight-line device code with compile-time LDS offsets and tile,
// so each op is its LDS reads, one or two dependent complex adds and its LDS
// write, and the compiler schedules every read as early as its operand allows.
// The arithmetic per op is the reference's (DPF_return7.cpp:134-195), so V stays
// bit-identical.  One build per (feeder topology, tile); compiled once at
// fpf_feeder_create and cached per process.
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <cstdio>
#include <map>
#include <mutex>
#include <sstream>
#include <string>

#include "fpf_internal.h"

namespace fpf {

#include "fpf_rtc_src.inc"

#ifdef FPF_STAMPS
// diagnostic build: the stamp buffer of the hipRTC module (fpf::fpf_stamp_buf)
void *g_rtc_stamp_ptr = nullptr;
extern "C" int fpf_debug_set_rtc_stamp_buffer(void *dptr) {
    g_rtc_stamp_ptr = dptr;
    return 0;
}
#endif

namespace {
std::mutex g_mu;
std::map<std::pair<int, std::string>, RtcKernel> g_cache;

std::string gen_program(const RtcSpec &sp) {
    const long slot = 3L * sp.tile;                       // double2 per node slot
    const long tbase = (long)(sp.nn + 2) * slot;
    auto W = [&](int k) { return (long)k * slot; };
    auto T = [&](int t) { return tbase + (long)t * slot; };
    std::ostringstream o;
    o << "namespace fpf {\nstruct GenProg {\n"
      << "  static constexpr int kTile = " << sp.tile << ";\n"
      << "  static constexpr bool kLdsProgram = false;\n"
      // backward: x = (T[a] + Ibl) + IL[k]  (T[a] = 0 for non-taps; 0 + Ibl == Ibl bit for
      // bit because Ibl is never -0), Ib[k] = x, separator: T[p] += x, Ibl = 0
      << "  __device__ static __forceinline__ void s1(char *L, uint32_t lane_off, const SeqBw *, int, cx &ibl) {\n"
      << "    double2 *B = (double2 *)(L + lane_off);\n    double2 w_, t_;\n    cx x;\n";
    for (const auto &op : sp.bw) {
        o << "    w_ = B[" << W(op[0]) << "];";
        if (op[1] >= 0)
            o << " t_ = B[" << T(op[1]) << "]; x = cadd(cadd(mk(t_.x, t_.y), ibl), mk(w_.x, w_.y));";
        else
            o << " x = cadd(ibl, mk(w_.x, w_.y));";
        o << " B[" << W(op[0]) << "] = make_double2(x.re, x.im);";
        if (op[2] >= 0)
            o << " t_ = B[" << T(op[2]) << "]; B[" << T(op[2]) << "] = make_double2(t_.x + x.re, t_.y + x.im); ibl = mk(0, 0);\n";
        else
            o << " ibl = x;\n";
    }
    o << "  }\n"
      // forward: V[dst] = V[src] - drop[dst], phases in mask zeroed
      << "  __device__ static __forceinline__ void s2(char *L, uint32_t lane_off, const SeqFw *, int, int qp) {\n"
      << "    double2 *B = (double2 *)(L + lane_off);\n    double2 d_, s_;\n    cx v = mk(0, 0);\n";
    int prev = -1;
    for (const auto &op : sp.fw) {
        o << "    d_ = B[" << W(op[0]) << "];";
        if (!(op[1] != 0 && op[1] == prev)) o << " s_ = B[" << W(op[1]) << "]; v = mk(s_.x, s_.y);";
        o << " v = csub(v, mk(d_.x, d_.y));";
        if (op[2]) o << " if ((" << op[2] << " >> qp) & 1) v = mk(0, 0);";
        o << " B[" << W(op[0]) << "] = make_double2(v.re, v.im);\n";
        prev = op[0];
    }
    o << "  }\n};\n}  // namespace fpf\n"
      << "extern \"C\" __global__ __launch_bounds__(" << sp.nt << ", 2) void fpf_rtc_tiled(fpf::FeederDev f, int B, "
      << "const double *__restrict__ pq, fpf::OutDev o) {\n"
      << "  fpf::tiled_body<" << sp.nt << ", fpf::GenProg>(f, B, pq, o);\n}\n";
    return o.str();
}
}  // namespace

int rtc_build(int device, const RtcSpec &sp, RtcKernel *out, std::string *err) {
    std::string src;
    for (const char *part : kRtcSources) src += part;
    src += gen_program(sp);
    std::lock_guard<std::mutex> lk(g_mu);
    auto key = std::make_pair(device, src);
    auto it = g_cache.find(key);
    if (it != g_cache.end()) {
        *out = it->second;
        return 0;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "fpf_rtc_tiled.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        *err = "hiprtcCreateProgram failed";
        return -1;
    }
#ifdef FPF_STAMPS
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17", "-DFPF_STAMPS"};
    hiprtcResult rr = hiprtcCompileProgram(prog, 5, opts);
#else
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17"};
    hiprtcResult rr = hiprtcCompileProgram(prog, 4, opts);
#endif
    if (rr != HIPRTC_SUCCESS) {
        size_t n = 0;
        hiprtcGetProgramLogSize(prog, &n);
        std::string log(n, '\0');
        if (n) hiprtcGetProgramLog(prog, &log[0]);
        *err = std::string("hipRTC compile failed: ") + hiprtcGetErrorString(rr) + "\n" + log.substr(0, 4000);
        hiprtcDestroyProgram(&prog);
        return -1;
    }
    size_t n = 0;
    hiprtcGetCodeSize(prog, &n);
    std::string code(n, '\0');
    hiprtcGetCode(prog, &code[0]);
    hiprtcDestroyProgram(&prog);
    RtcKernel k{};
    if (hipModuleLoadData(&k.mod, code.data()) != hipSuccess ||
        hipModuleGetFunction(&k.fn, k.mod, "fpf_rtc_tiled") != hipSuccess) {
        *err = "hipModuleLoadData / hipModuleGetFunction failed";
        return -1;
    }
    k.nt = sp.nt;
    g_cache[key] = k;
    *out = k;
    return 0;
}

hipError_t rtc_launch(const RtcKernel &k, const FeederDev &f, int n_scen, const double *pq, const OutDev &o,
                      hipStream_t st) {
    FeederDev fa = f;
    OutDev oa = o;
    int B = n_scen;
    const double *p = pq;
    void *args[] = {&fa, &B, &p, &oa};
    const unsigned grid = (unsigned)((n_scen + f.tile - 1) / f.tile);
    const size_t lds = tiled_lds_bytes_rtc(f, f.tile);
#ifdef FPF_STAMPS
    {
        hipDeviceptr_t sym;
        size_t bytes = 0;
        if (hipModuleGetGlobal(&sym, &bytes, k.mod, "_ZN3fpf13fpf_stamp_bufE") == hipSuccess && bytes == sizeof(void *))
            (void)hipMemcpyHtoDAsync(sym, &g_rtc_stamp_ptr, sizeof(void *), st);
    }
#endif
    return hipModuleLaunchKernel(k.fn, grid, 1, 1, (unsigned)k.nt, 1, 1, (unsigned)lds, st, args, nullptr);
}

}  // namespace fpf
