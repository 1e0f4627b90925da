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

#include <algorithm>
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

// Straight-line sequential programs as register dataflow: Ibl, the tap
// accumulators and the forward voltages are SSA values, so a row's dependent
// adds wait on the previous row's adds, never on an LDS store->load round trip.
// LDS only supplies the operands the parallel stages produced (IL, drop) --
// independent loads the compiler issues early -- and receives Ib / V for the
// parallel stages and the epilogue.
//
// Zero folding (exact): Ibl, Ib and tap sums are never -0 (each is a sum with
// an IL term; x + y == -0 needs both -0), so 0 + Ibl == Ibl and T + 0 == T bit
// for bit; a fresh Ibl (+0) plus IL keeps its add because IL may be -0.
// LDS operands are loaded kAhead rows ahead of their use: with the row's store
// in between, 2*kAhead LDS ops are in flight, inside lgkmcnt's 4-bit range.
constexpr int kAhead = 6;

std::string gen_program(const RtcSpec &sp) {
    const long slot = 3L * sp.tile;                       // double2 per node slot
    auto W = [&](int k) { return (long)k * slot; };
    std::ostringstream o;
    o << "namespace fpf {\nstruct GenProg {\n"
      << "  static constexpr int kTile = " << sp.tile << ";\n"
      << "  static constexpr int kNN = " << sp.nn << ";\n"
      << "  static constexpr bool kLdsProgram = false;\n"
      << "  static constexpr bool kLdsTaps = false;\n"
      << "  __device__ static __forceinline__ cx ld(const double2 *B, int i) { const double2 v = B[i]; return mk(v.x, v.y); }\n"
      << "  __device__ static __forceinline__ void st(double2 *B, int i, cx v) { B[i] = make_double2(v.re, v.im); }\n";
    // backward (DPF_return7.cpp:134-160 with separators folded into the preceding op):
    // x = (T[a] + Ibl) + IL[k]; Ib[k] = x; separator: T[p] = T[p] + x, Ibl = 0
    o << "  __device__ static __forceinline__ void s1(char *L, uint32_t lane_off, const SeqBw *, int, cx &) {\n"
      << "    double2 *B = (double2 *)(L + lane_off);\n";
    {
        std::string ibl;                       // "" = +0
        std::map<int, std::string> tap;        // absent = +0
        const size_t nbw = sp.bw.size();
        auto load_il = [&](size_t i) { o << "    const cx il" << i << " = ld(B, " << W(sp.bw[i][0]) << ");\n"; };
        for (size_t i = 0; i < std::min(nbw, (size_t)kAhead); ++i) load_il(i);
        for (size_t i = 0; i < nbw; ++i) {
            const auto &op = sp.bw[i];
            if (i + kAhead < nbw) load_il(i + kAhead);
            const std::string il = "il" + std::to_string(i), x = "x" + std::to_string(i);
            const std::string t = (op[1] >= 0 && tap.count(op[1])) ? tap[op[1]] : "";
            o << "    const cx " << x << " = ";
            if (!t.empty()) o << (ibl.empty() ? "cadd(" + t + ", " + il + ")" : "cadd(cadd(" + t + ", " + ibl + "), " + il + ")");
            else o << (ibl.empty() ? "cadd(mk(0, 0), " + il + ")" : "cadd(" + ibl + ", " + il + ")");
            o << "; st(B, " << W(op[0]) << ", " << x << ");";
            if (op[2] >= 0) {
                auto it = tap.find(op[2]);
                if (it == tap.end()) {
                    tap[op[2]] = x;
                } else {
                    const std::string tn = "t" + std::to_string(i);
                    o << " const cx " << tn << " = cadd(" << it->second << ", " << x << ");";
                    it->second = tn;
                }
                ibl.clear();
            } else {
                ibl = x;
            }
            o << "\n";
        }
    }
    o << "  }\n";
    // forward (:163-195): V[dst] = V[src] - drop[dst], phases in mask zeroed
    o << "  __device__ static __forceinline__ void s2(char *L, uint32_t lane_off, const SeqFw *, int, int qp) {\n"
      << "    double2 *B = (double2 *)(L + lane_off);\n"
      << "    const cx v0 = ld(B, 0);\n";
    const size_t nfw = sp.fw.size();
    auto load_d = [&](size_t i) { o << "    const cx d" << i << " = ld(B, " << W(sp.fw[i][0]) << ");\n"; };
    for (size_t i = 0; i < std::min(nfw, (size_t)kAhead); ++i) load_d(i);
    for (size_t i = 0; i < nfw; ++i) {
        const auto &op = sp.fw[i];
        if (i + kAhead < nfw) load_d(i + kAhead);
        const std::string v = "v" + std::to_string(op[0]);
        o << "    cx " << v << " = csub(v" << op[1] << ", d" << i << ");";
        if (op[2]) o << " if ((" << op[2] << " >> qp) & 1) " << v << " = mk(0, 0);";
        o << " st(B, " << W(op[0]) << ", " << v << ");\n";
    }
    o << "  }\n";
    o << "};\n}  // namespace fpf\n"
      << "extern \"C\" __global__ __launch_bounds__(" << sp.nt << ", " << sp.min_waves << ") void fpf_rtc_tiled(fpf::FeederDev f, int B, "
      << "const double *__restrict__ pq, fpf::OutDev o) {\n"
      << "  fpf::tiled_body<" << sp.nt << ", " << sp.maxt << ", fpf::GenProg>(f, B, pq, o);\n}\n";
    return o.str();
}
}  // namespace

std::string rtc_source(const RtcSpec &sp) {
    std::string src;
    for (const char *part : kRtcSources) src += part;
    src += gen_program(sp);
    return src;
}

int rtc_build(int device, const RtcSpec &sp, RtcKernel *out, std::string *err) {
    const std::string src = rtc_source(sp);
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
    // dynamic LDS above the default 64 KiB (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute((const void *)k.fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
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
