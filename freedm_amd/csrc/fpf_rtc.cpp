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

// Straight-line sequential programs, emitted in chunks of kChunk ops: each
// chunk first loads every LDS operand no earlier op of the chunk writes, then
// runs its dependent arithmetic, so LDS latency overlaps the chain instead of
// sitting on it.  Operands an earlier op of the chunk writes (a tap accumulator
// a separator of the same chunk just added into) are read in program order.
constexpr int kChunk = 8;

std::string gen_program(const RtcSpec &sp) {
    const long slot = 3L * sp.tile;                       // double2 per node slot
    const long tbase = (long)(sp.nn + 2) * slot;
    auto W = [&](int k) { return (long)k * slot; };
    auto T = [&](int t) { return tbase + (long)t * slot; };
    std::ostringstream o;
    o << "namespace fpf {\nstruct GenProg {\n"
      << "  static constexpr int kTile = " << sp.tile << ";\n"
      << "  static constexpr int kNN = " << sp.nn << ";\n"
      << "  static constexpr bool kInlineEmit = false;\n"
      << "  static constexpr bool kLdsProgram = false;\n";
    // backward: x = (T[a] + Ibl) + IL[k]  (non-taps: 0 + Ibl == Ibl bit for bit, Ibl is
    // never -0), Ib[k] = x; a separator folded in: T[p] = T[p] + x, Ibl = 0
    o << "  __device__ static __forceinline__ void s1(char *L, uint32_t lane_off, const SeqBw *, int, cx &ibl) {\n"
      << "    double2 *B = (double2 *)(L + lane_off);\n";
    const int nbw = (int)sp.bw.size();
    for (int c0 = 0; c0 < nbw; c0 += kChunk) {
        const int c1 = std::min(nbw, c0 + kChunk);
        o << "    {\n";
        std::vector<int> tw;   // T slots written so far in this chunk
        std::vector<char> ta_early(c1 - c0, 0), tp_early(c1 - c0, 0);
        for (int i = c0; i < c1; ++i) {
            const auto &op = sp.bw[i];
            o << "      const double2 w" << i - c0 << " = B[" << W(op[0]) << "];\n";
            if (op[1] >= 0 && std::find(tw.begin(), tw.end(), op[1]) == tw.end()) {
                ta_early[i - c0] = 1;
                o << "      const double2 a" << i - c0 << " = B[" << T(op[1]) << "];\n";
            }
            if (op[2] >= 0 && std::find(tw.begin(), tw.end(), op[2]) == tw.end()) {
                tp_early[i - c0] = 1;
                o << "      const double2 p" << i - c0 << " = B[" << T(op[2]) << "];\n";
            }
            if (op[2] >= 0) tw.push_back(op[2]);
        }
        for (int i = c0; i < c1; ++i) {
            const auto &op = sp.bw[i];
            const int j = i - c0;
            o << "      {";
            if (op[1] >= 0) {
                if (ta_early[j]) o << " const double2 t_ = a" << j << ";";
                else o << " const double2 t_ = B[" << T(op[1]) << "];";
                o << " const cx x = cadd(cadd(mk(t_.x, t_.y), ibl), mk(w" << j << ".x, w" << j << ".y));";
            } else {
                o << " const cx x = cadd(ibl, mk(w" << j << ".x, w" << j << ".y));";
            }
            o << " B[" << W(op[0]) << "] = make_double2(x.re, x.im);";
            if (op[2] >= 0) {
                if (tp_early[j]) o << " const double2 q_ = p" << j << ";";
                else o << " const double2 q_ = B[" << T(op[2]) << "];";
                o << " B[" << T(op[2]) << "] = make_double2(q_.x + x.re, q_.y + x.im); ibl = mk(0, 0); }\n";
            } else {
                o << " ibl = x; }\n";
            }
        }
        o << "    }\n";
    }
    o << "  }\n";
    // forward: V[dst] = V[src] - drop[dst], phases in mask zeroed
    o << "  __device__ static __forceinline__ void s2(char *L, uint32_t lane_off, const SeqFw *, int, int qp) {\n"
      << "    double2 *B = (double2 *)(L + lane_off);\n    cx v = mk(0, 0);\n";
    const int nfw = (int)sp.fw.size();
    int prev = -1;
    for (int c0 = 0; c0 < nfw; c0 += kChunk) {
        const int c1 = std::min(nfw, c0 + kChunk);
        o << "    {\n";
        std::vector<int> written;
        std::vector<char> s_early(c1 - c0, 0), s_prev(c1 - c0, 0);
        int pv = prev;
        for (int i = c0; i < c1; ++i) {
            const auto &op = sp.fw[i];
            o << "      const double2 d" << i - c0 << " = B[" << W(op[0]) << "];\n";
            if (op[1] != 0 && op[1] == pv) {
                s_prev[i - c0] = 1;
            } else if (std::find(written.begin(), written.end(), op[1]) == written.end()) {
                s_early[i - c0] = 1;
                o << "      const double2 s" << i - c0 << " = B[" << W(op[1]) << "];\n";
            }
            written.push_back(op[0]);
            pv = op[0];
        }
        for (int i = c0; i < c1; ++i) {
            const auto &op = sp.fw[i];
            const int j = i - c0;
            o << "      {";
            if (s_early[j]) o << " v = mk(s" << j << ".x, s" << j << ".y);";
            else if (!s_prev[j]) o << " { const double2 s_ = B[" << W(op[1]) << "]; v = mk(s_.x, s_.y); }";
            o << " v = csub(v, mk(d" << j << ".x, d" << j << ".y));";
            if (op[2]) o << " if ((" << op[2] << " >> qp) & 1) v = mk(0, 0);";
            o << " B[" << W(op[0]) << "] = make_double2(v.re, v.im); }\n";
            prev = op[0];
        }
        o << "    }\n";
    }
    o << "  }\n};\n}  // namespace fpf\n"
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
