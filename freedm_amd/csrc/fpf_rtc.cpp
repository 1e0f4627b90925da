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

#include <dlfcn.h>
#include <unistd.h>
#include <elf.h>

#include <algorithm>
#include <array>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cctype>
#include <cstring>
#include <type_traits>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

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
// one code object per (device, source), shared by the feeders that compile the
// same topology; unloaded when the last of them is destroyed (rtc_release)
struct RtcEntry {
    RtcKernel k;
    int refs;
};
std::map<std::pair<int, std::string>, RtcEntry> g_cache;

// The sequential stages as one straight-line instruction stream that runs the
// feeder's multi-track schedule (fpf_internal.h: TrackSched): at step s every
// lane of track t executes the op of cell (s, t).  Because node k's state lives
// in slot base[s] + t, the slot of step s is B + OFF(s) for every track, with
// B = L + lane_off + t*slot per lane -- one LDS read, 1-2 dependent complex adds
// and one LDS write per step serve all T tracks.  A track idle at a step reads
// whatever its comb position holds and does not store (its position may be
// another step's cell).
//
// Along a block the chain value (Ibl backward, V forward) stays in a register.
// Values crossing tracks -- a lateral's source voltage V(tap) forward, the
// child-block currents a tap accumulates backward -- go through LDS: the
// producing lane writes its slot, the consuming lane reads it at a track-relative
// offset, later in the same wave's program order (LDS executes a wave's
// operations in order; a wavefront-scope fence keeps the compiler from hoisting
// the read above the write).  Per-track differences (which lanes take a
// cross-track operand, reset Ibl, zero a phase) are compile-time constants
// tested against the lane's track.
//
// Arithmetic is the reference's (DPF_return7.cpp:134-195), so V stays
// bit-identical.  Zero folding (exact): Ibl, Ib and tap sums are never -0
// (each is a sum with an IL term; x + y == -0 needs both -0), so 0 + Ibl == Ibl
// and T + 0 == T bit for bit; a fresh Ibl (+0) plus IL keeps its add because IL
// may be -0.
std::string gen_program(const RtcSpec &sp) {
    const TrackSched &ts = sp.ts;
    const int T = ts.T, S = ts.S, A = std::max(1, sp.ahead);
    const long SL = sp.slot > 0 ? sp.slot : 3L * sp.tile;         // double2 per slot
    const long PS = sp.ps > 0 ? sp.ps : sp.tile;                   // double2 per phase
    auto OFF = [&](int s) { return (long)ts.base[s] * SL; };       // this step's cell, relative to B
    auto XOFF = [&](int node, int tcons) { return (long)(ts.slot(node) - tcons) * SL; };
    const unsigned all_tracks = (1u << T) - 1;
    auto cell = [&](int s, int t) { return ts.cell[(size_t)s * T + t]; };
    // a scheduling barrier after every step keeps the LDS reads where they are
    // placed (A steps ahead) instead of letting the scheduler hoist them all
    const char *sb_env = getenv("FPF_RTC_SCHEDBAR");
    const std::string sbar = (!sb_env || atoi(sb_env)) ? "    __builtin_amdgcn_sched_barrier(0);\n" : "";
    std::ostringstream o;
    o << "namespace fpf {\nstruct GenProg {\n"
      << "  static constexpr int kTile = " << sp.tile << ";\n"
      << "  static constexpr int kNN = " << sp.nn << ";\n"
      << "  static constexpr int kTracks = " << T << ";\n"
      << "  static constexpr int kNs = " << sp.ns << ";\n"
      << "  static constexpr int kSlots = " << ts.n_slots << ";\n"
      << "  static constexpr int kSlotBytes = " << SL * 16 << ";\n"
      << "  static constexpr int kPhaseBytes = " << PS * 16 << ";\n"
      << "  static constexpr bool kKeepIb = " << (sp.keep_ib ? "true" : "false") << ";\n"
      << "  static constexpr bool kExact = " << (sp.exact ? "true" : "false") << ";\n"
      << "  static constexpr bool kTempLds = " << (sp.temp_lds ? "true" : "false") << ";\n"
      << "  static constexpr bool kFullK = " << (sp.full_k ? "true" : "false") << ";\n"
      << "  static constexpr long kStagger = " << sp.stagger << ";\n"
      << "  static constexpr int kStaggerShift = " << sp.stagger_shift << ";\n"
      << "  static constexpr short kSlotOf[" << sp.nn << "] = {";
    for (int k = 0; k < sp.nn; ++k) o << (k ? ", " : "") << ts.slot(k);
    o << "};\n"
      << "  __device__ static __forceinline__ int node_slot(const FeederDev &, int k) { return kSlotOf[k]; }\n"
      << "  static constexpr bool kLdsProgram = false;\n"
      << "  static constexpr bool kLdsTaps = false;\n"
      << "  __device__ static __forceinline__ cx ld(const double2 *B, long i) { const double2 v = B[i]; return mk(v.x, v.y); }\n"
      << "  __device__ static __forceinline__ void st(double2 *B, long i, cx v) { B[i] = make_double2(v.re, v.im); }\n"
      << "  __device__ static __forceinline__ void xfence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, \"wavefront\"); }\n";

    // reads to emit at each execution index: (text, needs fence)
    struct Rd { std::string text; bool cross; };

    // ---------------- forward (:163-195), execution index e = step s
    {
        std::vector<std::vector<Rd>> reads(S);
        auto place = [&](int want, int after, const std::string &txt, bool cross) {
            int e = std::max(0, want);
            if (after >= 0) e = std::max(e, after + 1);
            reads[std::min(e, S - 1)].push_back({txt, cross});
        };
        for (int s = 0; s < S; ++s) {
            place(s - A, -1, "const cx d" + std::to_string(s) + " = ld(B, " + std::to_string(OFF(s)) + ");", false);
            for (int t = 0; t < T; ++t) {
                const int k = cell(s, t);
                if (k < 0) continue;
                const int src = ts.fw_src[k];
                const bool prev = s > 0 && src != 0 && cell(s - 1, t) == src;
                if (prev) continue;
                const std::string nm = "xs" + std::to_string(s) + "_" + std::to_string(t);
                if (src == 0) {   // V0: slots 0..T-1, offset 0 from every track's B
                    place(s - A, -1, "const cx " + nm + " = ld(B, 0);", false);
                } else {
                    place(s - A, ts.step[src], "const cx " + nm + " = ld(B, " + std::to_string(XOFF(src, t)) + ");", true);
                }
            }
        }
        o << "  __device__ static __forceinline__ void s2(char *L, uint32_t, uint32_t vbase, int trk, int qp, const SeqFw *, int) {\n"
          << "    double2 *B = (double2 *)(L + vbase);\n"
          << "    cx vp = mk(0, 0);\n";
        for (int s = 0; s < S; ++s) {
            bool fenced = false;
            for (const Rd &r : reads[s]) {
                if (r.cross && !fenced) { o << "    xfence();\n"; fenced = true; }
                o << "    " << r.text << "\n";
            }
            o << "    { cx vin = vp;";
            for (int t = 0; t < T; ++t) {
                const int k = cell(s, t);
                if (k < 0) continue;
                const int src = ts.fw_src[k];
                const bool prev = s > 0 && src != 0 && cell(s - 1, t) == src;
                if (!prev) o << " if (trk == " << t << ") vin = xs" << s << "_" << t << ";";
            }
            o << " cx v = csub(vin, d" << s << ");";
            for (int t = 0; t < T; ++t) {
                const int k = cell(s, t);
                if (k >= 0 && ts.fw_mask[k])
                    o << " if (trk == " << t << " && ((" << ts.fw_mask[k] << " >> qp) & 1)) v = mk(0, 0);";
            }
            if (ts.active[s] == all_tracks) o << " st(B, " << OFF(s) << ", v);";
            else o << " if ((" << ts.active[s] << "u >> trk) & 1u) st(B, " << OFF(s) << ", v);";   // idle cells alias other slots
            o << " vp = v; }\n" << sbar;
        }
        o << "  }\n";
    }

    // ---------------- backward (:134-160), execution index e = S-1-s
    {
        std::vector<std::vector<Rd>> reads(S);
        auto place = [&](int want, int after, const std::string &txt, bool cross) {
            int e = std::max(0, want);
            if (after >= 0) e = std::max(e, after + 1);
            reads[std::min(e, S - 1)].push_back({txt, cross});
        };
        for (int e = 0; e < S; ++e) {
            const int s = S - 1 - e;
            place(e - A, -1, "const cx il" + std::to_string(s) + " = ld(B, " + std::to_string(OFF(s)) + ");", false);
            for (int t = 0; t < T; ++t) {
                const int k = cell(s, t);
                if (k < 0) continue;
                const auto &ch = ts.children[k];
                for (size_t j = 0; j < ch.size(); ++j) {
                    const int c = ch[j];
                    const int prod = S - 1 - ts.step[c];
                    place(e - A, prod,
                          "const cx ch" + std::to_string(s) + "_" + std::to_string(t) + "_" + std::to_string(j) +
                              " = ld(B, " + std::to_string(XOFF(c, t)) + ");",
                          true);
                }
            }
        }
        o << "  __device__ static __forceinline__ void s1(char *L, uint32_t, uint32_t vbase, int trk, int, const SeqBw *, int) {\n"
          << "    double2 *B = (double2 *)(L + vbase);\n"
          << "    cx ibl = mk(0, 0);\n";
        for (int e = 0; e < S; ++e) {
            const int s = S - 1 - e;
            bool fenced = false;
            for (const Rd &r : reads[e]) {
                if (r.cross && !fenced) { o << "    xfence();\n"; fenced = true; }
                o << "    " << r.text << "\n";
            }
            unsigned rmask = 0;
            for (int t = 0; t < T; ++t) {
                const int k = cell(s, t);
                if (k >= 0 && ts.bw_reset[k]) rmask |= 1u << t;
            }
            o << "    { cx a = ibl;";
            if (rmask == (1u << T) - 1) o << " a = mk(0, 0);";
            else if (rmask) o << " if ((" << rmask << "u >> trk) & 1u) a = mk(0, 0);";
            o << " cx x = cadd(a, il" << s << ");";
            for (int t = 0; t < T; ++t) {
                const int k = cell(s, t);
                if (k < 0 || ts.children[k].empty()) continue;
                const std::string pre = "ch" + std::to_string(s) + "_" + std::to_string(t) + "_";
                o << " { cx tsum = " << pre << "0;";
                for (size_t j = 1; j < ts.children[k].size(); ++j) o << " tsum = cadd(tsum, " << pre << j << ");";
                o << " if (trk == " << t << ") x = cadd(cadd(tsum, a), il" << s << "); }";
            }
            if (ts.active[s] == all_tracks) o << " st(B, " << OFF(s) << ", x);";
            else o << " if ((" << ts.active[s] << "u >> trk) & 1u) st(B, " << OFF(s) << ", x);";
            o << " ibl = x; }\n" << sbar;
        }
        o << "  }\n";
    }
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

namespace {
// ---- which hipRTC compiles.  A process that imported PyTorch before this
// library (the Python mirror, bench.py, the GPU tests) has PyTorch's bundled
// HIP runtime, libhiprtc and libamd_comgr (ROCm 7.0) loaded under the same
// sonames, so the linked hiprtc* symbols resolve to that older compiler.  It
// builds the wave kernel with 32 AGPRs on top of the VGPRs the launch bounds
// allow (264 registers for a 512-thread workgroup, i.e. 2 waves per SIMD x 264
// > 512): the workgroup can never be resident, and the command processor
// rejects the dispatch (EC_QUEUE_PACKET_DISPATCH_REGISTER_INVALID, reported as
// HSA_STATUS_ERROR_INVALID_ISA -- profiles/r04rtc, profiles/r05rtc).  So the
// image's own hipRTC (the compiler the static kernels were built with) is
// loaded into a private link-map namespace (dlmopen), where its dlopen of
// comgr finds the image's comgr next to it instead of the process's.  The
// linked symbols remain the fallback; every build is checked for residency
// (rtc_resident) either way.
struct RtcApi {
    decltype(&hiprtcCreateProgram) create;
    decltype(&hiprtcAddNameExpression) add_name;
    decltype(&hiprtcCompileProgram) compile;
    decltype(&hiprtcGetProgramLogSize) log_size;
    decltype(&hiprtcGetProgramLog) log;
    decltype(&hiprtcGetLoweredName) lowered;
    decltype(&hiprtcGetCodeSize) code_size;
    decltype(&hiprtcGetCode) code;
    decltype(&hiprtcDestroyProgram) destroy;
    decltype(&hiprtcGetErrorString) errstr;
    std::string where;   // the library the entry points came from
    // the private namespace has its own libc, whose environ still points at the
    // array the process had when it was loaded; a setenv since then may have
    // freed that array (comgr reads its environment on every compile), so it is
    // pointed at the process's current one before each compile (sync_env)
    char ***ns_environ = nullptr;
    void sync_env() const {
        if (ns_environ) *ns_environ = environ;
    }
};

const RtcApi &rtc_api() {
    static const RtcApi api = [] {
        RtcApi a{&hiprtcCreateProgram, &hiprtcAddNameExpression, &hiprtcCompileProgram, &hiprtcGetProgramLogSize,
                 &hiprtcGetProgramLog, &hiprtcGetLoweredName, &hiprtcGetCodeSize, &hiprtcGetCode,
                 &hiprtcDestroyProgram, &hiprtcGetErrorString, "linked"};
        std::vector<std::string> cands;
        if (const char *e = getenv("FPF_HIPRTC_LIB")) {
            if (!*e || !strcmp(e, "linked")) return a;   // (diagnostics: the process's own hiprtc)
            cands.push_back(e);
        }
        if (const char *r = getenv("ROCM_PATH")) cands.push_back(std::string(r) + "/lib/libhiprtc.so");
        cands.push_back("/opt/rocm/lib/libhiprtc.so");
        for (const std::string &p : cands) {
            void *h = dlmopen(LM_ID_NEWLM, p.c_str(), RTLD_NOW | RTLD_LOCAL);
            if (!h) continue;
            RtcApi b = a;
            bool ok = true;
            auto get = [&](auto &fn, const char *sym) {
                void *s = dlsym(h, sym);
                if (!s) ok = false;
                else fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(s);
            };
            get(b.create, "hiprtcCreateProgram");
            get(b.add_name, "hiprtcAddNameExpression");
            get(b.compile, "hiprtcCompileProgram");
            get(b.log_size, "hiprtcGetProgramLogSize");
            get(b.log, "hiprtcGetProgramLog");
            get(b.lowered, "hiprtcGetLoweredName");
            get(b.code_size, "hiprtcGetCodeSize");
            get(b.code, "hiprtcGetCode");
            get(b.destroy, "hiprtcDestroyProgram");
            get(b.errstr, "hiprtcGetErrorString");
            b.ns_environ = static_cast<char ***>(dlsym(h, "environ"));
            if (!b.ns_environ) ok = false;
            if (ok) {
                b.where = p;
                return b;
            }
            dlclose(h);
        }
        return a;
    }();
    return api;
}

// the compiled code object's kernel descriptor (AMDHSA ABI): registers per
// lane (VGPRs + AGPRs, COMPUTE_PGM_RSRC1 granule 8 on gfx950) and the fixed
// private segment; false if the object has no such kernel
bool co_kernel_desc(const std::string &co, const std::string &kname, int *regs, int *scratch, int *group = nullptr) {
    const auto *eh = reinterpret_cast<const Elf64_Ehdr *>(co.data());
    if (co.size() < sizeof(Elf64_Ehdr) || memcmp(eh->e_ident, ELFMAG, SELFMAG) || eh->e_shoff + (size_t)eh->e_shnum *
        sizeof(Elf64_Shdr) > co.size())
        return false;
    const auto *sh = reinterpret_cast<const Elf64_Shdr *>(co.data() + eh->e_shoff);
    const std::string kd = kname + ".kd";
    for (int i = 0; i < eh->e_shnum; ++i) {
        if (sh[i].sh_type != SHT_SYMTAB && sh[i].sh_type != SHT_DYNSYM) continue;
        const Elf64_Shdr &st = sh[sh[i].sh_link];
        const auto *sym = reinterpret_cast<const Elf64_Sym *>(co.data() + sh[i].sh_offset);
        for (size_t j = 0; j < sh[i].sh_size / sizeof(Elf64_Sym); ++j) {
            if (sym[j].st_name >= st.sh_size || kd != co.data() + st.sh_offset + sym[j].st_name) continue;
            const Elf64_Shdr &sec = sh[sym[j].st_shndx];
            const size_t off = sec.sh_offset + (sym[j].st_value - sec.sh_addr);
            if (off + 64 > co.size()) return false;
            uint32_t rsrc1, pss, gss;
            memcpy(&gss, co.data() + off + 0, 4);     // kernel_descriptor_t: +0 group, +4 private segment
            memcpy(&pss, co.data() + off + 4, 4);
            memcpy(&rsrc1, co.data() + off + 48, 4);  // +48 compute_pgm_rsrc1
            *regs = ((int)(rsrc1 & 63) + 1) * 8;
            *scratch = (int)pss;
            if (group) *group = (int)gss;
            return true;
        }
    }
    return false;
}

// compile src for gfx950: the code object and the lowered kernel name (fname,
// or, given name_expr -- a template instantiation -- its lowered name)
int compile_co(const std::string &src, const char *file, const char *fname, const char *name_expr,
               std::vector<const char *> opts, std::string *code, std::string *lowered, std::string *err) {
    const RtcApi &R = rtc_api();
    static std::mutex env_mu;   // (one compile at a time reads the synced environment)
    std::lock_guard<std::mutex> elk(env_mu);
    R.sync_env();
    hiprtcProgram prog;
    if (R.create(&prog, src.c_str(), file, 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        *err = "hiprtcCreateProgram failed";
        return -1;
    }
    if (name_expr && R.add_name(prog, name_expr) != HIPRTC_SUCCESS) {
        R.destroy(&prog);
        *err = "hiprtcAddNameExpression failed";
        return -1;
    }
    opts.insert(opts.begin(), {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17"});
    hiprtcResult rr = R.compile(prog, (int)opts.size(), opts.data());
    if (rr != HIPRTC_SUCCESS) {
        size_t n = 0;
        R.log_size(prog, &n);
        std::string log(n, '\0');
        if (n) R.log(prog, &log[0]);
        *err = std::string("hipRTC compile failed: ") + R.errstr(rr) + "\n" + log.substr(0, 4000);
        R.destroy(&prog);
        return -1;
    }
    *lowered = fname ? fname : "";
    if (name_expr) {
        const char *low = nullptr;
        if (R.lowered(prog, name_expr, &low) != HIPRTC_SUCCESS || !low) {
            R.destroy(&prog);
            *err = "hiprtcGetLoweredName failed";
            return -1;
        }
        *lowered = low;
    }
    size_t n = 0;
    R.code_size(prog, &n);
    code->assign(n, '\0');
    R.code(prog, &(*code)[0]);
    R.destroy(&prog);
    return 0;
}

// can a workgroup of nt threads be resident at all: its waves share a CU's 4
// SIMDs, each with 512 registers per lane, and its static LDS (the descriptor's
// group segment) fits the CU's 160 KiB.  max_priv >= 0 (the hot per-plan wave
// builds, which exist to be faster than the static kernel): a private segment
// above max_priv bytes per lane is declined too -- the static kernel runs instead
// of a build that spills its sweep state.  (The light builds' private segment
// is not zero: it holds the call frame of the guard's exact re-solve,
// g3_fixup_local, a non-inlined call -- 112 bytes on the 123-bus plan.)
constexpr int WAVE_RTC_MAX_PRIV = 256;
bool rtc_resident(const std::string &co, const std::string &kname, int nt, std::string *err, int max_priv = -1) {
    int regs = 0, scratch = 0, group = 0;
    if (!co_kernel_desc(co, kname, &regs, &scratch, &group)) {
        *err = "no kernel descriptor for " + kname;
        return false;
    }
    const int waves_per_simd = ((nt + 63) / 64 + 3) / 4;
    if (regs * waves_per_simd > 512) {
        *err = "the build needs " + std::to_string(regs) + " registers per lane: a workgroup of " +
               std::to_string(nt) + " threads cannot be resident (" + rtc_api().where + ")";
        return false;
    }
    if (group > 160 * 1024) {
        *err = "the build's static LDS (" + std::to_string(group) + " bytes) exceeds a CU's 160 KiB";
        return false;
    }
    if (max_priv >= 0 && scratch > max_priv) {
        *err = "the build spills (" + std::to_string(scratch) + " bytes of private segment per lane)";
        return false;
    }
    return true;
}

int load_co(const std::string &code, const std::string &lowered, RtcKernel *k, std::string *err) {
    if (hipModuleLoadData(&k->mod, code.data()) != hipSuccess) {
        *err = "hipModuleLoadData failed";
        return -1;
    }
    if (hipModuleGetFunction(&k->fn, k->mod, lowered.c_str()) != hipSuccess) {
        (void)hipModuleUnload(k->mod);
        *err = "hipModuleGetFunction failed";
        return -1;
    }
    return 0;
}

int compile_load(const std::string &src, const char *file, const char *fname, const char *name_expr,
                 std::vector<const char *> opts, int nt, RtcKernel *k, std::string *err) {
    std::string code, lowered;
    if (compile_co(src, file, fname, name_expr, std::move(opts), &code, &lowered, err) != 0) return -1;
    if (!rtc_resident(code, lowered, nt, err)) return -1;
    return load_co(code, lowered, k, err);
}
}  // namespace

extern "C" long fpf_rtc_compile(const char *src, const char *name_expr, int ilp, int *regs, char *buf,
                                size_t buf_size) {
    if (!src || !name_expr) return FPF_ERR_ARG;
    std::string code, lowered, err;
    std::vector<const char *> opts;
    if (ilp) opts = {"-mllvm", "-amdgpu-sched-strategy=iterative-ilp"};
    if (compile_co(src, "fpf_rtc_check.hip", nullptr, name_expr, opts, &code, &lowered, &err) != 0) {
        if (getenv("FPF_DEBUG")) fprintf(stderr, "fpf_rtc_compile: %s\n", err.c_str());
        return FPF_ERR_UNSUPPORTED;
    }
    if (regs) {
        int scratch = 0;
        if (!co_kernel_desc(code, lowered, regs, &scratch)) *regs = -1;
    }
    if (buf && buf_size) memcpy(buf, code.data(), std::min(buf_size, code.size()));
    return (long)code.size();
}

extern "C" const char *fpf_rtc_compiler(void) { return rtc_api().where.c_str(); }

extern "C" int fpf_rtc_resident(const char *code, size_t size, const char *kernel, int nt, int max_priv, int *regs,
                                int *group, int *priv) {
    if (!code || !kernel || nt < 1) return FPF_ERR_ARG;
    const std::string co(code, size);
    int r = 0, sc = 0, g = 0;
    if (!co_kernel_desc(co, kernel, &r, &sc, &g)) return FPF_ERR_ARG;
    if (regs) *regs = r;
    if (group) *group = g;
    if (priv) *priv = sc;
    std::string err;
    return rtc_resident(co, kernel, nt, &err, max_priv < 0 ? -1 : max_priv) ? 1 : 0;
}

int rtc_build(int device, const RtcSpec &sp, RtcKernel *out, std::string *err) {
    const std::string src = rtc_source(sp);
    auto key = std::make_pair(device, src);
    auto cached = [&] {
        auto it = g_cache.find(key);
        if (it == g_cache.end()) return false;
        ++it->second.refs;
        *out = it->second.k;
        return true;
    };
    {
        std::lock_guard<std::mutex> lk(g_mu);
        if (cached()) return 0;
    }
    // compiled without g_mu held (~seconds): other feeders' builds, releases and
    // the wave kernels' cache lookups go on meanwhile
    RtcKernel k{};
#ifdef FPF_STAMPS
    if (compile_load(src, "fpf_rtc_tiled.hip", "fpf_rtc_tiled", nullptr, {"-DFPF_STAMPS"}, sp.nt, &k, err) != 0)
        return -1;
#else
    if (compile_load(src, "fpf_rtc_tiled.hip", "fpf_rtc_tiled", nullptr, {}, sp.nt, &k, err) != 0) return -1;
#endif
    k.nt = sp.nt;
    // dynamic LDS above the default 64 KiB (gfx950 has 160 KiB per CU)
    (void)hipFuncSetAttribute((const void *)k.fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    std::lock_guard<std::mutex> lk(g_mu);
    if (cached()) {   // another thread built the same source meanwhile: keep one module
        (void)hipModuleUnload(k.mod);
        return 0;
    }
    g_cache[key] = RtcEntry{k, 1};
    *out = k;
    return 0;
}

// ---- the wave kernel (fpf_wave_body.h) and the wave-block kernel
// (fpf_wblk_body.h) per plan, FPF_WSPEC: the same source as
// the static build with the plan's uniform values defined as constants, so the
// arithmetic -- and every result -- is the static kernel's.  Measured -4 to -5 %
// kernel time on the 123-bus feeder (profiles/r04sp, r04rtc).
// build switches of the wave and wave-block kernels' per-plan builds (experiments): FPF_WAVE_RTC_DEFS
// = comma-separated FPF_WAVE_* macro names (fpf_wave_body.h, fpf_wblk_body.h), each defined as 1
std::string wave_rtc_defs(const WaveDev &w) {
    std::string out;
    const char *e = getenv("FPF_WAVE_RTC_DEFS");
    (void)w;
    if (!e) return out;
    std::string s(e);
    size_t a = 0;
    while (a < s.size()) {
        size_t b = s.find(',', a);
        if (b == std::string::npos) b = s.size();
        // NAME or NAME=digits
        const std::string item = s.substr(a, b - a);
        const size_t eq = item.find('=');
        const std::string nm = item.substr(0, eq), val = eq == std::string::npos ? "1" : item.substr(eq + 1);
        bool ok = nm.size() > 9 && nm.compare(0, 9, "FPF_WAVE_") == 0 && !val.empty();
        for (char ch : nm) ok = ok && (isupper((unsigned char)ch) || isdigit((unsigned char)ch) || ch == '_');
        for (char ch : val) ok = ok && isdigit((unsigned char)ch);
        if (ok) out += "#define " + nm + " " + val + "\n";
        a = b + 1;
    }
    return out;
}

std::string wave_rtc_source(const WaveDev &w, bool full, std::string *name) {
    std::ostringstream s;
    s << "#define FPF_WSPEC 1\n"
      << "#define FPF_WSPEC_NN " << w.nn << "\n#define FPF_WSPEC_NL " << w.nl << "\n#define FPF_WSPEC_NBLK " << w.nblk
      << "\n#define FPF_WSPEC_BDEPTH " << w.bdepth << "\n#define FPF_WSPEC_NCOMP " << w.ncomp
      << "\n#define FPF_WSPEC_TEMP_SYM " << w.temp_sym << "\n#define FPF_WSPEC_OFF_IN_X " << w.off_in_x
      << "\n#define FPF_WSPEC_STAGE_U " << w.stage_u << "\n#define FPF_WSPEC_OUT_U " << w.out_u
      << "\n#define FPF_WSPEC_STAGE_UW " << w.stage_uw << "\n#define FPF_WSPEC_OUT_UW " << w.out_uw
      << "\n#define FPF_WSPEC_HAS_MASK " << w.has_mask << "\n#define FPF_WSPEC_HAS_REL " << w.has_rel
      << "\n#define FPF_WSPEC_MXITR " << w.mxitr << "\n";
    s << wave_rtc_defs(w);
    char nm[96];
    if (w.wps) {   // the wave-block kernel (fpf_wblk_body.h); full: its FULL variant
        s << "#define FPF_WSPEC_NCODE " << w.ncode << "\n";
        for (const char *part : kRtcWblkSources) s << part;
        snprintf(nm, sizeof nm, "fpf::dpf_wblk_kernel<%d, %s, %d, %s>", w.wps, full || w.has_rel ? "true" : "false", w.C,
                 w.has_rel ? "true" : "false");
    } else {
        for (const char *part : kRtcWaveSources) s << part;
        snprintf(nm, sizeof nm, "fpf::dpf_wave_kernel<%d, %d, %s, %d>", w.spw, w.C, full ? "true" : "false", w.wpb);
    }
    s << "\ntemplate __global__ void " << nm << "(fpf::WaveDev, int, const double *, fpf::OutDev);\n";
    *name = nm;
    return s.str();
}

// launches of at least this many scenarios run the per-plan build: the
// large-batch geometry (4-wave workgroups of the wave kernel, fpf_api.cpp:
// WAVE_SMALL_WPB_MIN_SCEN) and the wave-block kernel's batches -- config 4 0.908 ->
// 0.863 ms, config 3 10.08 -> 9.72 ms (profiles/r05rtc), config 2 38.9-39.2 ->
// 37.3 us with the 4-wave geometry (profiles/r05wio; the 8-wave geometry's build
// measured slower, 38.1 -> 39.4 us).  FPF_WAVE_RTC=n sets the threshold, 0 turns
// the per-plan builds off (read per call: tests switch it)
constexpr int WAVE_RTC_DEFAULT_MIN = 4096;
int wave_rtc_min() {
    const char *e = getenv("FPF_WAVE_RTC");
    if (e && *e) return atoi(e) == 0 ? INT32_MAX : (atoi(e) == 1 ? 1 : atoi(e));
    return WAVE_RTC_DEFAULT_MIN;
}

int g_wave_rtc_builds = 0;   // successful builds in this process (fpf_wave_rtc_builds)

hipFunction_t wave_rtc_function(int device, const WaveDev &w, bool full) {
    // every launch looks its build up: by the plan values the source is made of
    // (forming the ~300 KB source and comparing it as the key cost ~10 us a launch),
    // then, for a plan not seen yet, by the source itself
    // (the key's fields are every value wave_rtc_source writes into the source --
    // FPF_WSPEC_* and the template arguments -- plus the scheduler switch and the
    // FPF_WAVE_RTC_DEFS text itself; keep it in step with wave_rtc_source)
    typedef std::array<int32_t, 23> PlanKey;
    const char *se0 = getenv(w.wps ? "FPF_WBLK_RTC_SCHED" : "FPF_WAVE_RTC_SCHED");
    const PlanKey pk0 = {device, (int)full, w.nn, w.nl, w.nblk, w.bdepth, w.ncomp, w.temp_sym, w.off_in_x, w.stage_u,
                         w.out_u, w.stage_uw, w.out_uw, w.has_mask, w.has_rel, w.mxitr, w.ncode, w.wps, w.spw, w.C,
                         w.wpb, se0 ? atoi(se0) : -1, 0};
    const std::pair<PlanKey, std::string> pk(pk0, wave_rtc_defs(w));
    static std::map<std::pair<PlanKey, std::string>, hipFunction_t> by_plan;
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = by_plan.find(pk);
        if (it != by_plan.end()) return it->second;
    }
    const hipFunction_t fn = wave_rtc_function_src(device, w, full);
    std::lock_guard<std::mutex> lk(g_mu);
    by_plan[pk] = fn;
    return fn;
}

hipFunction_t wave_rtc_function_src(int device, const WaveDev &w, bool full) {
    std::string name;
    const std::string src = wave_rtc_source(w, full, &name);
    static std::map<std::pair<int, std::string>, hipFunction_t> built;   // NULL: the build failed
    static std::mutex build_mu;   // one compile at a time; g_mu is not held across it
    const auto key = std::make_pair(device, src);
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = built.find(key);
        if (it != built.end()) return it->second;
    }
    std::lock_guard<std::mutex> blk(build_mu);
    {
        std::lock_guard<std::mutex> lk(g_mu);   // (another thread may have built it meanwhile)
        auto it = built.find(key);
        if (it != built.end()) return it->second;
    }
    RtcKernel k{};
    std::string err, code, lowered;
    hipFunction_t fn = nullptr;
    // the static build's ILP-first scheduler (Makefile: fpf_wave.o / fpf_wblk.o);
    // FPF_WAVE_RTC_SCHED / FPF_WBLK_RTC_SCHED = 0: the default one (experiments)
    const char *se = getenv(w.wps ? "FPF_WBLK_RTC_SCHED" : "FPF_WAVE_RTC_SCHED");
    std::vector<const char *> opts;
    if (!(se && atoi(se) == 0)) opts = {"-mllvm", "-amdgpu-sched-strategy=iterative-ilp"};
    const int nt = 64 * (w.wps ? w.wps : w.wpb);
    if (compile_co(src, "fpf_rtc_wave.hip", nullptr, name.c_str(), opts, &code, &lowered, &err) == 0 &&
        rtc_resident(code, lowered, nt, &err, full ? -1 : WAVE_RTC_MAX_PRIV) && load_co(code, lowered, &k, &err) == 0) {
        int stat = 0;
        if (hipFuncGetAttribute(&stat, HIP_FUNC_ATTRIBUTE_SHARED_SIZE_BYTES, k.fn) == hipSuccess &&
            hipFuncSetAttribute((const void *)k.fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024 - stat) ==
                hipSuccess)
            fn = k.fn;
        else
            err = "hipFuncSetAttribute failed";
    }
    if (!fn && getenv("FPF_DEBUG")) fprintf(stderr, "wave_rtc_function: %s (the static kernel runs)\n", err.c_str());
    std::lock_guard<std::mutex> lk(g_mu);
    if (fn) ++g_wave_rtc_builds;
    built[key] = fn;   // (the module stays loaded for the process)
    return fn;
}

extern "C" int fpf_wave_rtc_builds(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    return g_wave_rtc_builds;
}

void rtc_release(const RtcKernel &k) {
    if (!k.mod) return;
    std::lock_guard<std::mutex> lk(g_mu);
    for (auto it = g_cache.begin(); it != g_cache.end(); ++it)
        if (it->second.k.mod == k.mod) {
            if (--it->second.refs == 0) {
                (void)hipModuleUnload(it->second.k.mod);
                g_cache.erase(it);
            }
            return;
        }
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
