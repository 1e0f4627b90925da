"""The topology-specialised kernel source that libfreedm_pf generates at
fpf_feeder_create compiles with hipRTC for gfx950 (no GPU needed: hipRTC is a
compiler; loading the code object is the GPU tests' job)."""
import ctypes as C
import os
import sys
import time

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _hiprtc():
    for p in ("/opt/rocm/lib/libhiprtc.so", "libhiprtc.so"):
        try:
            return C.CDLL(p)
        except OSError:
            continue
    pytest.skip("libhiprtc not available")


OPTS = [b"--offload-arch=gfx950", b"-O3", b"-ffp-contract=off", b"-std=c++17"]


@pytest.mark.parametrize("nn,tracks", [(9, 0), (123, 0), (123, 1), (123, 2), (123, 4)])
def test_rtc_source_compiles(nn, tracks, monkeypatch):
    if tracks:
        monkeypatch.setenv("FPF_RTC_TRACKS", str(tracks))
    from rtc_dump import rtc_source
    from freedm_amd import demo_feeder, synthetic_feeder
    f = demo_feeder() if nn == 9 else synthetic_feeder(nn, nn)
    src = rtc_source(f)
    assert "fpf_rtc_tiled" in src and "__launch_bounds__(" in src
    R = _hiprtc()
    prog = C.c_void_p()
    assert R.hiprtcCreateProgram(C.byref(prog), src.encode(), b"fpf_rtc.hip", 0, None, None) == 0
    opts = (C.c_char_p * len(OPTS))(*OPTS)
    t0 = time.time()
    rc = R.hiprtcCompileProgram(prog, len(OPTS), opts)
    n = C.c_size_t()
    R.hiprtcGetProgramLogSize(prog, C.byref(n))
    log = C.create_string_buffer(n.value + 1)
    R.hiprtcGetProgramLog(prog, log)
    assert rc == 0, log.value.decode(errors="replace")[-4000:]
    R.hiprtcGetCodeSize(prog, C.byref(n))
    assert n.value > 1000
    R.hiprtcDestroyProgram(C.byref(prog))
    assert time.time() - t0 < 120


def _compile(src, name, extra=()):
    R = _hiprtc()
    prog = C.c_void_p()
    assert R.hiprtcCreateProgram(C.byref(prog), src.encode(), b"fpf_rtc_wave.hip", 0, None, None) == 0
    assert R.hiprtcAddNameExpression(prog, name.encode()) == 0
    o = OPTS + list(extra)
    opts = (C.c_char_p * len(o))(*o)
    rc = R.hiprtcCompileProgram(prog, len(o), opts)
    n = C.c_size_t()
    R.hiprtcGetProgramLogSize(prog, C.byref(n))
    log = C.create_string_buffer(n.value + 1)
    R.hiprtcGetProgramLog(prog, log)
    assert rc == 0, log.value.decode(errors="replace")[-4000:]
    low = C.c_char_p()
    R.hiprtcGetLoweredName.argtypes = [C.c_void_p, C.c_char_p, C.POINTER(C.c_char_p)]
    assert R.hiprtcGetLoweredName(prog, name.encode(), C.byref(low)) == 0
    lowered = low.value.decode()
    R.hiprtcGetCodeSize(prog, C.byref(n))
    assert n.value > 1000
    R.hiprtcDestroyProgram(C.byref(prog))
    return lowered


@pytest.mark.parametrize("nn,big,full", [(9, 1, 0), (60, 0, 1), (123, 1, 0)])
def test_wave_rtc_source_compiles(nn, big, full):
    """The per-plan wave kernel (fpf_rtc.cpp: wave_rtc_source, fpf_wave_body.h
    under FPF_WSPEC) compiles with the static build's flags; its plan constants
    are the ones fpf_feeder_wave_plan reports."""
    from wave_rtc_dump import wave_rtc_source
    from freedm_amd import demo_feeder, synthetic_feeder
    from test_wave_plan import _plan
    f = demo_feeder() if nn == 9 else synthetic_feeder(nn, nn)
    src = wave_rtc_source(f, big, full)
    plan = _plan(f)
    assert f"#define FPF_WSPEC_NCOMP {plan['ncomp']}\n" in src
    assert f"#define FPF_WSPEC_NBLK {plan['nblk']}\n" in src
    assert f"#define FPF_WSPEC_NN {nn}\n" in src
    tail = src.rsplit("template __global__ void ", 1)[1]
    name = tail.split("(")[0]
    assert name.startswith(f"fpf::dpf_wave_kernel<{plan['spw']}, {plan['C']}, {'true' if full else 'false'},")
    lowered = _compile(src, name, [b"-mllvm", b"-amdgpu-sched-strategy=iterative-ilp"])
    assert lowered.startswith("_ZN3fpf15dpf_wave_kernelI")


@pytest.mark.parametrize("nn", [700, 2048])
def test_wblk_rtc_source_compiles(nn):
    """The per-plan wave-block kernel (fpf_wblk_body.h under FPF_WSPEC) compiles."""
    from wave_rtc_dump import wave_rtc_source
    from freedm_amd import synthetic_feeder
    src = wave_rtc_source(synthetic_feeder(nn, nn), 1, 0)
    assert f"#define FPF_WSPEC_NN {nn}\n" in src and "#define FPF_WSPEC_NCODE " in src
    name = src.rsplit("template __global__ void ", 1)[1].split("(")[0]
    assert name.startswith("fpf::dpf_wblk_kernel<")
    assert _compile(src, name, [b"-mllvm", b"-amdgpu-sched-strategy=iterative-ilp"]).startswith("_ZN3fpf15dpf_wblk_kernelI")


def test_wblk_two_slot_geometry_plan_and_source(monkeypatch):
    """The experimental wave-block geometry FPF_WBLK_C=2 (2 slots per
    lane, 16 wavefronts for 1025..2048 branches, per-plan build only -- measured
    slower on config 3): the plan and the per-plan source carry it, and the
    source compiles; the default plan is unchanged without the switch."""
    from wave_rtc_dump import wave_rtc_source
    from test_wave_plan import _plan
    from freedm_amd import synthetic_feeder
    f = synthetic_feeder(2048, 2048)
    assert (_plan(f)["C"], _plan(f)["wpb"]) == (4, 8)
    monkeypatch.setenv("FPF_WBLK_C", "2")
    p = _plan(f)
    assert (p["C"], p["wpb"]) == (2, 16)
    src = wave_rtc_source(f, 1, 0)
    name = src.rsplit("template __global__ void ", 1)[1].split("(")[0]
    assert name.startswith("fpf::dpf_wblk_kernel<16, false, 2,")
    assert _compile(src, name, [b"-mllvm", b"-amdgpu-sched-strategy=iterative-ilp"]).startswith("_ZN3fpf15dpf_wblk_kernelI")


def _notes(co: bytes) -> dict:
    import re
    import subprocess
    import tempfile
    exe = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not os.path.exists(exe):
        pytest.skip("llvm-readelf not available")
    with tempfile.NamedTemporaryFile(suffix=".co") as t:
        t.write(co)
        t.flush()
        txt = subprocess.run([exe, "--notes", t.name], capture_output=True, text=True, check=True).stdout
    return {k: int(re.findall(rf"\.{k}:\s+(\d+)", txt)[-1]) for k in ("agpr_count", "vgpr_count",
                                                                        "max_flat_workgroup_size")}


@pytest.mark.parametrize("big,full", [(0, 0), (1, 0), (0, 1)])
def test_wave_rtc_build_is_resident_with_torch_loaded(big, full):
    """Round 4's dispatch abort (HSA_STATUS_ERROR_INVALID_ISA, profiles/r04rtc):
    in a process that imported PyTorch first, the linked hiprtc* symbols are
    PyTorch's bundled (older) hipRTC/comgr, which built the 512-thread wave
    kernel with 32 AGPRs on top of its VGPRs -- 264 registers x 2 waves per SIMD
    > 512, a workgroup that can never be resident, so the command processor
    refused the dispatch.  The library now compiles with the image's own hipRTC
    (dlmopen, fpf_rtc.cpp: rtc_api): every build of the config-2 plan fits."""
    import torch  # noqa: F401  (the failing configuration: torch's HIP libraries loaded first)
    from wave_rtc_dump import wave_rtc_source
    from freedm_amd import _lib, synthetic_feeder
    L = _lib.load()
    assert L.fpf_rtc_compiler().decode().endswith("libhiprtc.so"), L.fpf_rtc_compiler()
    src = wave_rtc_source(synthetic_feeder(123, 123), big, full)
    name = src.rsplit("template __global__ void ", 1)[1].split("(")[0].encode()
    regs = C.c_int(0)
    n = L.fpf_rtc_compile(src.encode(), name, 1, C.byref(regs), None, 0)
    assert n > 1000
    buf = C.create_string_buffer(n)
    assert L.fpf_rtc_compile(src.encode(), name, 1, None, buf, n) == n
    md = _notes(buf.raw)
    waves_per_simd = -(-md["max_flat_workgroup_size"] // 256)
    assert md["agpr_count"] == 0, md
    assert -(-md["vgpr_count"] // 8) * 8 == regs.value, (md, regs.value)   # the descriptor the check reads
    assert regs.value * waves_per_simd <= 512, md


def test_rtc_compile_survives_setenv():
    """The private-namespace hipRTC has its own libc, whose environ was the
    process's array at load time: a setenv that reallocates the process's array
    freed it, and the next compile (comgr reads its environment) crashed -- the
    round-5 GPU test run died this way at its second plan (monkeypatch.setenv of
    FPF_WAVE_GEOM).  fpf_rtc.cpp syncs the namespace's environ before each compile."""
    from wave_rtc_dump import wave_rtc_source
    from freedm_amd import _lib, synthetic_feeder
    L = _lib.load()
    src = wave_rtc_source(synthetic_feeder(30, 30), 1, 0)
    name = src.rsplit("template __global__ void ", 1)[1].split("(")[0].encode()
    assert L.fpf_rtc_compile(src.encode(), name, 0, None, None, 0) > 1000
    added = [f"FPF_TEST_ENV_GROW_{i}" for i in range(200)]
    try:
        for k in added:   # (grows the process's environ array until it moves)
            os.environ[k] = "x" * 64
        assert L.fpf_rtc_compile(src.encode(), name, 0, None, None, 0) > 1000
    finally:
        for k in added:
            os.environ.pop(k, None)
    assert L.fpf_rtc_compile(src.encode(), name, 0, None, None, 0) > 1000


def test_wave_rtc_defs_switches(monkeypatch):
    """FPF_WAVE_RTC_DEFS (experiments): FPF_WAVE_* names become `#define NAME 1`,
    NAME=digits `#define NAME digits`, anything else is dropped; the switches are
    part of the source (and so of the per-plan build cache key); none by default."""
    from wave_rtc_dump import wave_rtc_source
    from freedm_amd import synthetic_feeder
    f = synthetic_feeder(123, 123)
    base = wave_rtc_source(f, 1, 0)
    assert "#define FPF_WAVE_GROUP 2\n" not in base and "#define FPF_WAVE_TEMP_LATE 1\n" not in base
    monkeypatch.setenv("FPF_WAVE_RTC_DEFS", "FPF_WAVE_GROUP=2,FPF_WAVE_TEMP_LATE,BOGUS=1,FPF_WAVE_X=abc,FPF_WAVE_Y=")
    src = wave_rtc_source(f, 1, 0)
    assert "#define FPF_WAVE_GROUP 2\n" in src and "#define FPF_WAVE_TEMP_LATE 1\n" in src
    assert "BOGUS" not in src and "#define FPF_WAVE_X " not in src and "#define FPF_WAVE_Y" not in src


def test_rtc_resident_checks_lds_and_scratch():
    """The residency check a per-plan build passes before it is loaded
    (fpf_rtc.cpp: rtc_resident): registers, the static LDS of the group segment
    (<= 160 KiB) and, for the hot light-output wave builds, a private segment of
    at most 256 bytes per lane -- the call frame of the guard's exact re-solve
    fits, a spilled sweep state does not (the build is declined and the static
    kernel runs).  The config-2 plan's light build passes; a kernel that spills a
    private array passes only without the bound."""
    from wave_rtc_dump import wave_rtc_source
    from freedm_amd import _lib, synthetic_feeder
    L = _lib.load()
    L.fpf_rtc_resident.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_int, C.c_int, C.POINTER(C.c_int),
                                   C.POINTER(C.c_int), C.POINTER(C.c_int)]
    L.fpf_rtc_resident.restype = C.c_int

    def build(src, name, ilp=0):
        n = L.fpf_rtc_compile(src.encode(), name, ilp, None, None, 0)
        assert n > 100
        buf = C.create_string_buffer(n)
        L.fpf_rtc_compile(src.encode(), name, ilp, None, buf, n)
        return buf.raw

    def check(co, kname, nt, max_priv):
        regs, group, priv = C.c_int(-1), C.c_int(-1), C.c_int(-1)
        low = next(s for s in _symbols(co) if kname in s)
        rc = L.fpf_rtc_resident(co, len(co), low.encode(), nt, max_priv, C.byref(regs), C.byref(group), C.byref(priv))
        return rc, regs.value, group.value, priv.value

    src = wave_rtc_source(synthetic_feeder(123, 123), 1, 0)
    name = src.rsplit("template __global__ void ", 1)[1].split("(")[0].encode()
    co = build(src, name, 1)
    rc, regs, group, priv = check(co, "dpf_wave_kernel", 256, 256)
    assert rc == 1 and 0 <= priv <= 256 and 0 < group <= 160 * 1024 and regs <= 256, (rc, regs, group, priv)
    spill = ("template <int N> __global__ void spill(double *o, const int *ix) {\n"
             "  double a[N]; for (int i = 0; i < N; ++i) a[i] = o[i * 7 + threadIdx.x];\n"
             "  __shared__ double s[64]; s[threadIdx.x & 63] = a[ix[threadIdx.x]];\n"
             "  __syncthreads(); o[threadIdx.x] = s[(threadIdx.x + 1) & 63]; }\n"
             "template __global__ void spill<512>(double *, const int *);\n")
    co2 = build(spill, b"spill<512>")
    rc2, _, group2, priv2 = check(co2, "spill", 64, 256)
    assert priv2 > 256 and rc2 == 0 and group2 >= 512, (rc2, group2, priv2)
    assert check(co2, "spill", 64, -1)[0] == 1


def _symbols(co):
    """The kernel symbols of a code object (their .kd descriptors, from the string table)."""
    import re
    return sorted({m.decode()[:-3] for m in re.findall(rb"_Z[A-Za-z0-9_]*\.kd", co)})
