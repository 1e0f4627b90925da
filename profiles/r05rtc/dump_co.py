import ctypes as C, sys, os
sys.path.insert(0, "/root/repo/tools"); sys.path.insert(0, "/root/repo")
from wave_rtc_dump import wave_rtc_source
from freedm_amd import synthetic_feeder
nn = int(sys.argv[1]); big = int(sys.argv[2]); full = int(sys.argv[3]); ilp = int(sys.argv[4]); out = sys.argv[5]
src = wave_rtc_source(synthetic_feeder(nn, nn), big, full)
open(out + ".hip", "w").write(src)
name = src.rsplit("template __global__ void ", 1)[1].split("(")[0]
R = C.CDLL("/opt/rocm/lib/libhiprtc.so")
prog = C.c_void_p()
assert R.hiprtcCreateProgram(C.byref(prog), src.encode(), b"fpf_rtc_wave.hip", 0, None, None) == 0
assert R.hiprtcAddNameExpression(prog, name.encode()) == 0
o = [b"--offload-arch=gfx950", b"-O3", b"-ffp-contract=off", b"-std=c++17"] + ([b"-mllvm", b"-amdgpu-sched-strategy=iterative-ilp"] if ilp else [])
opts = (C.c_char_p * len(o))(*o)
rc = R.hiprtcCompileProgram(prog, len(o), opts)
n = C.c_size_t(); R.hiprtcGetProgramLogSize(prog, C.byref(n)); log = C.create_string_buffer(n.value + 1); R.hiprtcGetProgramLog(prog, log)
assert rc == 0, log.value.decode()[-3000:]
R.hiprtcGetCodeSize(prog, C.byref(n)); buf = C.create_string_buffer(n.value); R.hiprtcGetCode(prog, buf)
open(out, "wb").write(buf.raw)
print(name, n.value)
