"""Register report of the hipRTC kernel libfreedm_pf generates for a feeder:
compiles the generated source offline for gfx950 (no GPU needed) and prints
.vgpr_count / .vgpr_spill_count / .sgpr_count / scratch of fpf_rtc_tiled.

    python tools/rtc_regs.py [nn] [--asm out.s]
Environment knobs are those of fpf_feeder_create (FPF_RTC_TRACKS, FPF_RTC_AHEAD,
FPF_RTC_GEOM)."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rtc_dump import rtc_source  # noqa: E402
from freedm_amd import demo_feeder, dl_new_feeder, synthetic_feeder  # noqa: E402


def compile_report(src, asm_out=None):
    with tempfile.TemporaryDirectory() as d:
        hip = os.path.join(d, "k.hip")
        s = asm_out or os.path.join(d, "k.s")
        open(hip, "w").write(src)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17",
                        "--cuda-device-only", "-S", "-x", "hip", "-include", "hip/hip_runtime.h", hip, "-o", s],
                       check=True, capture_output=True)
        a = open(s).read()
    get = lambda k: int(re.findall(rf"\.{k}:\s+(\d+)", a)[-1])  # noqa: E731
    return {k: get(k) for k in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "private_segment_fixed_size")}


if __name__ == "__main__":
    nn = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 123
    asm = sys.argv[sys.argv.index("--asm") + 1] if "--asm" in sys.argv else None
    f = {9: demo_feeder, 34: dl_new_feeder}.get(nn, lambda: synthetic_feeder(nn, nn))()
    print(compile_report(rtc_source(f), asm))
