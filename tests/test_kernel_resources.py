"""Register-spill guard for the fast kernels (no device): the built objects'
code-object metadata (`.vgpr_spill_count`, read with the image's llvm-readelf)
for the wave and wave-block kernels.  Round 5 found the static light builds and
the full-output variants spilling 118-226 VGPRs after changes that looked
neutral in the per-plan builds; these bounds keep that from
coming back unnoticed.  Skipped when the objects or the tools are absent."""
import os
import re
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "freedm_amd", "lib")
LLVM = "/opt/rocm/lib/llvm/bin"


def _spills(obj):
    if not (os.path.exists(obj) and os.path.exists(f"{LLVM}/llvm-readelf")):
        pytest.skip("built objects or LLVM tools absent")
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run([f"{LLVM}/llvm-objcopy", "--dump-section=.hip_fatbin=" + fb, obj, os.path.join(d, "x")],
                       check=True, capture_output=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--input=" + fb,
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + co, "--unbundle"],
                       check=True, capture_output=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                               check=True).stdout
    out = {}
    for block in notes.split("  - .agpr_count")[1:]:
        n = re.search(r"\.name:\s+(\S+)", block)
        v = re.search(r"\.vgpr_spill_count:\s+(\d+)", block)
        if n and v:
            out[n.group(1)] = int(v.group(1))
    return out


def test_wave_kernel_spills():
    """Every geometry the default plan picks (spw x C = 4x1, 4x2, 2x2, 2x4, 1x4),
    light and full-output (each general path), at the workgroup sizes the plan
    uses for batches below the per-plan build's threshold (8 waves) -- at most 16
    VGPRs spilled (the 1-scenario 2-slot geometry is an experiment only)."""
    sp = _spills(os.path.join(LIB, "fpf_wave.o"))
    wave = {k: v for k, v in sp.items() if "dpf_wave_kernel" in k and "ILi1ELi2E" not in k}
    assert len(wave) >= 20, sorted(sp)
    bad = {k: v for k, v in wave.items() if v > 16 and "ELi8E" in k.split("ELb")[1][:6]}
    assert not bad, bad


def test_wave_block_kernel_spills():
    """The wave-block kernel's light variant and its lean full-output variant (a
    tree feeder without zeroed phases) spill nothing in the static build (4-slot
    geometry; the general full variants and the 8-slot experiment are not bounded)."""
    sp = _spills(os.path.join(LIB, "fpf_wblk.o"))
    lean = {k: v for k, v in sp.items() if "dpf_wblk_kernel" in k and "ELi4ELb0ELi0E" in k}
    assert len(lean) >= 6, sorted(sp)
    bad = {k: v for k, v in lean.items() if v > 0}
    assert not bad, bad
