"""CPU tests of the drop-in boundary: libfreedm_pf builds for gfx950, loads, and
exports exactly the entry points include/freedm_pf.h declares; the header is
C89 and C++98-pedantic clean (the Broker compiles with -std=c++98,
Broker/CMakeLists.txt:55).  No compute call is made without a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HDR = os.path.join(ROOT, "include", "freedm_pf.h")


def declared_functions():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"\b(fpf_[a-z_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    from freedm_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "run __graft_entry__.build() first"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (fpf_\w+)", out))
    decl = declared_functions()
    assert decl, "no declarations parsed"
    assert set(decl) == exported, (set(decl) ^ exported)
    assert set(decl) == set(_lib.EXPORTS)


def test_library_loads_and_reports_abi():
    from freedm_amd import _lib
    L = ctypes.CDLL(_lib.LIB_PATH)
    assert L.fpf_abi_version() == 3
    o = _lib.FpfOpts()
    L.fpf_opts_default(ctypes.byref(o))
    assert (o.bkva, o.bkv, o.eps, o.mxitr) == (1000.0, 12.47, 1e-4, 20)
    assert o.vo_kv == 12.47 * 1.015 and (o.lb_v, o.ub_v) == (0.96, 1.05)


@pytest.mark.parametrize("cmd", [
    ["gcc", "-std=c89", "-pedantic", "-Wall", "-Werror", "-x", "c", "-fsyntax-only"],
    ["g++", "-std=c++98", "-pedantic", "-Wall", "-Werror", "-x", "c++", "-fsyntax-only"],
])
def test_header_is_c89_and_cxx98_clean(cmd, tmp_path):
    src = tmp_path / "use.c"
    src.write_text('#include "freedm_pf.h"\nint main(void){ fpf_opts o; fpf_opts_default(&o); return o.mxitr == 20 ? 0 : 1; }\n')
    subprocess.run(cmd + ["-I", os.path.join(ROOT, "include"), str(src)], check=True)


def test_struct_layouts_match_ctypes(tmp_path):
    from freedm_amd import _lib
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include "freedm_pf.h"\nint main(void){printf("%zu %zu %zu %zu %zu\\n",'
                   ' sizeof(fpf_opts), sizeof(fpf_feeder_info), sizeof(fpf_outputs), sizeof(fpf_aggregate),'
                   ' sizeof(fpf_line_search)); return 0;}\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [ctypes.sizeof(_lib.FpfOpts), ctypes.sizeof(_lib.FpfFeederInfo),
                   ctypes.sizeof(_lib.FpfOutputs), ctypes.sizeof(_lib.FpfAggregate), ctypes.sizeof(_lib.FpfLineSearch)]


def test_product_path_never_touches_the_oracle():
    # the oracle is test infrastructure only: nothing under freedm_amd/ may import, link or call it
    bad = ("import oracle", "from oracle", "libfpf_oracle", "ref_dpf", "np_dpf")
    for dirpath, _, files in os.walk(os.path.join(ROOT, "freedm_amd")):
        for fn in files:
            if fn.endswith((".py", ".cpp", ".hip", ".h", ".hpp")) or fn == "Makefile":
                txt = open(os.path.join(dirpath, fn), errors="ignore").read()
                for b in bad:
                    assert b not in txt, (fn, b)
