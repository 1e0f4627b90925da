"""ctypes binding of libfreedm_pf (include/freedm_pf.h).

This is the same binding a maintainer would write for any FFI: plain pointers
and sizes, no torch types.  The library is built in-tree (freedm_amd/lib/) by
__graft_entry__.build() / `make -C freedm_amd/csrc`; there is no fallback --
if the library is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libfreedm_pf.so")

ABI_VERSION = 3   # include/freedm_pf.h FPF_ABI_VERSION
FPF_OK, FPF_ERR_ARG, FPF_ERR_TOPOLOGY, FPF_ERR_HIP, FPF_ERR_NOMEM, FPF_ERR_UNSUPPORTED = 0, -1, -2, -3, -4, -5
FPF_CONVERGED, FPF_NONCONVERGED = 0, 1
FPF_KERNEL_AUTO, FPF_KERNEL_GENERIC, FPF_KERNEL_TILED, FPF_KERNEL_WAVE = 0, 1, 2, 3
KERNELS = {"auto": FPF_KERNEL_AUTO, "generic": FPF_KERNEL_GENERIC, "tiled": FPF_KERNEL_TILED, "wave": FPF_KERNEL_WAVE}

EXPORTS = ["fpf_abi_version", "fpf_opts_default", "fpf_ctx_create", "fpf_ctx_destroy", "fpf_last_error",
           "fpf_feeder_create", "fpf_feeder_destroy", "fpf_feeder_get_info", "fpf_feeder_reserve",
           "fpf_solve_batch", "fpf_solve_batch_device", "fpf_aggregate_device", "fpf_feeder_rtc_source",
           "fpf_selftest_division", "fpf_vvc_line_search", "fpf_feeder_wave_plan",
           "fpf_multi_create", "fpf_multi_destroy", "fpf_multi_last_error", "fpf_multi_solve", "fpf_multi_get_feeder",
           "fpf_multi_shard", "fpf_multi_schedule", "fpf_aggregate_fold", "fpf_areas_create", "fpf_areas_destroy", "fpf_areas_last_error",
           "fpf_areas_info", "fpf_areas_solve", "fpf_vvc_gradient", "fpf_vvc_gradient_at", "fpf_vvc_round",
           "fpf_vvc_gradient_batch", "fpf_feeder_check", "fpf_vvc_round_batch", "fpf_feeder_wave_rtc_source",
           "fpf_wave_rtc_builds", "fpf_rtc_compile", "fpf_rtc_compiler", "fpf_feeder_lane_plan", "fpf_lane_launches", "fpf_lane_dma_launches",
           "fpf_rtc_resident", "fpf_multi_collectives"]


class FpfOpts(C.Structure):
    _fields_ = [("bkva", C.c_double), ("bkv", C.c_double), ("vo_kv", C.c_double), ("eps", C.c_double),
                ("mxitr", C.c_int), ("kernel", C.c_int), ("lb_v", C.c_double), ("ub_v", C.c_double),
                ("tile", C.c_int), ("specialize", C.c_int), ("exact", C.c_int), ("layout", C.c_int),
                ("no_guard", C.c_int), ("reserved", C.c_int * 3)]


class FpfFeederInfo(C.Structure):
    _fields_ = [("nl", C.c_int), ("ncols", C.c_int), ("nn", C.c_int), ("nb", C.c_int), ("n_codes", C.c_int),
                ("n_sep", C.c_int), ("n_taps", C.c_int), ("well_formed", C.c_int), ("lnum", C.c_int * 3),
                ("depth", C.c_int), ("kernel", C.c_int), ("tile", C.c_int), ("specialized", C.c_int),
                ("reserved", C.c_int * 3)]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k not in ("reserved", "lnum")}
        d["lnum"] = list(self.lnum)
        return d


_dp = C.POINTER(C.c_double)


class FpfOutputs(C.Structure):
    _fields_ = [("vpolar", C.c_void_p), ("pqb", C.c_void_p), ("pql", C.c_void_p), ("v_re", C.c_void_p),
                ("v_im", C.c_void_p), ("iters", C.c_void_p), ("status", C.c_void_p), ("loss", C.c_void_p),
                ("vmin", C.c_void_p), ("vmax", C.c_void_p), ("errmx", C.c_void_p), ("guard", C.c_void_p)]


class FpfAggregate(C.Structure):
    _fields_ = [("loss_sum", C.c_double), ("vmin", C.c_double), ("vmax", C.c_double), ("n_conv", C.c_double),
                ("n_nonconv", C.c_double), ("n_over", C.c_double), ("n_under", C.c_double),
                ("n_scen", C.c_double)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class FpfLineSearch(C.Structure):
    _fields_ = [("stop", C.c_int), ("reverse", C.c_int), ("first_nonconv", C.c_int), ("reserved", C.c_int),
                ("loss", C.c_void_p), ("vmin", C.c_void_p), ("vmax", C.c_void_p)]


_lib = None


def _preload_torch_runtime():
    """torch ships its own libamdhip64 (SONAME libamdhip64.so.7); loading torch
    first makes this library bind to that same HIP runtime instead of a second
    copy from /opt/rocm."""
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def load(path: str | None = None):
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("FPF_LIB_PATH") or LIB_PATH   # override: diagnostic builds only
    if not os.path.exists(path):
        raise RuntimeError(f"libfreedm_pf not built: {path} missing (run __graft_entry__.build() "
                           "or `make -C freedm_amd/csrc`); there is no CPU fallback")
    _preload_torch_runtime()
    L = C.CDLL(path)
    vp = C.c_void_p
    L.fpf_abi_version.restype = C.c_int
    L.fpf_opts_default.argtypes = [C.POINTER(FpfOpts)]
    L.fpf_opts_default.restype = None
    L.fpf_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.fpf_ctx_destroy.argtypes = [vp]
    L.fpf_ctx_destroy.restype = None
    L.fpf_last_error.argtypes = [vp]
    L.fpf_last_error.restype = C.c_char_p
    L.fpf_feeder_create.argtypes = [vp, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.POINTER(FpfOpts),
                                    C.POINTER(vp)]
    L.fpf_feeder_destroy.argtypes = [vp]
    L.fpf_feeder_destroy.restype = None
    L.fpf_feeder_get_info.argtypes = [vp, C.POINTER(FpfFeederInfo)]
    L.fpf_feeder_reserve.argtypes = [vp, C.c_int]
    L.fpf_solve_batch.argtypes = [vp, C.c_int, _dp, C.POINTER(FpfOutputs), C.POINTER(FpfAggregate)]
    L.fpf_solve_batch_device.argtypes = [vp, C.c_int, vp, C.POINTER(FpfOutputs), vp, vp]
    L.fpf_aggregate_device.argtypes = [vp, C.c_int, vp, vp, vp, vp, vp, vp]
    L.fpf_feeder_check.argtypes = [vp, vp]
    L.fpf_feeder_rtc_source.argtypes = [_dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.POINTER(FpfOpts),
                                        C.c_char_p, C.c_size_t]
    L.fpf_feeder_rtc_source.restype = C.c_long
    if hasattr(L, "fpf_feeder_wave_rtc_source"):   # (older diagnostic builds lack it)
        L.fpf_feeder_wave_rtc_source.argtypes = [_dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.POINTER(FpfOpts),
                                                 C.c_int, C.c_int, C.c_char_p, C.c_size_t]
        L.fpf_feeder_wave_rtc_source.restype = C.c_long
    L.fpf_vvc_line_search.argtypes = [vp, _dp, C.c_int, C.c_int, _dp, _dp, C.POINTER(C.c_int), C.c_int, C.c_double,
                                      C.c_double, C.c_int, C.c_double, C.POINTER(FpfLineSearch)]
    L.fpf_vvc_line_search.restype = C.c_int
    if hasattr(L, "fpf_feeder_wave_plan") or path == LIB_PATH:   # (older diagnostic builds lack it)
        L.fpf_feeder_wave_plan.argtypes = [_dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.POINTER(FpfOpts),
                                           C.POINTER(C.c_int)]
        L.fpf_feeder_wave_plan.restype = C.c_int
    if hasattr(L, "fpf_feeder_lane_plan") or path == LIB_PATH:   # (older diagnostic builds lack it)
        L.fpf_feeder_lane_plan.argtypes = [_dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.POINTER(FpfOpts),
                                           C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int, C.POINTER(C.c_int),
                                           C.c_int]
        L.fpf_feeder_lane_plan.restype = C.c_int
        L.fpf_lane_launches.restype = C.c_int
        L.fpf_lane_dma_launches.restype = C.c_int
    L.fpf_selftest_division.argtypes = [C.c_int, C.c_long, C.c_ulong]
    L.fpf_selftest_division.restype = C.c_long
    if hasattr(L, "fpf_multi_create") or path == LIB_PATH:   # (older diagnostic builds lack them)
        L.fpf_multi_create.argtypes = [C.c_int, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.POINTER(FpfOpts),
                                       C.POINTER(vp)]
        L.fpf_multi_create.restype = C.c_int
        L.fpf_multi_destroy.argtypes = [vp]
        L.fpf_multi_destroy.restype = None
        L.fpf_multi_last_error.argtypes = [vp]
        L.fpf_multi_last_error.restype = C.c_char_p
        L.fpf_multi_solve.argtypes = [vp, C.c_int, _dp, C.POINTER(FpfOutputs), C.POINTER(FpfAggregate)]
        L.fpf_multi_solve.restype = C.c_int
        L.fpf_multi_get_feeder.argtypes = [vp, C.c_int, C.POINTER(vp)]
        L.fpf_multi_get_feeder.restype = C.c_int
        L.fpf_multi_shard.argtypes = [C.c_int, C.c_int, C.c_long, C.POINTER(C.c_long), C.POINTER(C.c_long)]
        L.fpf_multi_shard.restype = C.c_int
        L.fpf_multi_schedule.argtypes = [C.c_int, C.c_long, C.c_long, C.POINTER(C.c_long), C.c_long]
        L.fpf_multi_schedule.restype = C.c_long
        L.fpf_aggregate_fold.argtypes = [C.POINTER(FpfAggregate), C.c_int, C.POINTER(FpfAggregate)]
        L.fpf_aggregate_fold.restype = None
    if hasattr(L, "fpf_areas_create") or path == LIB_PATH:
        L.fpf_areas_create.argtypes = [vp, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.POINTER(C.c_int), C.c_int,
                                       C.POINTER(FpfOpts), C.POINTER(vp)]
        L.fpf_areas_create.restype = C.c_int
        L.fpf_areas_destroy.argtypes = [vp]
        L.fpf_areas_destroy.restype = None
        L.fpf_areas_last_error.argtypes = [vp]
        L.fpf_areas_last_error.restype = C.c_char_p
        L.fpf_areas_info.argtypes = [vp, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.fpf_areas_info.restype = C.c_int
        L.fpf_areas_solve.argtypes = [vp, C.c_int, _dp, C.c_double, C.c_int, C.POINTER(FpfOutputs),
                                      C.POINTER(FpfAggregate)]
        L.fpf_areas_solve.restype = C.c_int
    if hasattr(L, "fpf_vvc_round") or path == LIB_PATH:
        L.fpf_vvc_gradient.argtypes = [vp, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.c_double, C.c_int, _dp, _dp,
                                       C.POINTER(C.c_int), _dp]
        L.fpf_vvc_gradient.restype = C.c_int
        L.fpf_vvc_gradient_at.argtypes = [_dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_double,
                                          C.c_double, C.c_double, C.c_int, _dp, _dp, C.POINTER(C.c_int), _dp]
        L.fpf_vvc_gradient_at.restype = C.c_int
        L.fpf_vvc_round.argtypes = [vp, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.c_double, C.c_double, C.c_int,
                                    C.c_int, _dp, _dp, C.POINTER(C.c_int), _dp, _dp, _dp, _dp]
        L.fpf_vvc_round.restype = C.c_int
    if hasattr(L, "fpf_vvc_gradient_batch") or path == LIB_PATH:
        L.fpf_vvc_gradient_batch.argtypes = [vp, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.c_int, _dp,
                                             C.c_double, C.c_int, _dp, _dp, C.POINTER(C.c_int), _dp,
                                             C.POINTER(C.c_int8)]
        L.fpf_vvc_gradient_batch.restype = C.c_int
    if hasattr(L, "fpf_vvc_round_batch") or path == LIB_PATH:
        L.fpf_vvc_round_batch.argtypes = [vp, _dp, C.c_int, C.c_int, _dp, C.c_int, C.c_int, C.c_int, _dp,
                                          C.c_double, C.c_double, C.c_int, C.c_int, _dp, _dp, C.POINTER(C.c_int),
                                          _dp, _dp, _dp, _dp, C.POINTER(C.c_int8)]
        L.fpf_vvc_round_batch.restype = C.c_int
    if hasattr(L, "fpf_rtc_compile") or path == LIB_PATH:
        L.fpf_rtc_compile.argtypes = [C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_int), C.c_char_p, C.c_size_t]
        L.fpf_rtc_compile.restype = C.c_long
        L.fpf_rtc_compiler.argtypes = []
        L.fpf_rtc_compiler.restype = C.c_char_p
    for name in ("fpf_ctx_create", "fpf_feeder_create", "fpf_feeder_get_info", "fpf_feeder_reserve",
                 "fpf_solve_batch", "fpf_solve_batch_device", "fpf_aggregate_device", "fpf_feeder_check"):
        getattr(L, name).restype = C.c_int
    if L.fpf_abi_version() != ABI_VERSION:
        raise RuntimeError("libfreedm_pf ABI mismatch")
    _lib = L
    return L


def default_opts(**kw) -> FpfOpts:
    o = FpfOpts()
    load().fpf_opts_default(C.byref(o))
    for k, v in kw.items():
        if k == "kernel" and isinstance(v, str):
            v = KERNELS[v]
        setattr(o, k, v)
    return o
