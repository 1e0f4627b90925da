"""Device batches in caller buffers of exactly the batch's size (hipMalloc, no
slack after the data): the scenario-major wave kernel's per-wave staging reads
nothing past the last scenario in a ragged last workgroup (round-5 advisor
finding: idle waves used to base their loads past the tile), on the static
kernel and the per-plan build; the results equal the same batch's in a torch
tensor bit for bit."""
import ctypes as C

import numpy as np
import pytest

from freedm_amd import feeder as F

pytestmark = pytest.mark.gpu


class _Raw:
    """A raw device pointer with the shape solve_device reads."""

    def __init__(self, ptr, shape):
        self.p, self.shape = ptr, shape

    def data_ptr(self):
        return self.p


def _hip():
    h = C.CDLL("libamdhip64.so")
    h.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
    h.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    h.hipFree.argtypes = [C.c_void_p]
    return h


@pytest.mark.parametrize("B", [45, 37, 4101])
def test_scenario_major_batch_in_an_exact_size_buffer(B):
    import torch
    from freedm_amd import PowerFlow
    f = F.synthetic_feeder(123, 123)
    pq = np.ascontiguousarray(F.scenario_loads(f, np.arange(B)).transpose(2, 0, 1))   # [B][6][Nl]
    pf = PowerFlow(f, layout=1)
    dev = torch.device("cuda:0")

    def outs():
        return {"v_re": torch.zeros((B, 3, pf.nn), dtype=torch.float64, device=dev),
                "v_im": torch.zeros((B, 3, pf.nn), dtype=torch.float64, device=dev),
                "iters": torch.zeros(B, dtype=torch.int32, device=dev),
                "loss": torch.zeros(B, dtype=torch.float64, device=dev)}

    ref = outs()
    pf.solve_device(torch.from_numpy(pq).to(dev), ref)
    torch.cuda.synchronize()
    hip = _hip()
    p = C.c_void_p()
    assert hip.hipMalloc(C.byref(p), pq.nbytes) == 0
    try:
        assert hip.hipMemcpy(p, pq.ctypes.data, pq.nbytes, 1) == 0   # host to device
        got = outs()
        pf.solve_device(_Raw(p.value, pq.shape), got)
        torch.cuda.synchronize()
    finally:
        hip.hipFree(p)
    for k in ref:
        np.testing.assert_array_equal(got[k].cpu().numpy(), ref[k].cpu().numpy(), err_msg=k)
    assert (got["iters"].cpu().numpy() > 0).all()
