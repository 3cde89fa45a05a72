"""The LDS A/B micro-benchmark (csrc/bench/lds_stencil.hip, tools/lds_ab.py): both the
global-load and the LDS-tiled 27-point stencil match a torch.roll reference (fp64) on a
small periodic box, and the host rejects shapes the tiling does not cover."""
import ctypes
import importlib.util
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
def test_lds_stencil_modes_match_reference():
    from tclb_amd.build import bench_lib_path
    spec = importlib.util.spec_from_file_location("lds_ab", os.path.join(ROOT, "tools", "lds_ab.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    lib = ctypes.CDLL(bench_lib_path("lds_stencil"))        # no fallback: the .so must exist
    fn = lib.tclb_lds_ab_run
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.POINTER(ctypes.c_float)]
    n = 64
    phi = torch.rand((n, n, n), dtype=torch.float64, device="cuda")
    ref = mod.reference(phi)
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    for mode in (0, 1):
        out = torch.full_like(phi, float("nan"))
        ms = ctypes.c_float()
        assert fn(mode, phi.data_ptr(), out.data_ptr(), n, 2, stream, ctypes.byref(ms)) == 0
        torch.cuda.synchronize()
        assert (out - ref).abs().max().item() < 1e-12, mode
    ms = ctypes.c_float()
    assert fn(1, phi.data_ptr(), phi.data_ptr(), 48, 1, stream, ctypes.byref(ms)) == -1   # 48 % 64 != 0
