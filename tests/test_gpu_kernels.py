"""GPU numerics: HIP kernels vs plain PyTorch references (fp64 and fp32) and vs the
CPU executor of the same model."""
import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice
from lbm_reference import U27, W27, bgk_step

gpu = pytest.mark.gpu
needs = pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")


def _mk(shape, device, precision="double"):
    lat = Lattice("d3q27", shape, device=device, precision=precision)
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint16)
    fl[:, lat.gy, :] = m.node_type("Wall").value
    lat.set_flags(fl)
    lat.set_setting("nu", 0.05)
    lat.set_setting("ForceX", 1e-4)
    lat.set_setting("Velocity", 0.02)
    return lat


@gpu
@needs
def test_hip_loaded_not_cpu():
    lat = _mk((64, 16, 8), torch.device("cuda", 0))
    assert lat.lib.kind == "hip" and lat.lib.path.endswith("_hip.so")


@gpu
@needs
@pytest.mark.parametrize("shape", [(64, 16, 8), (100, 20, 6), (33, 7, 5)])
def test_hip_matches_cpu_fp64(shape):
    a = _mk(shape, torch.device("cuda", 0))
    b = _mk(shape, torch.device("cpu"))
    for lat in (a, b):
        lat.init()
        lat.iterate(6)
    torch.cuda.synchronize()
    assert torch.allclose(a.fields_interior().cpu(), b.fields_interior(), atol=1e-13, rtol=0)
    for k in a.globals:
        assert abs(a.globals[k] - b.globals[k]) <= 1e-9 * (1 + abs(b.globals[k])), k
    ua = a.quantity("U").cpu()
    ub = b.quantity("U")
    assert torch.allclose(ua, ub, atol=1e-13)


@gpu
@needs
def test_hip_fp32_vs_torch_fp32_reference():
    shape = (64, 16, 8)
    lat = Lattice("d3q27", shape, device=torch.device("cuda", 0), precision="float")
    fl = np.full((lat.NZ, lat.NY, shape[0]), lat.model.node_type("MRT").value, dtype=np.uint16)
    lat.set_flags(fl)
    lat.set_setting("nu", 0.05)
    lat.set_setting("Velocity", 0.02)
    lat.init()
    torch.manual_seed(1)
    f0 = lat.fields_interior().clone()
    f0 = f0 * (1 + 0.01 * torch.rand_like(f0))
    lat.set_fields_interior(f0)
    lat.iterate(5)
    r = f0.cpu().double()
    for _ in range(5):
        r = bgk_step(r, lat.get_setting("omega"), U27, W27)
    assert torch.allclose(lat.fields_interior().cpu().double(), r, atol=3e-6)


@gpu
@needs
def test_hip_mass_conservation_large():
    lat = _mk((256, 64, 32), torch.device("cuda", 0))
    lat.init()
    m0 = lat.fields_interior().sum().item()
    lat.iterate(20)
    assert abs(lat.fields_interior().sum().item() - m0) / m0 < 1e-12


@gpu
@needs
@pytest.mark.parametrize("precision,tol", [("mixed-shift", 1e-12), ("half-shift", 2e-3), ("half", 2e-3)])
def test_hip_reduced_storage_matches_cpu(precision, tol):
    """fp32 / fp16 storage (shifted or not): the HIP kernels (native _Float16) and the CPU
    executor (software binary16) round identically up to compute-order differences"""
    shape = (64, 16, 8)
    a = _mk(shape, torch.device("cuda", 0), precision)
    b = _mk(shape, torch.device("cpu"), precision)
    assert a.snaps[0].dtype == b.snaps[0].dtype
    for lat in (a, b):
        lat.init()
        lat.iterate(6)
    torch.cuda.synchronize()
    fa = a.fields_interior().cpu().double()
    fb = b.fields_interior().double()
    assert (fa - fb).abs().max().item() <= tol * fb.abs().max().item()


@gpu
@needs
def test_hip_sampler_matches_quantity():
    from tclb_amd.sampler import Sampler
    lat = _mk((64, 16, 8), torch.device("cuda", 0))
    lat.init()
    smp = Sampler(lat, [(3, 4, 2), (63, 15, 7)], ["P", "U"], rows=4)
    lat.samplers.append(smp)
    lat.iterate(4)                                   # native loop records 4 rows
    rows = smp.flush()
    assert len(rows) == 8
    u = lat.quantity("U").cpu().numpy()
    rho = lat.quantity("P").cpu().numpy()
    for it, i, (x, y, z), v in rows[-2:]:
        assert it == 4
        np.testing.assert_allclose(v, [rho[0, z, y, x], *u[:, z, y, x]], rtol=1e-13)
