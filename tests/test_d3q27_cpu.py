import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice
from lbm_reference import U27, W27, bgk_step, stream, bounce_back_mask, feq, moments


def make(shape=(24, 12, 8), **kw):
    lat = Lattice("d3q27", shape, **kw)
    mrt = lat.model.node_type("MRT").value
    lat.set_flags(np.full((lat.NZ, lat.NY, shape[0]), mrt, dtype=np.uint16))
    return lat


def test_periodic_bgk_matches_torch_reference():
    lat = make()
    lat.set_setting("nu", 0.05)
    lat.set_setting("ForceX", 1e-4)
    lat.set_setting("Velocity", 0.03)
    lat.init()
    torch.manual_seed(0)
    f = lat.fields_interior().clone() * (1 + 0.02 * torch.rand_like(lat.fields_interior()))
    lat.set_fields_interior(f)
    lat.iterate(7)
    r = f.clone()
    for _ in range(7):
        r = bgk_step(r, lat.get_setting("omega"), U27, W27, force=(1e-4, 0, 0))
    assert torch.allclose(lat.fields_interior(), r, atol=1e-13, rtol=0)


def test_mass_conservation_and_globals():
    lat = make()
    lat.set_setting("nu", 0.1)
    lat.set_setting("Velocity", 0.05)
    lat.init()
    m0 = lat.fields_interior().sum().item()
    lat.iterate(5)
    assert abs(lat.fields_interior().sum().item() - m0) < 1e-9
    n = 24 * 12 * 8
    # XFlux = sum (Jx + 1.5 F)/rho over nodes = n * Velocity for uniform flow
    assert abs(lat.globals["XFlux"] - n * 0.05) < 1e-9


def test_wall_bounce_back_channel():
    lat = make()
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, 24), m.node_type("MRT").value, dtype=np.uint16)
    fl[:, lat.gy + 0, :] = m.node_type("Wall").value
    fl[:, lat.gy + 11, :] = m.node_type("Wall").value
    lat.set_flags(fl)
    lat.set_setting("nu", 0.1)
    lat.set_setting("ForceX", 1e-5)
    lat.init()
    lat.iterate(3)
    # wall rows are bounced-back only (no collision): check one step against torch
    f = lat.fields_interior().clone()
    lat.iterate(1)
    fs = stream(f, U27)
    wall = torch.zeros(f.shape[1:], dtype=torch.bool)
    wall[:, 0, :] = True
    wall[:, 11, :] = True
    bb = bounce_back_mask(fs, wall, U27)
    rho, J = moments(fs, U27)
    fe = feq(rho, J, U27, W27)
    om = lat.get_setting("omega")
    coll = feq(rho, J + torch.tensor([1e-5, 0, 0], dtype=f.dtype)[:, None, None, None], U27, W27) + (1 - om) * (fs - fe)
    ref = torch.where(wall[None], bb, coll)
    assert torch.allclose(lat.fields_interior(), ref, atol=1e-13)
    # drag on walls is recorded
    assert lat.globals["XDragForce"] != 0.0


def test_quantities():
    lat = make()
    lat.set_setting("Velocity", 0.02)
    lat.set_setting("Pressure", 0.001)
    lat.init()
    u = lat.quantity("U")
    p = lat.quantity("P")
    # reference Init sets J = Velocity (not rho*Velocity): u = Velocity / rho
    assert torch.allclose(u[0], torch.full_like(u[0], 0.02 / 1.003), atol=1e-12)
    assert torch.allclose(p[0], torch.full_like(p[0], 0.001), atol=1e-12)


def test_float_precision_close_to_double():
    a = make(precision="double")
    b = make(precision="float")
    for lat in (a, b):
        lat.set_setting("nu", 0.05)
        lat.set_setting("Velocity", 0.03)
        lat.init()
        lat.iterate(5)
    assert torch.allclose(a.fields_interior().float(), b.fields_interior(), atol=2e-6)
