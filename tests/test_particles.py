"""Particle coupling: a sphere moving through fluid at rest feels a drag opposite to its
velocity; forces are all-reduced and integrated; momentum exchange is two-way."""
import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice
from tclb_amd.particles import SimplePart


def make(device="cpu"):
    lat = Lattice("auto_d3q19_part", (32, 24, 24), device=torch.device(device))
    lat.set_flags(np.full((lat.NZ, lat.NY, 32), lat.model.node_type("MRT").value, dtype=np.uint32))
    lat.set_setting("Viscosity", 0.1)
    sp = SimplePart()
    sp.add([16.0, 12.0, 12.0], 4.0, v=[0.01, 0, 0], m=1e9)   # heavy: keeps its velocity
    lat.particles = sp
    lat.init()
    return lat, sp


def test_sphere_drag_cpu():
    lat, sp = make()
    lat.iterate(40)
    assert sp.force[0, 0] < 0                      # drag opposes the motion
    assert abs(sp.force[0, 1]) < 1e-3 * abs(sp.force[0, 0]) + 1e-12
    u = lat.quantity("U").numpy()
    assert u[0].max() > 1e-3                       # fluid dragged along (two-way coupling)
    assert lat.quantity("Solid").numpy().max() > 0


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_sphere_drag_gpu_matches_cpu():
    a, pa = make("cuda")
    b, pb = make("cpu")
    a.iterate(10)
    b.iterate(10)
    assert np.allclose(pa.force, pb.force, rtol=1e-9, atol=1e-12)
    assert torch.allclose(a.fields_interior().cpu(), b.fields_interior(), atol=1e-12)
