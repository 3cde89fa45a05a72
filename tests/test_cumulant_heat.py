"""d3q27_cumulant_heat: the D3Q7 temperature diffuses with D = Alpha and a uniform
temperature excess accelerates the fluid by (T - T0) * Buoyancy per step (reference
models/heat/experimental/d3q27_cumulant_heat/Dynamics.c.Rt)."""
import math

import numpy as np
import torch

from tclb_amd.lattice import Lattice


def _lat(shape, **settings):
    lat = Lattice("d3q27_cumulant_heat", shape)
    m = lat.model
    lat.set_flags(np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint32))
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


def test_temperature_diffusion():
    nx, alpha, steps, a = 32, 0.05, 300, 0.05
    lat = _lat((nx, 4, 4), Alpha=alpha, Temperature=1.0, nu=0.1)
    m = lat.model
    f = lat.fields_interior().clone()
    x = torch.arange(nx, dtype=f.dtype)
    prof = 1 + a * torch.sin(2 * math.pi * x / nx)
    sel = [i for i, fl in enumerate(m.fields) if fl.group == "g"]
    f[sel] = f[sel] * prof[None, None, None, :]
    lat.set_fields_interior(f)
    lat.iterate(steps)
    t = lat.quantity("T")[0, 0, 0].double().numpy()
    amp = (t.max() - t.min()) / 2
    k = 2 * math.pi / nx
    expect = a * math.exp(-alpha * k * k * steps)
    assert abs(amp - expect) / expect < 0.02, (amp, expect)


def test_boussinesq_acceleration():
    n, B, T, T0 = 20, 1e-4, 1.5, 1.0
    lat = _lat((6, 6, 6), Alpha=0.1, Temperature=T, Buoyancy=B, BuoyancyT0=T0, nu=0.1)
    lat.iterate(n)
    uy = float(lat.quantity("U")[1].double().mean())
    assert abs(uy - n * (T - T0) * B) < 1e-9, (uy, n * (T - T0) * B)
    assert abs(float(lat.quantity("T").double().mean()) - T) < 1e-12
