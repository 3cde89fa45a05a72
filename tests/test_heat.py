"""d3q19_heat: a sinusoidal temperature mode decays with the D3Q7 diffusivity
D = c_s^2 (tau - 1/2), c_s^2 = 1/4, tau = 3*FluidAlpha + 1/2 (independent analytic check)."""
import math

import numpy as np
import torch

from tclb_amd.lattice import Lattice


def test_temperature_mode_decay():
    nx = 32
    lat = Lattice("d3q19_heat", (nx, 4, 4))
    m = lat.model
    lat.set_flags(np.full((lat.NZ, lat.NY, nx), m.node_type("MRT").value, dtype=np.uint32))
    alpha = 0.1
    lat.set_setting("FluidAlpha", alpha)
    lat.set_setting("nu", 0.1)
    lat.init()
    # impose T(x) = 1 + a sin(kx) via g equilibrium at rest: g scales with rhoT
    f = lat.fields_interior().clone()
    x = torch.arange(nx, dtype=f.dtype)
    a = 0.05
    T = 1 + a * torch.sin(2 * math.pi * x / nx)
    f[19:] = f[19:] * T[None, None, None, :]
    lat.set_fields_interior(f)
    steps = 200
    lat.iterate(steps)
    Tn = lat.quantity("T")[0, 0, 0].numpy()
    amp = (Tn.max() - Tn.min()) / 2
    tau = 3 * alpha + 0.5
    D = 0.25 * (tau - 0.5)
    k = 2 * math.pi / nx
    expect = a * math.exp(-D * k * k * steps)
    assert abs(amp - expect) / expect < 0.02, (amp, expect)
