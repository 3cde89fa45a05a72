"""d3q19_heat_adj_art: temperature diffuses with D = alpha (sigma^2 = 1/4), the design
weight scales momentum by 2 w - 1, heaters pin T and report HeatInput, and the adjoint
design gradient of a thermometer objective matches finite differences (reference
models/article/d3q19_heat_adj_art/Dynamics.c)."""
import math

import numpy as np
import torch

from tclb_amd.lattice import Lattice


def _lat(shape, flags_fn=None, **settings):
    lat = Lattice("d3q19_heat_adj_art", shape, device=torch.device("cpu"))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint32)
    if flags_fn is not None:
        flags_fn(fl, m, lat)
    lat.set_flags(fl)
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


def test_temperature_diffusion():
    nx, alpha, steps, a = 32, 0.05, 300, 0.05
    lat = _lat((nx, 3, 3), FluidAlpha=alpha, SolidAlpha=alpha, Temperature=1.0, nu=0.1)
    m = lat.model
    f = lat.fields_interior().clone()
    x = torch.arange(nx, dtype=f.dtype)
    sel = [i for i, fl in enumerate(m.fields) if fl.group == "T"]
    f[sel] = f[sel] * (1 + a * torch.sin(2 * math.pi * x / nx))[None, None, None, :]
    lat.set_fields_interior(f)
    lat.iterate(steps)
    t = lat.quantity("T")[0, 0, 0].double().numpy()
    amp = (t.max() - t.min()) / 2
    kk = 2 * math.pi / nx
    expect = a * math.exp(-alpha * kk * kk * steps)
    assert abs(amp - expect) / expect < 0.02, (amp, expect)


def test_design_weight_scales_momentum():
    lat = _lat((4, 4, 4), Velocity=0.02, nu=0.1)
    m = lat.model
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    f[wi] = 0.5
    lat.set_fields_interior(f)
    lat.iterate(1)
    assert float(lat.quantity("U").abs().max()) < 1e-15
    lat2 = _lat((4, 4, 4), Velocity=0.02, nu=0.1)
    f = lat2.fields_interior().clone()
    f[wi] = 0.0
    lat2.set_fields_interior(f)
    lat2.iterate(1)
    assert abs(float(lat2.quantity("U")[0].mean()) + 0.02) < 1e-14   # w = 0 reverses the flow


def test_heater_and_objectives():
    def fl(flags, m, lat):
        zi = lat.zone_index("hot")
        flags[:, :, 0] |= m.node_type("Heater").value | (zi << m.zone_shift)
        flags[:, :, 5] |= m.node_type("Thermometer").value
        flags[:, :, 7] |= m.node_type("Outlet").value

    lat = Lattice("d3q19_heat_adj_art", (16, 3, 3), device=torch.device("cpu"))
    m = lat.model
    flags = np.full((lat.NZ, lat.NY, 16), m.node_type("MRT").value, dtype=np.uint32)
    fl(flags, m, lat)
    lat.set_flags(flags)
    for k, v in dict(FluidAlpha=0.1, Temperature=0.0, nu=0.1, LimitTemperature=0.9).items():
        lat.set_setting(k, v)
    lat.set_setting("Temperature", 1.0, zone="hot")
    lat.init()
    lat.iterate(200)
    t = lat.quantity("T")[0, 0, 0].double().numpy()
    assert abs(t[0] - 1.0) < 0.05 and 0 < t[5] < t[1]
    g = lat.globals
    assert g["HeatInput"] > 0
    assert abs(g["TemperatureAtPoint"] - 9 * t[5]) < 0.01 * g["TemperatureAtPoint"]   # sum of T vs T = sum / rho, one step apart
    assert g["LowTemperature"] > 0 and g["HighTemperature"] == 0.0


def test_design_gradient_matches_fd():
    from tclb_amd.adjoint import Adjoint
    n, steps = 6, 8

    def fl(flags, m, lat):
        flags[:, :, 0] |= m.node_type("Heater").value
        flags[:, 2:4, 4] |= m.node_type("Thermometer").value
        flags[:, :, 1:5] |= m.node_type("DesignSpace").value

    lat = _lat((n, 4, 3), fl, FluidAlpha=0.1, SolidAlpha=0.02, Temperature=1.0, nu=0.1, Velocity=0.01,
               TemperatureAtPointInObj=1.0, MaterialPenaltyInObj=0.1)
    m = lat.model
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    z, y, x = np.mgrid[0:3, 0:4, 0:n]
    f[wi] = torch.as_tensor(0.7 + 0.1 * np.sin(x + 2 * y + 3 * z), dtype=f.dtype)
    sel = [i for i, fld in enumerate(m.fields) if fld.group == "T"]
    f[sel] = f[sel] * 0.5
    lat.set_fields_interior(f)
    base = lat.snaps[lat.cur].clone()
    ad = Adjoint(lat)
    ad.unsteady(steps)
    wb = lat.quantity("WB")[0].numpy()
    p, h = (1, 2, 3), 1e-6
    js = []
    for s in (+1, -1):
        lat.snaps[lat.cur].copy_(base)
        lat.iter = 0
        g = lat.fields_interior().clone()
        g[wi][p] += s * h
        lat.set_fields_interior(g)
        tot = 0.0
        for _ in range(steps):
            lat.iterate(1, glob_last=True)
            tot += lat.globals["Objective"]
        js.append(tot)
    fd = (js[0] - js[1]) / (2 * h)
    assert abs(fd) > 0 and abs(fd - wb[p]) < 1e-5 * abs(fd), (fd, wb[p])


def _prop(shape, flags_fn=None, **settings):
    lat = Lattice("d3q19_heat_adj_prop", shape, device=torch.device("cpu"))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint32)
    if flags_fn is not None:
        flags_fn(fl, m)
    lat.set_flags(fl)
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


def test_prop_weight_propagation():
    """effective weight eff(x) = w(x) - P (1 - eff(x - 1)) on Propagate nodes, one cell per step"""
    nx, P, steps = 12, 0.5, 15
    lat = _prop((nx, 3, 3), lambda fl, m: fl.__ior__(m.node_type("Propagate").value),
                FluidAlpha=0.1, SolidAlpha=0.1, nu=0.1, PropagateX=P, InletTemperature=1.0)
    m = lat.model
    wi = m.field_index("w")
    wv = np.ones(nx)
    wv[3] = 0.2
    f = lat.fields_interior().clone()
    f[wi] = torch.as_tensor(wv)[None, None, :]
    lat.set_fields_interior(f)
    lat.iterate(steps)
    eff = np.ones(nx)
    for _ in range(steps):
        eff = wv - P * (1 - np.roll(eff, 1))
    w0 = lat.quantity("W0")[0, 0, 0].double().numpy()     # streamed from x + 1
    assert np.allclose(w0, np.roll(eff, -1), atol=1e-13), (w0, np.roll(eff, -1))


def test_prop_heat_source_and_stopped_flow():
    def fl(flags, m):
        flags[:, :, 2] |= m.node_type("HeatSource").value
        flags[:, :, 6] |= m.node_type("Thermometer").value

    lat = _prop((12, 3, 3), fl, FluidAlpha=0.1, SolidAlpha=0.1, nu=0.1, InletVelocity=0.01,
                InletTemperature=0.0, HeatSource=1e-3, LimitTemperature=1.0)
    m = lat.model
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    f[wi] = 0.0                       # w0 = 0: the fluid stops after one collision
    lat.set_fields_interior(f)
    lat.iterate(50)
    assert float(lat.quantity("U").abs().max()) < 1e-15
    T = lat.quantity("T")[0, 0, 0].double().numpy()
    # 9 source nodes x 1e-3 per step, no advection: total heat grows linearly
    assert abs(T.sum() * 9 - 50 * 9e-3) < 1e-10, T.sum() * 9
    assert lat.globals["Temperature"] > 0 and lat.globals["LowTemperature"] > 0


def test_prop_design_gradient_matches_fd():
    from tclb_amd.adjoint import Adjoint
    n, steps = 6, 8

    def fl(flags, m):
        flags[:, :, 0] |= m.node_type("Heater").value
        flags[:, 2:4, 4] |= m.node_type("Thermometer").value
        flags[:, :, 1:5] |= m.node_type("DesignSpace").value | m.node_type("Propagate").value

    lat = _prop((n, 4, 3), fl, FluidAlpha=0.1, SolidAlpha=0.02, HeaterTemperature=1.0, nu=0.1, InletVelocity=0.01,
                PropagateX=0.3, TemperatureInObj=1.0, MaterialPenaltyInObj=0.1)
    m = lat.model
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    z, y, x = np.mgrid[0:3, 0:4, 0:n]
    f[wi] = torch.as_tensor(0.7 + 0.1 * np.sin(x + 2 * y + 3 * z), dtype=f.dtype)
    lat.set_fields_interior(f)
    base = lat.snaps[lat.cur].clone()
    ad = Adjoint(lat)
    ad.unsteady(steps)
    wb = lat.quantity("WB")[0].numpy()
    p, h = (1, 2, 2), 1e-6
    js = []
    for s in (+1, -1):
        lat.snaps[lat.cur].copy_(base)
        lat.iter = 0
        g = lat.fields_interior().clone()
        g[wi][p] += s * h
        lat.set_fields_interior(g)
        tot = 0.0
        for _ in range(steps):
            lat.iterate(1, glob_last=True)
            tot += lat.globals["Objective"]
        js.append(tot)
    fd = (js[0] - js[1]) / (2 * h)
    assert abs(fd) > 0 and abs(fd - wb[p]) < 1e-5 * abs(fd), (fd, wb[p])
