"""d2q9_kuper_adj: with a uniform density the interaction force vanishes, mass is
conserved, and the design parameter w damps the gravity-driven velocity to the fixed point
u* = g (1 + w) / (2 (1 - w)) of u <- w (u + g/2) + g/2 (reference
models/optimization/experimental/d2q9_kuper_adj/Dynamics.c.Rt:423-494)."""
import numpy as np

from tclb_amd.lattice import Lattice


def test_kuper_adj_damping_fixed_point():
    n = 8
    lat = Lattice("d2q9_kuper_adj", (n, n, 1))
    m = lat.model
    lat.set_flags(np.full((lat.NZ, lat.NY, n), m.node_type("MRT").value, dtype=np.uint32))
    g, wv = 1e-4, 0.5
    for k, v in dict(InitDensity=1.0, Temperature=0.56, FAcc=1.0, Magic=0.01, MagicA=-0.152, MagicF=1.0,
                     GravitationX=g, nu=0.1).items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    names = [fl.name for fl in m.fields]
    f[names.index("w")] = wv
    lat.set_fields_interior(f)
    m0 = float(lat.quantity("Rho").double().sum())
    lat.iterate(200)
    rho = lat.quantity("Rho").double()
    u = lat.quantity("U").double()
    assert abs(float(rho.sum()) - m0) < 1e-10 * m0
    ustar = g * (1 + wv) / (2 * (1 - wv))
    assert abs(float(u[0].mean()) - ustar) < 1e-8, (float(u[0].mean()), ustar)
    assert float(u[1].abs().max()) < 1e-12
    assert float(lat.quantity("W").double().mean()) == wv
    assert float(lat.quantity("WB").abs().max()) == 0.0     # no adjoint sweep yet


def test_kuper_adj_design_gradient():
    """adjoint dJ/dw (J = time-integrated FluidVelocityX at Obj1 nodes) against a central
    finite difference"""
    import torch
    from tclb_amd.adjoint import Adjoint
    n, steps = 8, 10
    lat = Lattice("d2q9_kuper_adj", (n, n, 1), device=torch.device("cpu"))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, n), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, 2:5, 3:6] |= m.node_type("Obj1").value
    lat.set_flags(fl)
    for k, v in dict(InitDensity=1.0, Temperature=0.56, FAcc=1.0, Magic=0.01, MagicA=-0.152, MagicF=1.0,
                     GravitationX=1e-3, nu=0.1, FluidVelocityXInObj=1.0).items():
        lat.set_setting(k, v)
    lat.init()
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    y, x = np.mgrid[0:n, 0:n]
    f[wi, 0] = torch.as_tensor(0.8 + 0.05 * np.sin(x + 2 * y), dtype=f.dtype)
    lat.set_fields_interior(f)
    base = lat.snaps[lat.cur].clone()
    ad = Adjoint(lat)
    ad.unsteady(steps)
    wb = lat.quantity("WB")[0].numpy()
    y0, x0, h = 3, 4, 1e-6
    js = []
    for s in (+1, -1):
        lat.snaps[lat.cur].copy_(base)
        lat.iter = 0
        g = lat.fields_interior().clone()
        g[wi, 0, y0, x0] += s * h
        lat.set_fields_interior(g)
        tot = 0.0
        for _ in range(steps):
            lat.iterate(1, glob_last=True)
            tot += lat.globals["Objective"]
        js.append(tot)
    fd = (js[0] - js[1]) / (2 * h)
    assert abs(fd) > 0 and abs(fd - wb[0, y0, x0]) < 1e-5 * abs(fd), (fd, wb[0, y0, x0])
