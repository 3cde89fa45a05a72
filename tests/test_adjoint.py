"""Discrete adjoint by automatic differentiation of the node code (tclb_amd.adjoint,
csrc/include/tclb/ad.hpp): gradients of the time-integrated Objective must equal
central finite differences — with respect to a global setting, a zonal setting, the
initial populations, for a single-stage model (d2q9) and a two-stage model with a
stencil field (d2q9_kuper)."""
import numpy as np
import pytest
import torch

from tclb_amd.adjoint import Adjoint
from tclb_amd.lattice import Lattice


def channel(model="d2q9", g=1e-5, nx=16, ny=8):
    lat = Lattice(model, (nx, ny, 1), device=torch.device("cpu"))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, nx), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, lat.gy + 0, :] = m.node_type("Wall").value
    fl[:, lat.gy + ny - 1, :] = m.node_type("Wall").value
    if model == "d2q9":
        fl[:, lat.gy + 1:lat.gy + ny - 1, 10] |= m.node_type("Outlet").value
        lat.set_flags(fl)
        lat.set_setting("Viscosity", 0.1)
        lat.set_setting("GravitationX", g)
        lat.set_setting("OutletFluxInObj", 1.0)
    else:
        lat.set_flags(fl)
        for k, v in {"nu": 0.1666, "Magic": 0.005, "FAcc": 1.0, "Temperature": 0.65, "GravitationX": g}.items():
            lat.set_setting(k, v)
        lat.set_setting("Density", 1.0)
        lat.set_setting("WallForceXInObj", 1.0)
    return lat


def objective(lat, steps):
    tot = 0.0
    for _ in range(steps):
        lat.iterate(1, glob_last=True)
        tot += lat.globals["Objective"]
    return tot


@pytest.mark.parametrize("model", ["d2q9", "d2q9_kuper"])
def test_setting_gradient_matches_fd(model):
    steps, g, h = 15, 1e-5, 1e-7
    lat = channel(model, g)
    lat.init()
    ad = Adjoint(lat, settings=["GravitationX"])
    ad.unsteady(steps)
    grad = ad.setting_gradient("GravitationX")

    def J(gv):
        L2 = channel(model, gv)
        L2.init()
        return objective(L2, steps)
    fd = (J(g + h) - J(g - h)) / (2 * h)
    assert abs(grad - fd) <= 1e-6 * abs(fd) + 1e-12, (grad, fd)


def test_initial_state_and_zonal_gradient_match_fd():
    steps, eps = 12, 1e-6
    lat = channel()
    lat.init()
    ad = Adjoint(lat, zonal=["OutletFluxInObj"])
    ad.unsteady(steps)
    gf = ad.field_gradient("f[1]")
    gz = ad.setting_gradient("OutletFluxInObj")

    def J(node=None, dv=0.0, w=1.0):
        L2 = channel()
        L2.set_setting("OutletFluxInObj", w)
        L2.init()
        if node is not None:
            f = L2.fields_interior().clone()
            f[(1,) + node] += dv
            L2.set_fields_interior(f)
        return objective(L2, steps)
    node = (0, 3, 7)
    fd = (J(node, eps) - J(node, -eps)) / (2 * eps)
    assert abs(gf[node] - fd) <= 1e-6 * abs(fd) + 1e-10, (gf[node], fd)
    # J is linear in the objective weight: dJ/dw = J(w=1)
    assert abs(gz - J()) <= 1e-9 * abs(gz)


def test_adjoint_quantities_d2q9_diff():
    """d2q9_diff (reference ADJOINT=1 model with adjoint quantities RhoB, WB): after an
    unsteady adjoint the WB quantity is dJ/dw and matches a finite difference of the
    Diff objective with respect to one node's material parameter."""
    nx, ny, steps = 12, 6, 10
    lat = Lattice("d2q9_diff", (nx, ny, 1), device=torch.device("cpu"))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, nx), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, :, 0] |= m.node_type("WPressure").value
    fl[:, :, nx - 1] |= m.node_type("EPressure").value
    fl[:, lat.gy:lat.gy + ny, 3] |= m.node_type("Obj2").value
    fl[:, lat.gy:lat.gy + ny, 8] |= m.node_type("Obj1").value
    lat.set_flags(fl)
    for k, v in {"nu0": 0.05, "nu1": 0.2, "InitDensity": 1.0, "InletDensity": 1.1, "OutletDensity": 1.0,
                 "DiffInObj": 1.0}.items():
        lat.set_setting(k, v)
    lat.init()
    # blend the material: w = 0.5 everywhere
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    f[wi] = 0.5
    lat.set_fields_interior(f)
    assert float(lat.quantity("WB").abs().max()) == 0.0      # no adjoint yet
    base = lat.snaps[lat.cur].clone()
    ad = Adjoint(lat)
    ad.unsteady(steps)
    wb = lat.quantity("WB")[0, 0].numpy()
    assert np.abs(wb).max() > 0
    assert np.allclose(wb, ad.field_gradient("w")[0])
    rhob = lat.quantity("RhoB")[0, 0].numpy()
    assert np.isfinite(rhob).all() and np.abs(rhob).max() > 0
    # finite difference on one node's w
    y, x, h = ny // 2, 5, 1e-6
    js = []
    for s in (+1, -1):
        lat.snaps[lat.cur].copy_(base)
        lat.iter = 0
        g = lat.fields_interior().clone()
        g[wi, 0, y, x] += s * h
        lat.set_fields_interior(g)
        js.append(objective(lat, steps))
    fd = (js[0] - js[1]) / (2 * h)
    assert abs(fd - wb[y, x]) < 1e-6 * max(1.0, abs(fd)) + 1e-9, (fd, wb[y, x])


def test_d3q19_adj_porosity_gradient():
    """d3q19_adj: pressure-driven duct through a porous design region; the adjoint
    gradient of the time-integrated outlet Flux with respect to one design node's w
    matches a central finite difference, and closing the design (w = 0) cuts the flux."""
    nx, ny, nz, steps = 10, 6, 6, 12
    lat = Lattice("d3q19_adj", (nx, ny, nz), device=torch.device("cpu"))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, :, 0] = m.node_type("WPressure").value | mrt
    fl[:, :, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, :, 7] |= m.node_type("Outlet").value
    fl[:, :, 4:6] |= m.node_type("DesignSpace").value
    lat.set_flags(fl)
    for k, v in {"nu": 0.1, "InletDensity": 1.03, "FluxInObj": 1.0, "Theta": 1.0}.items():
        lat.set_setting(k, v)
    lat.init()
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    f[wi, :, :, 4:6] = 0.7
    lat.set_fields_interior(f)
    base = lat.snaps[lat.cur].clone()
    ad = Adjoint(lat)
    ad.unsteady(steps)
    wb = lat.quantity("WB")[0].numpy()
    J0 = ad.J
    assert J0 > 0
    z, y, x, h = nz // 2, ny // 2, 4, 1e-6
    js = []
    for s in (+1, -1):
        lat.snaps[lat.cur].copy_(base)
        lat.iter = 0
        g = lat.fields_interior().clone()
        g[wi, z, y, x] += s * h
        lat.set_fields_interior(g)
        js.append(objective(lat, steps))
    fd = (js[0] - js[1]) / (2 * h)
    assert fd > 0 and abs(fd - wb[z, y, x]) < 1e-5 * abs(fd), (fd, wb[z, y, x])
    # closing the design region (w = 0) cuts the flux
    lat.snaps[lat.cur].copy_(base)
    lat.iter = 0
    g = lat.fields_interior().clone()
    g[wi, :, :, 4:6] = 0.0
    lat.set_fields_interior(g)
    assert objective(lat, steps) < 0.5 * J0


def test_late_reads_keep_segment_matches_checkpoint_only():
    """A model whose later stages read a field before the action writes it (Model.late_reads:
    d2q9_poison_boltzmann's subiter) depends on what the output snapshot held, the state two
    steps back.  The reverse sweep's segment re-run (keep_segment) must reproduce that
    (each fresh output buffer is seeded with it), so it equals the
    checkpoint-only sweep, which re-runs every step through the A/B swap."""
    from model_cases import CASE_SETTINGS
    assert Lattice("d2q9_poison_boltzmann", (6, 10, 1)).model.late_reads("Iteration") == ["subiter"]

    def case():
        lat = Lattice("d2q9_poison_boltzmann", (6, 10, 1), device=torch.device("cpu"))
        m = lat.model
        fl = np.full((lat.NZ, lat.NY, 6), m.node_type("Collision").value, dtype=np.uint32)
        fl[:, lat.gy + 0, :] = m.node_type("Wall").value
        fl[:, lat.gy + 9, :] = m.node_type("Wall").value
        lat.set_flags(fl)
        for k, v in CASE_SETTINGS["d2q9_poison_boltzmann"].items():
            lat.set_setting(k, v)
        lat.init()
        lat.iterate(3)
        return lat

    out, seen = [], []
    for keep in (True, False):
        lat = case()
        ad = Adjoint(lat)
        states = []
        orig = ad.step_back

        def spy(a, action="Iteration", state=None, other=None, **kw):
            # the state each reverse step linearises about (the recomputed primal state)
            s = state if state is not None else lat.snaps[lat.cur]
            states.append(s[:, :, lat.gy:lat.gy + 10, :6].clone())
            return orig(a, action, state=state, other=other, **kw)
        ad.step_back = spy
        gen = torch.Generator().manual_seed(5)
        a_final = torch.randn(lat.snaps[0].shape, generator=gen, dtype=torch.float64)
        a = ad.unsteady(8, checkpoint=4, a_final=a_final, keep_segment=keep)
        out.append(a[:, :, lat.gy:lat.gy + 10, :6].clone())
        seen.append(states)
    assert torch.count_nonzero(out[0]) > 0
    assert len(seen[0]) == len(seen[1]) == 8
    for s0, s1 in zip(*seen):
        assert torch.equal(s0, s1)                      # subiter included: it counts on from the real value
    assert torch.allclose(out[0], out[1], rtol=1e-12, atol=1e-14), (out[0] - out[1]).abs().max()
