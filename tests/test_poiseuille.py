"""Physics validation: force-driven channel flow between bounce-back walls converges to
the analytic Poiseuille profile (independent oracle, no reference code involved)."""
import numpy as np
import pytest

from tclb_amd.lattice import Lattice

CASES = {
    # model: (shape, force setting(s), viscosity setting, force->acceleration factor, u shift)
    "d3q27": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d3q19": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d2q9": ((4, 18, 1), {"GravitationX": 1e-6}, "Viscosity"),
    "d2q9_SRT": ((4, 18, 1), {"GravitationX": 1e-6}, "nu"),
    "d2q9_cumulant": ((4, 18, 1), {"ForceX": 1e-6}, "nu"),
    "d3q27_cumulant": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d3q19_les": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "auto_d3q19_BGK": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "auto_d3q19_TRT": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "auto": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "auto_WMRT": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "auto_d3q19_WMRT_HiOrd": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "auto_FMT_HiOrd": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "d3q27_cumulant_AVG_IB_SMAG": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d3q27_cumulant_part": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d3q27_BGK": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d3q27_BGK_galcor": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d3q27_viscoplastic": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),     # YieldStress = 0: Newtonian
    "d3q27_kl": ((4, 18, 4), {"GravitationX": 1e-6}, "eta1"),       # sigmaY = eta2 = 0: Newtonian
    "d2q9_lbmpy": ((4, 18, 1), {"GravitationX": 1e-6}, "nu"),
    "d2q9_inc": ((4, 18, 1), {"GravitationX": 1e-6}, "nu"),
}


@pytest.mark.parametrize("model", list(CASES))
def test_poiseuille(model):
    shape, force, visc = CASES[model]
    lat = Lattice(model, shape)
    m = lat.model
    coll = m.node_type("MRT") or m.node_type("BGK")
    nx = shape[0]
    fl = np.full((lat.NZ, lat.NY, nx), coll.value, dtype=np.uint32)
    wall = m.node_type("Wall").value
    fl[:, lat.gy + 0, :] = wall
    fl[:, lat.gy + shape[1] - 1, :] = wall
    if lat.slab.axis == 1 and lat.gy:     # ghost rows (multi-rank layouts) image the walls
        fl[:, :lat.gy, :] = wall
        fl[:, -lat.gy:, :] = wall
    lat.set_flags(fl)
    nu = 1.0 / 6.0
    lat.set_setting(visc, nu)
    for k, v in force.items():
        lat.set_setting(k, v, zone=None)
    g = list(force.values())[0]
    lat.init()
    lat.iterate(6000, glob_last=False)
    u = lat.quantity("U").numpy()[0]  # (nz, ny, nx)
    prof = u[0, :, 0]
    ny = shape[1]
    y = np.arange(ny, dtype=float)
    ana = g / (2 * nu) * (y - 0.5) * (ny - 1.5 - y)
    sel = slice(1, ny - 1)
    err = np.abs(prof[sel] - ana[sel]).max() / ana[sel].max()
    assert err < 0.02, (model, err, prof[sel][:4], ana[sel][:4])


@pytest.mark.parametrize("model,extra", [("d2q9_les", {"Smag": 0.0}), ("d2q9_les", {"Smag": 0.16}),
                                         ("d2q9_cumulant", {"nubuffer": 1.0 / 6.0})])
def test_inlet_channel_develops_parabola(model, extra):
    """Zou/He velocity inlet (WVelocity) + pressure outlet (EPressure): downstream the
    profile is the parabola carrying the inlet flux (2-D models without a body force)."""
    nx, ny, U0 = 48, 18, 0.01
    lat = Lattice(model, (nx, ny, 1))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, nx), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, :, 0] = m.node_type("WVelocity").value | m.node_type("MRT").value
    fl[:, :, nx - 1] = m.node_type("EPressure").value | m.node_type("MRT").value
    fl[:, lat.gy + 0, :] = m.node_type("Wall").value
    fl[:, lat.gy + ny - 1, :] = m.node_type("Wall").value
    lat.set_flags(fl)
    lat.set_setting("nu", 1.0 / 6.0)
    lat.set_setting("Velocity", U0)
    for k, v in extra.items():
        lat.set_setting(k, v)
    lat.init()
    lat.iterate(4000, glob_last=False)
    u = lat.quantity("U").numpy()[0][0]          # (ny, nx)
    prof = u[1:ny - 1, 36]
    h = ny - 2                                   # walls on the node rows 0 and ny-1
    y = np.arange(1, ny - 1) - 0.5
    ana = 6 * U0 * y * (h - y) / h ** 2
    assert np.isfinite(u).all()
    assert np.abs(prof - ana).max() < 0.03 * ana.max(), (prof, ana)
