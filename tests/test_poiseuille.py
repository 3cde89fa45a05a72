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
    "d3q27_cumulant": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "d3q19_les": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
    "auto_d3q19_BGK": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "auto_d3q19_TRT": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "auto": ((4, 18, 4), {"ForceX": 1e-6}, "Viscosity"),
    "d3q27_cumulant_AVG_IB_SMAG": ((4, 18, 4), {"ForceX": 1e-6}, "nu"),
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
    if lat.slab.axis == 2:
        fl[:, lat.gy + 0, :] = wall
        fl[:, lat.gy + shape[1] - 1, :] = wall
    else:
        fl[:, 0, :] = wall   # ghost row of y=0 plane image is y=ny-1: also wall
        fl[:, 1, :] = wall
        fl[:, lat.gy + shape[1] - 1, :] = wall
        fl[:, -1, :] = wall
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
