"""Non-Newtonian models against analytic channel flows (independent oracles).

* d3q27_viscoplastic: force-driven Bingham channel flow — a rigid plug of half-width
  tau_y / g around the centre line, parabolic shear layers outside
  (u = g/(2 mu) (H^2/4 - y^2) - tau_y/mu (H/2 - |y|)).
* d3q27_kl: in the Newtonian limit (sigmaY = eta2 = 0) covered by test_poiseuille; here
  the shear-thinning branch must lower the apparent viscosity where the shear is high."""
import numpy as np

from tclb_amd.lattice import Lattice


def _channel(model, shape, coll="MRT"):
    lat = Lattice(model, shape)
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, shape[0]), m.node_type(coll).value, dtype=np.uint32)
    wall = m.node_type("Wall").value
    fl[:, lat.gy + 0, :] = wall
    fl[:, lat.gy + shape[1] - 1, :] = wall
    lat.set_flags(fl)
    return lat


def test_bingham_plug_flow():
    shape = (4, 34, 4)
    nu, g, ty = 1.0 / 6.0, 1e-6, 4e-6
    lat = _channel("d3q27_viscoplastic", shape)
    lat.set_setting("nu", nu)
    lat.set_setting("ForceX", g)
    lat.set_setting("YieldStress", ty)
    lat.init()
    lat.iterate(20000, glob_last=False)
    u = lat.quantity("U").numpy()[0][0, :, 0]
    ys = lat.quantity("yield_stat").numpy()[0, 0, :, 0]
    ny = shape[1]
    h = ny - 2
    yc = np.arange(ny) - 0.5 - h / 2
    yp = ty / g
    outer = g / (2 * nu) * ((h / 2) ** 2 - yc ** 2) - ty / nu * (h / 2 - np.abs(yc))
    plug = g / (2 * nu) * ((h / 2) ** 2 - yp ** 2) - ty / nu * (h / 2 - yp)
    ana = np.where(np.abs(yc) > yp, outer, plug)
    sel = slice(1, ny - 1)
    assert np.abs(u[sel] - ana[sel]).max() < 0.01 * ana.max()
    # unyielded exactly inside the plug
    inside = np.abs(yc) < yp
    assert (ys[inside] == 1).all() and (ys[~inside][1:-1] == 0).all()


def test_kl_shear_thinning_viscosity():
    shape = (4, 18, 4)
    lat = _channel("d3q27_kl", shape, coll="BGK")
    lat.set_setting("eta1", 0.05)
    lat.set_setting("eta2", 0.02)
    lat.set_setting("sigmaY", 0.0)
    lat.set_setting("m", 1e4)
    lat.set_setting("GravitationX", 1e-5, zone=None)
    lat.init()
    lat.iterate(3000, glob_last=False)
    nu = lat.quantity("Nu_app").numpy()[0, 0, :, 0]
    shear = lat.quantity("Shear").numpy()[0, 0, :, 0]
    ny = shape[1]
    sel = slice(1, ny - 1)
    assert np.isfinite(nu[sel]).all() and (shear[sel] > 0).all()
    # converged fixed point: nu_app = eta1 + eta2/sqrt(g) (1 - exp(-m g)) at every node
    g = shear[sel]
    kl = 0.05 + 0.02 / np.sqrt(g) * (1 - np.exp(-1e4 * g))
    assert np.abs(nu[sel] - kl).max() < 1e-9
    # the shear rate peaks at the walls and vanishes on the centre line; the viscosity
    # follows it through the regularised branch (non-constant, above eta1)
    assert shear[1] > shear[ny // 2] and nu[sel].min() > 0.05 and nu[sel].max() > 1.5 * nu[sel].min()
