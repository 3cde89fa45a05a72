"""d2q9q9_cm_cht: the enthalpy population diffuses with D = conductivity (cp = rho = 1)
under every heat collision, buoyancy accelerates the fluid by g (rho - B T) / rho per
step, and the equilibrium Dirichlet heater pins T (reference
models/heat/d2q9q9_cm_cht/Dynamics.c.Rt)."""
import math

import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice


def _lat(shape, collision="CM_HIGHER", extra=None, model="d2q9q9_cm_cht", **settings):
    lat = Lattice(model, shape)
    m = lat.model
    flags = np.full((lat.NZ, lat.NY, shape[0]), m.node_type(collision).value, dtype=np.uint32)
    if extra is not None:
        extra(flags, m)
    lat.set_flags(flags)
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


@pytest.mark.parametrize("collision", ["CM_HIGHER", "CM_HIGHER_PROB", "CM_HIGHER_PROB_M_EQ", "Cumulants"])
def test_heat_diffusion(collision):
    nx, k, steps, a = 32, 0.05, 300, 0.05
    lat = _lat((nx, 4), collision, conductivity=k, InitTemperature=1.0, nu=0.1)
    m = lat.model
    f = lat.fields_interior().clone()
    x = torch.arange(nx, dtype=f.dtype)
    prof = 1 + a * torch.sin(2 * math.pi * x / nx)
    sel = [i for i, fl in enumerate(m.fields) if fl.group == "h"]
    f[sel] = f[sel] * prof[None, None, None, :]
    lat.set_fields_interior(f)
    lat.iterate(steps)
    t = lat.quantity("T")[0, 0, 0].double().numpy()
    amp = (t.max() - t.min()) / 2
    kk = 2 * math.pi / nx
    expect = a * math.exp(-k * kk * kk * steps)
    assert abs(amp - expect) / expect < 0.03, (collision, amp, expect)
    assert abs(t.mean() - 1.0) < 1e-10


def test_boussinesq_acceleration():
    n, g, B, T = 20, 1e-5, 0.5, 1.5
    lat = _lat((6, 6), InitTemperature=T, GravitationY=g, BoussinesqCoeff=B, nu=0.1, conductivity=0.1)
    lat.iterate(n)
    uy = lat.quantity("U")[1].double()
    expect = n * g * (1 - B * T) + g * (1 - B * T) / 2   # reported U includes F / (2 rho)
    assert float((uy - expect).abs().max()) < 1e-10, (float(uy.mean()), expect)


def _heater_lat(kind, nx=24):
    """west column (x = 0, 1) is a heater zone at T = 1; the bulk starts at T = 0"""
    lat = Lattice("d2q9q9_cm_cht", (nx, 3))
    m = lat.model
    zi = lat.zone_index("heater")
    flags = np.full((lat.NZ, lat.NY, nx), m.node_type("CM_HIGHER").value, dtype=np.uint32)
    flags[:, :, :2] |= m.node_type(kind).value | (zi << m.zone_shift)
    if kind == "HeaterDirichletTemperatureABB":
        flags[:, :, :2] |= m.node_type("Wall").value
    lat.set_flags(flags)
    for k, v in dict(conductivity=0.1, nu=0.1, InitTemperature=0.0).items():
        lat.set_setting(k, v)
    lat.set_setting("InitTemperature", 1.0, zone="heater")
    lat.init()
    return lat


@pytest.mark.parametrize("kind", ["HeaterDirichletTemperatureEQ", "HeaterDirichletTemperatureABB"])
def test_dirichlet_heater(kind):
    lat = _heater_lat(kind)
    lat.iterate(400)
    t = lat.quantity("T")[0, 0, 0].double().numpy()
    inner = t[2:12]
    # heat enters from the west heater: T decays monotonically away from it, within (0, 1)
    assert np.all(np.diff(inner) < 0), inner
    assert 0.0 < inner[-1] < inner[0] < 1.0, inner
    assert lat.globals["HeatSource"] > 0.0


@pytest.mark.parametrize("variant", ["d2q9q9_cm_cht_OutFlowNeumann", "d2q9q9_cm_cht_OutFlowConvective",
                                     "d2q9q9_cm_cht_AVG", "d2q9q9_cm_cht_CHT"])
def test_variants_conserve_uniform_state(variant):
    lat = _lat((8, 6), model=variant, InitTemperature=1.0, nu=0.1, conductivity=0.1)
    lat.iterate(10)
    assert abs(float(lat.quantity("T").double().mean()) - 1.0) < 1e-12
    assert float(lat.quantity("U").double().abs().max()) < 1e-12
