"""d3q27q7_cm_cht: the D3Q7 enthalpy population diffuses with D = conductivity (cp = rho =
1) under the CM, CM_PROB and BGK heat collisions, buoyancy accelerates the fluid by
g (rho - B (T - 10)) / rho per step, the equilibrium / anti-bounce-back heaters pin T, and
every option variant keeps a uniform state at rest (reference
models/heat/d3q27q7_cm_cht/Dynamics.c.Rt:247-1487)."""
import math

import numpy as np
import pytest
import torch

from conftest import DEVICES
from tclb_amd.lattice import Lattice


def _lat(shape, collision="CM", extra=None, model="d3q27q7_cm_cht", device="cpu", **settings):
    lat = Lattice(model, shape, device=torch.device(device))
    m = lat.model
    flags = np.full((lat.NZ, lat.NY, shape[0]), m.node_type(collision).value, dtype=np.uint32)
    if extra is not None:
        extra(flags, m)
    lat.set_flags(flags)
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


Q27_COLLISIONS = ["CM_HIGHER", "CM_HIGHER_PROB", "CM_HIGHER_PROB_M_EQ", "Cumulants", "Cumulants_HIGHER", "CM", "BGK"]


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("model,collision", [("d3q27q7_cm_cht", c) for c in ("CM", "CM_PROB", "BGK")] +
                         [("d3q27q27_cm_cht", c) for c in Q27_COLLISIONS])
def test_heat_diffusion(model, collision, device):
    nx, k, steps, a = 32, 0.05, 300, 0.05
    lat = _lat((nx, 2, 2), collision, model=model, device=device, conductivity=k, InitTemperature=1.0, nu=0.1)
    m = lat.model
    f = lat.fields_interior().clone()
    x = torch.arange(nx, dtype=f.dtype, device=f.device)
    prof = 1 + a * torch.sin(2 * math.pi * x / nx)
    sel = [i for i, fl in enumerate(m.fields) if fl.group == "h"]
    f[sel] = f[sel] * prof[None, None, None, :]
    lat.set_fields_interior(f)
    lat.iterate(steps)
    t = lat.quantity("T")[0, 0, 0].double().cpu().numpy()
    amp = (t.max() - t.min()) / 2
    kk = 2 * math.pi / nx
    expect = a * math.exp(-k * kk * kk * steps)
    assert abs(amp - expect) / expect < 0.03, (collision, amp, expect)
    assert abs(t.mean() - 1.0) < 1e-10


@pytest.mark.parametrize("model,collision", [("d3q27q7_cm_cht", "CM"), ("d3q27q27_cm_cht", "CM_HIGHER")])
def test_boussinesq_acceleration(model, collision):
    n, g, B, T = 20, 1e-5, 0.05, 12.0
    lat = _lat((4, 4, 4), collision, model=model, InitTemperature=T, GravitationZ=g, BoussinesqCoeff=B, nu=0.1, conductivity=0.1)
    lat.iterate(n)
    uz = lat.quantity("U")[2].double()
    a = g * (1 - B * (T - 10.0))
    expect = n * a + a / 2   # reported U includes F / (2 rho)
    assert float((uz - expect).abs().max()) < 1e-10, (float(uz.mean()), expect)
    assert float(lat.quantity("U")[:2].double().abs().max()) < 1e-12


def _heater_lat(kind, nx=24, model="d3q27q7_cm_cht", collision="CM"):
    """west slab (x = 0, 1) is a heater zone at T = 1; the bulk starts at T = 0"""
    lat = Lattice(model, (nx, 2, 2))
    m = lat.model
    zi = lat.zone_index("heater")
    flags = np.full((lat.NZ, lat.NY, nx), m.node_type(collision).value, dtype=np.uint32)
    flags[:, :, :2] |= m.node_type(kind).value | (zi << m.zone_shift)
    if kind == "HeaterDirichletTemperatureABB":
        flags[:, :, :2] |= m.node_type("Wall").value
    lat.set_flags(flags)
    for k, v in dict(conductivity=0.1, nu=0.1, InitTemperature=0.0).items():
        lat.set_setting(k, v)
    lat.set_setting("InitTemperature", 1.0, zone="heater")
    lat.init()
    return lat


@pytest.mark.parametrize("model,collision", [("d3q27q7_cm_cht", "CM"), ("d3q27q27_cm_cht", "CM_HIGHER")])
@pytest.mark.parametrize("kind", ["HeaterDirichletTemperatureEQ", "HeaterDirichletTemperatureABB"])
def test_dirichlet_heater(kind, model, collision):
    lat = _heater_lat(kind, model=model, collision=collision)
    lat.iterate(400)
    t = lat.quantity("T")[0, 0, 0].double().numpy()
    inner = t[2:12]
    assert np.all(np.diff(inner) < 0), inner
    assert 0.0 < inner[-1] < inner[0] < 1.0, inner
    assert lat.globals["HeatSource"] > 0.0


def test_neumann_flux_q27_moments():
    """the east Neumann heater's D3Q27 increment (first, third and fifth order moments
    along the normal) carries no enthalpy: the HeatSource global stays zero"""
    lat = Lattice("d3q27q27_cm_cht", (4, 2, 2))
    m = lat.model
    zi = lat.zone_index("hot")
    fl = np.full((lat.NZ, lat.NY, 4), m.node_type("CM_HIGHER").value, dtype=np.uint32)
    fl[:, :, 0] |= m.node_type("HeaterNeumannHeatFluxEast").value | (zi << m.zone_shift)
    lat.set_flags(fl)
    lat.set_setting("InitTemperature", 1.0)
    lat.set_setting("InitHeatFlux", 0.01, zone="hot")
    lat.init()
    lat.iterate(1)
    assert abs(lat.globals["HeatSource"]) < 1e-12


def test_pressure_driven_channel():
    """W/E pressure planes drive a flow between bounce-back walls; the inflow imposes
    the inlet temperature on the heat populations"""
    nx, ny = 24, 9

    def extra(fl, m):
        fl[:, :, 0] = m.node_type("WPressure").value | m.node_type("CM").value
        fl[:, :, -1] = m.node_type("EPressure").value | m.node_type("CM").value
        fl[:, 0, :] = m.node_type("Wall").value
        fl[:, -1, :] = m.node_type("Wall").value

    lat = Lattice("d3q27q7_cm_cht", (nx, ny, 2))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, nx), m.node_type("CM").value, dtype=np.uint32)
    extra(fl, m)
    zi = lat.zone_index("inlet")
    fl[:, 1:-1, 0] |= zi << m.zone_shift
    lat.set_flags(fl)
    lat.set_setting("nu", 0.1)
    lat.set_setting("conductivity", 0.1)
    lat.set_setting("Pressure", 1e-4, zone="inlet")
    lat.set_setting("InitTemperature", 1.0, zone="inlet")
    lat.init()
    lat.iterate(600)
    u = lat.quantity("U")[0, 0].double().numpy()
    t = lat.quantity("T")[0, 0].double().numpy()
    mid = u[1:-1, nx // 2]
    assert mid.min() > 0, mid
    assert mid[len(mid) // 2] > mid[0], mid          # parabolic-like profile
    assert 0.0 < t[ny // 2, nx // 2] < 1.0 + 1e-9


@pytest.mark.parametrize("variant", [f"d3q27q{q}_cm_cht_{o}" for q in (7, 27) for o in
                                     ("OutFlowNeumann", "OutFlowConvective", "AVG", "CHT", "SMAG", "IBB")])
def test_variants_conserve_uniform_state(variant):
    coll = "CM" if "q7_" in variant else "CM_HIGHER"
    lat = _lat((6, 4, 4), coll, model=variant, InitTemperature=1.0, nu=0.1, conductivity=0.1)
    lat.iterate(10)
    assert abs(float(lat.quantity("T").double().mean()) - 1.0) < 1e-12
    assert float(lat.quantity("U").double().abs().max()) < 1e-12


CHT_XML = """<?xml version="1.0"?>
<CLBConfig version="2.0" output="output/" permissive="true">
  <Geometry nx="24" ny="10" nz="4">
    <CM><Box/></CM>
    <WVelocity name="Inlet"><Box nx="1"/></WVelocity>
    <EPressure name="Outlet"><Box dx="-1"/></EPressure>
    <Wall mask="ALL"><Box ny="1"/><Box dy="-1"/></Wall>
    <HeaterDirichletTemperatureEQ name="hot"><Box dx="10" nx="4" dy="1" ny="2"/></HeaterDirichletTemperatureEQ>
  </Geometry>
  <Model>
    <Param name="VelocityX" value="0.01"/>
    <Param name="nu" value="0.05"/>
    <Param name="conductivity" value="0.05"/>
    <Param name="InitTemperature" value="10"/>
    <Param name="InitTemperature" value="11" zone="hot"/>
  </Model>
  <VTK Iterations="100"/>
  <Log Iterations="50"/>
  <Solve Iterations="100"/>
</CLBConfig>"""


def test_cht_xml_case(tmp_path, monkeypatch):
    """XML case (Geometry zones, zonal Param, Solve, VTK, Log) on d3q27q7_cm_cht: the heated
    patch raises T, T stays within [9.9, 11], and the HeatSource global is logged"""
    import xml.etree.ElementTree as ET
    from tclb_amd import handlers  # noqa: F401
    from tclb_amd.io.vtk import read_vti
    from tclb_amd.solver import Solver
    monkeypatch.chdir(tmp_path)
    s = Solver("d3q27q7_cm_cht", ET.fromstring(CHT_XML), conffile=str(tmp_path / "case.xml"), device="cpu")
    s.run()
    assert s.iter == 100
    d = read_vti(str(tmp_path / "output" / "case_VTK_P00_00000100.vti"))
    t = np.asarray(d["T"])
    assert np.isfinite(t).all()
    # T = H / (rho cp): the start-up pressure waves from the inlet move rho, so T dips a
    # few per mille below the inflow value near the inlet
    assert 9.9 <= t.min() and t.max() <= 11.0 + 1e-6
    assert t.max() > 10.01
    log = open(tmp_path / "output" / "case_Log_P00_00000000.csv").read().splitlines()
    assert "HeatSource" in log[0]


def test_q27_collision_types_in_reference_order():
    """flag values follow the reference's registration order (models/heat/d3q27q27_cm_cht/
    Dynamics.R:114-119, BGK at :221), so raw NodeType dumps are interchangeable"""
    from tclb_amd.models import registry
    m = registry.get("d3q27q27_cm_cht")
    names = ["CM", "CM_HIGHER", "CM_HIGHER_PROB", "CM_HIGHER_PROB_M_EQ", "Cumulants", "Cumulants_HIGHER", "BGK"]
    vals = [m.node_type(n).value for n in names]
    assert vals == sorted(vals) and len(set(vals)) == len(vals)


def test_neumann_flux_q27_increment_moments():
    """the east Neumann heater adds raw moments m100 = n_x first, m120 = m102 = n_x first s2
    and m122 = n_x first s2^2 (first = -2 InitHeatFlux h_stability_enhancement, s2 = 1/3,
    reference ImposeHeatFlux): one step with and without the flux on heater nodes that do
    not collide, difference of the stored h, raw moments"""
    def run(flux):
        lat = Lattice("d3q27q27_cm_cht", (4, 3, 3))
        m = lat.model
        zi = lat.zone_index("hot")
        fl = np.full((lat.NZ, lat.NY, 4), m.node_type("CM_HIGHER").value, dtype=np.uint32)
        fl[:, :, 0] = m.node_type("HeaterNeumannHeatFluxEast").value | (zi << m.zone_shift)
        lat.set_flags(fl)
        lat.set_setting("InitTemperature", 1.0)
        lat.set_setting("InitHeatFlux", flux, zone="hot")
        lat.init()
        lat.iterate(1)
        dens = [d for d in m.densities if d.field.group == "h"]
        hi = [m.fields.index(d.field) for d in dens]
        C = np.array([[d.dx, d.dy, d.dz] for d in dens], dtype=float)
        return lat, C, lat.fields_interior()[hi][:, :, :, 0].numpy()
    lat, C, ha = run(0.01)
    _, _, hb = run(0.0)
    d = ha - hb
    hs = lat.svals[lat.gsettings.index("h_stability_enhancement")] if "h_stability_enhancement" in lat.gsettings else 1.0
    first = -2 * 0.01 * hs
    s2 = 1 / 3
    expect = {(1, 0, 0): -first, (1, 2, 0): -first * s2, (1, 0, 2): -first * s2, (1, 2, 2): -first * s2 * s2}
    for a in range(3):
        for b in range(3):
            for c in range(3):
                mom = np.tensordot(C[:, 0] ** a * C[:, 1] ** b * C[:, 2] ** c, d, 1)
                np.testing.assert_allclose(mom, expect.get((a, b, c), 0.0), atol=1e-15, err_msg=str((a, b, c)))


def _central_matrix(C, u):
    """A[(a, b, c), i] = prod_d (C[i, d] - u[d])^(exponent d), exponents a + 3 b + 9 c"""
    P = [(a, b, c) for c in range(3) for b in range(3) for a in range(3)]
    return np.array([[np.prod([(C[i, d] - u[d]) ** p[d] for d in range(3)]) for i in range(len(C))] for p in P]), P


def _oracle_q27(collision, h, C, om, uhyd, s2=1 / 3):
    """post-collision h of relax_and_collide_ADE_CM_HIGHER_PROB[_M_EQ], written from the
    reference formulas (models/heat/d3q27q27_cm_cht/Dynamics.c.Rt:1799-1831, 2008-2047):
    central moments about u_h = m1 / m0, odd orders relax with omega, even ones take the
    equilibrium; PROB returns about the blend u_hydro omega + u_h (1 - omega) with the
    z component blended from u_hydro.y, M_EQ about u_h with the equilibrium moving with
    du = u_hydro - u_h"""
    H = h.sum()
    uh = np.array([C[:, 0] @ h, C[:, 1] @ h, C[:, 2] @ h]) / H
    A, P = _central_matrix(C, uh)
    k = A @ h
    out = np.empty(27)
    du = uhyd - uh
    for q, p in enumerate(P):
        order = sum(p)
        if collision == "CM_HIGHER_PROB":
            eq = 0.0 if 1 in p else H * s2 ** sum(1 for e in p if e == 2)
        else:
            f = [1.0 if e == 0 else du[d] if e == 1 else s2 + du[d] ** 2 for d, e in enumerate(p)]
            eq = H * np.prod(f)
        if order % 2 == 1:
            out[q] = (1 - om) * k[q] + (om * eq if collision == "CM_HIGHER_PROB_M_EQ" else 0.0)
        else:
            out[q] = eq
    if collision == "CM_HIGHER_PROB":
        back = np.array([om * uhyd[0] + (1 - om) * uh[0], om * uhyd[1] + (1 - om) * uh[1],
                         om * uhyd[1] + (1 - om) * uh[2]])
    else:
        back = uh
    B, _ = _central_matrix(C, back)
    return np.linalg.solve(B, out)


@pytest.mark.parametrize("collision", ["CM_HIGHER_PROB", "CM_HIGHER_PROB_M_EQ"])
def test_q27_collision_with_moving_fluid(collision):
    """uniform periodic state with a moving fluid (u = (0.03, -0.02, 0.05)) and perturbed h:
    one step leaves every node at the post-collision h, which must equal an independent
    NumPy transcription of the reference formulas (exercises the u_hydro blend, including
    the reference's u_hydro.y in the z component, and the du-shifted equilibrium)"""
    k = 0.07
    U = np.array([0.03, -0.02, 0.05])
    lat = _lat((4, 4, 4), collision, model="d3q27q27_cm_cht", nu=0.1, conductivity=k, InitTemperature=1.0,
               VelocityX=U[0], VelocityY=U[1], VelocityZ=U[2])
    m = lat.model
    dens = [d for d in m.densities if d.field.group == "h"]
    hi = [m.fields.index(d.field) for d in dens]
    C = np.array([[d.dx, d.dy, d.dz] for d in dens], dtype=float)
    f = lat.fields_interior().clone()
    rng = np.random.default_rng(3)
    pert = 1 + 0.2 * rng.standard_normal(27)
    h0 = f[hi][:, 0, 0, 0].double().numpy() * pert
    f[hi] = torch.as_tensor(h0, dtype=f.dtype)[:, None, None, None].expand(-1, *f.shape[1:]).clone()
    lat.set_fields_interior(f)
    gi = [m.fields.index(d.field) for d in m.densities if d.field.group == "f"]
    Cg = np.array([[d.dx, d.dy, d.dz] for d in m.densities if d.field.group == "f"], dtype=float)
    g = f[gi][:, 0, 0, 0].double().numpy()
    uhyd = Cg.T @ g / g.sum()
    np.testing.assert_allclose(uhyd, U, atol=1e-12)
    lat.iterate(1)
    h1 = lat.fields_interior()[hi].double().numpy()
    expect = _oracle_q27(collision, h0, C, 1 / (3 * k + 0.5), uhyd)
    assert np.abs(h1 - expect[:, None, None, None]).max() < 1e-13, (h1[:, 0, 0, 0], expect)
    # the blend / moving equilibrium matters: a plain CM_HIGHER step gives another result
    plain = _oracle_q27("CM_HIGHER_PROB", h0, C, 1 / (3 * k + 0.5), np.array([uhyd[0], uhyd[1], uhyd[2]]))
    if collision == "CM_HIGHER_PROB_M_EQ":
        assert np.abs(plain - expect).max() > 1e-6
