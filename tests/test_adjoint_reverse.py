"""Hand-written reverse sweeps of the node update (Model.set_reverse; d3q19_adj rev_run,
the counterpart of the reference's Tapenade Run_b) against the dual-number adjoint of the
same node code: the unsteady adjoint state, the objective and the design gradient agree
to rounding, with Zou/He pressure and velocity planes, bounce-back, solid, flag-free and
non-MRT nodes (reverse sweeps) and a limited-pressure node (dual passes) in one lattice, objectives on Inlet/Outlet planes and the material penalty; with a
seeded setting the sweeps step aside (dual passes everywhere)."""
import numpy as np
import pytest
import torch

from tclb_amd.adjoint import Adjoint
from tclb_amd.lattice import Lattice


def _case(device, reverse, settings=()):
    nx, ny, nz = 12, 6, 8
    lat = Lattice("d3q19_adj", (nx, ny, nz), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, :, 0] = m.node_type("WPressure").value | mrt
    fl[:, :, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, :, 8] |= m.node_type("Outlet").value
    fl[:, :, 2] |= m.node_type("Inlet").value
    fl[:, :, 4:7] |= m.node_type("DesignSpace").value
    fl[:, 0, 3] = m.node_type("Wall").value
    fl[:, 1, 9] = m.node_type("WVelocity").value | mrt
    fl[:, 2, 9] = m.node_type("Solid").value | mrt
    fl[:, 3, 9] = m.node_type("WPressureL").value | mrt
    fl[:, 4, 9] = m.node_type("BGK").value
    fl[2, 5, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu": 0.1, "InletDensity": 1.03, "FluxInObj": 1.0, "EnergyFluxInObj": 0.3,
                 "PressureFluxInObj": -0.2, "PressureDiffInObj": 0.7, "MaterialPenaltyInObj": 0.05,
                 "Theta": 1.3, "InletVelocity": 0.01}.items():
        lat.set_setting(k, v)
    lat.init()
    wi = m.field_index("w")
    f = lat.fields_interior().clone()
    z = torch.arange(nz, dtype=f.dtype, device=f.device)[:, None, None]
    y = torch.arange(ny, dtype=f.dtype, device=f.device)[None, :, None]
    f[wi, :, :, 4:7] = (0.55 + 0.03 * z + 0.02 * y).expand(nz, ny, 3)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, settings=settings, reverse=reverse)
    ad.unsteady(10)
    return lat, ad


def _check(device):
    lat_r, r = _case(device, True)
    lat_d, d = _case(device, False)
    a, b = r.a0.cpu(), d.a0.cpu()
    scale = b.abs().max().item()
    assert scale > 0
    assert torch.allclose(a, b, rtol=0, atol=1e-12 * scale), (a - b).abs().max().item() / scale
    assert abs(r.J - d.J) <= 1e-13 * abs(d.J)
    gw_r, gw_d = r.field_gradient("w"), d.field_gradient("w")
    assert np.abs(gw_d).max() > 0
    np.testing.assert_allclose(gw_r, gw_d, rtol=0, atol=1e-12 * np.abs(gw_d).max())
    return r


def test_reverse_sweep_matches_dual_cpu():
    _check("cpu")


def test_seeded_setting_uses_dual_passes():
    lat, ad = _case("cpu", True, settings=["Theta"])
    assert ad._seeded and ad.setting_gradient("Theta") != 0.0
    lat2, ad2 = _case("cpu", False, settings=["Theta"])
    assert ad.setting_gradient("Theta") == pytest.approx(ad2.setting_gradient("Theta"), rel=1e-12)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_reverse_sweep_matches_dual_gpu():
    r = _check("cuda")
    assert r.lib.kind == "adhip" if hasattr(r.lib, "kind") else True


# ---------------------------------------------------------------- d3q19_heat_adj
def _heat_case(device, reverse, steps=8):
    """heat-exchanger lattice: walls, MRT fluid with heaters, thermometers, an outlet plane,
    a design block, a BGK and a flag-free node; every objective weight on"""
    nx, ny, nz = 12, 7, 6
    lat = Lattice("d3q19_heat_adj", (nx, ny, nz), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, :] = m.node_type("Wall").value
    fl[:, 1:3, 3] |= m.node_type("Heater").value
    fl[:, 3, 6] |= m.node_type("Thermometer").value
    fl[:, 4, 7] |= m.node_type("Thermometer").value
    fl[:, 1:ny - 1, 9] |= m.node_type("Outlet").value
    fl[:, 2:5, 4:6] |= m.node_type("DesignSpace").value
    fl[1, 3, 10] = m.node_type("BGK").value
    fl[2, 3, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu": 0.1, "FluidAlpha": 0.08, "Velocity": 0.02, "Temperature": 1.3, "LimitTemperature": 1.05,
                 "FluxInObj": 0.4, "HeatFluxInObj": 1.0, "HeatSquareFluxInObj": -0.3,
                 "TemperatureAtPointInObj": 0.6, "HighTemperatureInObj": 2.0, "LowTemperatureInObj": 0.7,
                 "MaterialPenaltyInObj": 0.05}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(3)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi = m.field_index("w")
    f[wi] = (0.4 + 0.5 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def _check_heat(device):
    lat_r, r = _heat_case(device, True)
    lat_d, d = _heat_case(device, False)
    a, b = r.a0.cpu(), d.a0.cpu()
    scale = b.abs().max().item()
    assert scale > 0
    assert torch.allclose(a, b, rtol=0, atol=1e-12 * scale), (a - b).abs().max().item() / scale
    assert abs(r.J - d.J) <= 1e-13 * abs(d.J)
    gw_r, gw_d = r.field_gradient("w"), d.field_gradient("w")
    assert np.abs(gw_d).max() > 0
    np.testing.assert_allclose(gw_r, gw_d, rtol=0, atol=1e-12 * np.abs(gw_d).max())
    return r


def test_heat_reverse_sweep_matches_dual_cpu():
    """d3q19_heat_adj rev_run (emitter-differentiated equilibria, transposed moment
    maps) = the dual-number adjoint of Run, every node type"""
    _check_heat("cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_heat_reverse_sweep_matches_dual_gpu():
    _check_heat("cuda")


# ---------------------------------------------------------------- d3q19_heat_adj_art
def _art_case(device, reverse, steps=8):
    """article heat exchanger: W velocity / pressure inlets, a limited-pressure node and an
    E outlet (dual passes), walls, heaters, thermometers, outlet plane, design block"""
    nx, ny, nz = 12, 7, 6
    lat = Lattice("d3q19_heat_adj_art", (nx, ny, nz), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, :] = m.node_type("Wall").value
    fl[:, 1:4, 0] = m.node_type("WVelocity").value | mrt
    fl[:, 4:ny - 1, 0] = m.node_type("WPressure").value | mrt
    fl[:, 3, 0] = m.node_type("WPressureL").value | mrt
    fl[:, 1:ny - 1, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 1:3, 3] |= m.node_type("Heater").value
    fl[:, 3, 6] |= m.node_type("Thermometer").value
    fl[:, 4, 7] |= m.node_type("Thermometer").value
    fl[:, 1:ny - 1, 9] |= m.node_type("Outlet").value
    fl[:, 2:5, 4:6] |= m.node_type("DesignSpace").value
    fl[1, 3, 10] = m.node_type("BGK").value
    fl[2, 3, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu": 0.1, "FluidAlpha": 0.08, "SolidAlpha": 0.02, "Velocity": 0.02, "Pressure": 0.003,
                 "Temperature": 1.3, "LimitTemperature": 1.05, "FluxInObj": 0.4, "HeatFluxInObj": 1.0,
                 "HeatSquareFluxInObj": -0.3, "TemperatureAtPointInObj": 0.6, "HighTemperatureInObj": 2.0,
                 "LowTemperatureInObj": 0.7, "HeatInputInObj": 0.25, "MaterialPenaltyInObj": 0.05}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(4)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi = m.field_index("w")
    f[wi] = (0.4 + 0.5 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def _check_art(device):
    lat_r, r = _art_case(device, True)
    lat_d, d = _art_case(device, False)
    a, b = r.a0.cpu(), d.a0.cpu()
    scale = b.abs().max().item()
    assert scale > 0
    assert torch.allclose(a, b, rtol=0, atol=1e-12 * scale), (a - b).abs().max().item() / scale
    assert abs(r.J - d.J) <= 1e-13 * abs(d.J)
    gw_r, gw_d = r.field_gradient("w"), d.field_gradient("w")
    assert np.abs(gw_d).max() > 0
    np.testing.assert_allclose(gw_r, gw_d, rtol=0, atol=1e-12 * np.abs(gw_d).max())
    return r


def test_art_reverse_sweep_matches_dual_cpu():
    """d3q19_heat_adj_art rev_run (collision transpose + probed affine inlets/walls; the
    limited inlet and the outlet on dual passes) = the dual-number adjoint"""
    _check_art("cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_art_reverse_sweep_matches_dual_gpu():
    _check_art("cuda")


# ---------------------------------------------------------------- d2q9_adj
def _d2q9_case(device, reverse, steps=10):
    """porous channel: W velocity / pressure inlets, E pressure / velocity outlets, walls,
    solid, BGK and flag-free nodes, inlet / outlet objective planes, a design block"""
    nx, ny = 16, 10
    lat = Lattice("d2q9_adj", (nx, ny, 1), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, :] = m.node_type("Wall").value
    fl[:, 1:5, 0] = m.node_type("WVelocity").value | mrt
    fl[:, 5:ny - 1, 0] = m.node_type("WPressure").value | mrt
    fl[:, 1:6, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 6:ny - 1, nx - 1] = m.node_type("EVelocity").value | mrt
    fl[:, 1:ny - 1, 2] |= m.node_type("Inlet").value
    fl[:, 1:ny - 1, 12] |= m.node_type("Outlet").value
    fl[:, 3:7, 5:9] |= m.node_type("DesignSpace").value
    fl[:, 4, 10] = m.node_type("Solid").value | mrt
    fl[:, 5, 10] = m.node_type("BGK").value
    fl[:, 6, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu": 0.1, "Velocity": 0.02, "Pressure": 0.002, "ForceX": 1e-5, "ForceY": -2e-6,
                 "PorocityTheta": -1.2, "DragInObj": 0.3, "LiftInObj": -0.2, "MaterialPenaltyInObj": 0.05,
                 "MaterialInObj": 0.02, "PressureLossInObj": 1.0, "OutletFluxInObj": 0.5,
                 "InletFluxInObj": -0.4}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(6)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi = m.field_index("w")
    f[wi] = (0.4 + 0.5 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def _check_d2q9(device):
    lat_r, r = _d2q9_case(device, True)
    lat_d, d = _d2q9_case(device, False)
    a, b = r.a0.cpu(), d.a0.cpu()
    scale = b.abs().max().item()
    assert scale > 0
    assert torch.allclose(a, b, rtol=0, atol=1e-12 * scale), (a - b).abs().max().item() / scale
    assert abs(r.J - d.J) <= 1e-13 * abs(d.J)
    gw_r, gw_d = r.field_gradient("w"), d.field_gradient("w")
    assert np.abs(gw_d).max() > 0
    np.testing.assert_allclose(gw_r, gw_d, rtol=0, atol=1e-12 * np.abs(gw_d).max())
    return r


def test_d2q9_adj_reverse_sweep_matches_dual_cpu():
    """d2q9_adj rev_run (hand-transposed porous MRT collision, probed Zou/He planes and
    bounce-back) = the dual-number adjoint, every node type"""
    _check_d2q9("cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_d2q9_adj_reverse_sweep_matches_dual_gpu():
    _check_d2q9("cuda")


# ---------------------------------------------------------------- d2q9_heat_adj
def _d2q9_heat_case(device, reverse, steps=10):
    nx, ny = 16, 10
    lat = Lattice("d2q9_heat_adj", (nx, ny, 1), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, :] = m.node_type("Wall").value
    fl[:, 1:4, 0] = m.node_type("WVelocity").value | mrt
    fl[:, 4, 0] = m.node_type("WVelocity").value | m.node_type("Heater").value | mrt
    fl[:, 5:ny - 1, 0] = m.node_type("WPressure").value | mrt
    fl[:, 1:6, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 6:ny - 1, nx - 1] = m.node_type("EVelocity").value | mrt
    fl[:, 2:4, 4] |= m.node_type("Heater").value
    fl[:, 5, 7] |= m.node_type("Thermometer").value
    fl[:, 6, 8] |= m.node_type("Thermometer").value
    fl[:, 1:ny - 1, 12] |= m.node_type("Outlet").value
    fl[:, 4, 10] = m.node_type("Solid").value | mrt
    fl[:, 6, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu0": 0.1, "InletVelocity": 0.02, "InletPressure": 0.003, "InletTemperature": 1.1,
                 "InitTemperature": 1.0, "HeaterTemperature": 1.4, "FluidAlpha": 0.08, "SolidAlpha": 0.03,
                 "LimitTemperature": 1.05, "FluxInObj": 0.4, "HeatFluxInObj": 1.0, "HeatSquareFluxInObj": -0.3,
                 "TemperatureInObj": 0.6, "HighTemperatureInObj": 2.0, "LowTemperatureInObj": 0.7}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(7)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi = m.field_index("w")
    f[wi] = (0.4 + 0.5 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def _check_d2q9_heat(device):
    lat_r, r = _d2q9_heat_case(device, True)
    lat_d, d = _d2q9_heat_case(device, False)
    a, b = r.a0.cpu(), d.a0.cpu()
    scale = b.abs().max().item()
    assert scale > 0
    assert torch.allclose(a, b, rtol=0, atol=1e-12 * scale), (a - b).abs().max().item() / scale
    assert abs(r.J - d.J) <= 1e-13 * abs(d.J)
    gw_r, gw_d = r.field_gradient("w"), d.field_gradient("w")
    assert np.abs(gw_d).max() > 0
    np.testing.assert_allclose(gw_r, gw_d, rtol=0, atol=1e-12 * np.abs(gw_d).max())


def test_d2q9_heat_adj_reverse_sweep_matches_dual_cpu():
    _check_d2q9_heat("cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_d2q9_heat_adj_reverse_sweep_matches_dual_gpu():
    _check_d2q9_heat("cuda")


# ---------------------------------------------------------------- sw (shallow water)
def _sw_case(device, reverse, steps=10):
    nx, ny = 16, 10
    lat = Lattice("sw", (nx, ny, 1), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, :] = m.node_type("Wall").value
    fl[:, 1:5, 0] = m.node_type("WVelocity").value | mrt
    fl[:, 5:ny - 1, 0] = m.node_type("WPressure").value | mrt
    fl[:, 1:6, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 6:ny - 1, nx - 1] = m.node_type("EVelocity").value | mrt
    fl[:, 2:7, 5:9] |= m.node_type("Obj1").value
    fl[:, 4, 10] = m.node_type("BGK").value
    fl[:, 6, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu": 0.1, "InletVelocity": 0.01, "Gravity": 0.2, "Height": 1.0, "EnergySink": 0.1,
                 "TotalDiffInObj": 0.5, "EnergyGainInObj": 1.0, "MaterialInObj": 0.05}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(8)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi = m.field_index("w")
    f[wi] = (0.4 + 0.5 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def _check_generic(case, device, param="w"):
    lat_r, r = case(device, True)
    lat_d, d = case(device, False)
    assert r.reverse and not d.reverse
    a, b = r.a0.cpu(), d.a0.cpu()
    scale = b.abs().max().item()
    assert scale > 0
    assert torch.allclose(a, b, rtol=0, atol=1e-12 * scale), (a - b).abs().max().item() / scale
    assert abs(r.J - d.J) <= 1e-13 * abs(d.J)
    if param is None:           # a model without a design field: the state adjoint only
        return
    gw_r, gw_d = r.field_gradient(param), d.field_gradient(param)
    assert np.abs(gw_d).max() > 0
    np.testing.assert_allclose(gw_r, gw_d, rtol=0, atol=1e-12 * np.abs(gw_d).max())


def test_sw_reverse_sweep_matches_dual_cpu():
    _check_generic(_sw_case, "cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_sw_reverse_sweep_matches_dual_gpu():
    _check_generic(_sw_case, "cuda")


# ---------------------------------------------------------------- d2q9_diff
def _diff_case(device, reverse, steps=10):
    nx, ny = 16, 10
    lat = Lattice("d2q9_diff", (nx, ny, 1), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, :] = m.node_type("Wall").value
    fl[:, 1:ny - 1, 0] = m.node_type("WPressure").value | mrt
    fl[:, 1:ny - 1, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 2:5, 5:9] |= m.node_type("Obj1").value
    fl[:, 6:8, 5:9] |= m.node_type("Obj2").value
    fl[:, 5, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu0": 0.05, "nu1": 0.2, "InitDensity": 1.0, "InletDensity": 1.02, "OutletDensity": 0.99,
                 "DiffInObj": 1.0}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(9)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi, ri = m.field_index("w"), m.field_index("r")
    f[wi] = (0.2 + 0.6 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    f[ri] = (0.9 + 0.2 * torch.rand(f[ri].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def test_d2q9_diff_reverse_sweep_matches_dual_cpu():
    _check_generic(_diff_case, "cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_d2q9_diff_reverse_sweep_matches_dual_gpu():
    _check_generic(_diff_case, "cuda")


# ---------------------------------------------------------------- d3q19_heat_adj_prop
def _prop_case(device, reverse, steps=8):
    nx, ny, nz = 12, 7, 6
    lat = Lattice("d3q19_heat_adj_prop", (nx, ny, nz), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, :] = m.node_type("Wall").value
    fl[:, 1:4, 0] = m.node_type("WVelocity").value | mrt
    fl[:, 4:ny - 1, 0] = m.node_type("WPressure").value | mrt
    fl[:, 3, 0] = m.node_type("WPressureL").value | mrt
    fl[:, 1:ny - 1, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 1:3, 3] |= m.node_type("Heater").value
    fl[:, 4:6, 3] |= m.node_type("HeatSource").value
    fl[:, 3, 6] |= m.node_type("Thermometer").value
    fl[:, 1:ny - 1, 9] |= m.node_type("Outlet").value
    fl[:, 2:5, 4:8] |= m.node_type("DesignSpace").value
    fl[:, 2:5, 5:8] |= m.node_type("Propagate").value
    fl[1, 3, 10] = m.node_type("BGK").value
    fl[2, 3, 10] = 0
    lat.set_flags(fl)
    for k, v in {"nu": 0.1, "FluidAlpha": 0.08, "SolidAlpha": 0.02, "InletVelocity": 0.02, "InletPressure": 0.003,
                 "InletTemperature": 1.1, "HeaterTemperature": 1.3, "HeatSource": 0.01, "LimitTemperature": 1.05,
                 "PropagateX": 0.3, "FluxInObj": 0.4, "HeatFluxInObj": 1.0, "HeatSquareFluxInObj": -0.3,
                 "TemperatureInObj": 0.6, "HighTemperatureInObj": 2.0, "LowTemperatureInObj": 0.7,
                 "MaterialPenaltyInObj": 0.05}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(10)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi = m.field_index("w")
    f[wi] = (0.4 + 0.5 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def test_prop_reverse_sweep_matches_dual_cpu():
    _check_generic(_prop_case, "cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_prop_reverse_sweep_matches_dual_gpu():
    _check_generic(_prop_case, "cuda")


# ---------------------------------------------------------------- d2q9_optimalMixing
def _mixing_case(device, reverse, steps=10):
    nx, ny = 14, 10
    lat = Lattice("d2q9_optimalMixing", (nx, ny, 1), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, :, 0] = m.node_type("Wall").value
    fl[:, :, nx - 1] = m.node_type("Solid").value
    fl[:, ny - 1, 1:nx - 1] = m.node_type("NMovingWall").value | mrt
    fl[:, 4, 6] = 0
    lat.set_flags(fl)
    for k, v in {"nu": 0.08, "K": 0.05, "MovingWallVelocity": 0.05, "TotalTempSqrInObj": 1.0,
                 "NMovingWallForceInObj": 0.7, "MovingWallPowerInObj": -2.0}.items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(11)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    for i in range(5):                         # a temperature pattern to mix
        gi = m.field_index(f"g[{i}]")
        f[gi] = (0.1 + 0.2 * torch.rand(f[gi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def test_optimalmixing_reverse_sweep_matches_dual_cpu():
    _check_generic(_mixing_case, "cpu", param=None)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_optimalmixing_reverse_sweep_matches_dual_gpu():
    _check_generic(_mixing_case, "cuda", param=None)


# ---------------------------------------------------------------- d2q9_plate
def _plate_case(device, reverse, steps=10, bf=1.0):
    nx, ny = 18, 12
    lat = Lattice("d2q9_plate", (nx, ny, 1), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, ny - 1, 1:nx - 1] = m.node_type("NVelocity").value | mrt
    fl[:, 1:7, 0] = m.node_type("WVelocity").value | mrt
    fl[:, 7:ny, 0] = m.node_type("WPressure").value | mrt
    fl[:, 1:ny, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 1, 1:nx - 1] = m.node_type("SPressure").value | mrt
    fl[:, 5, 12] = m.node_type("Solid").value
    lat.set_flags(fl)
    for k, v in {"nu": 0.05, "VelocityX": 0.03, "VelocityY": 0.01, "Smag": 0.3, "PRAD": 2.5, "SM": 2.0,
                 "BF": bf, "PX": 7.3, "PY": 5.6, "PR": 0.4, "ExternalForceX": 1e-4,
                 "ForceXInObj": 1.0, "ForceYInObj": -0.5, "MomentInObj": 0.2, "PowerXInObj": 0.3,
                 "PowerYInObj": 0.4, "PowerRInObj": -0.6, "PowerInObj": 0.8, "VolumeWInObj": 0.05}.items():
        lat.set_setting(k, v)
    for k, v in {"PX": 0.02, "PY": -0.01, "PR": 0.03}.items():
        lat.set_setting_dt(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(12)
    f = f * (1 + 0.03 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def test_plate_reverse_sweep_matches_dual_cpu():
    _check_generic(_plate_case, "cpu", param=None)
    _check_generic(lambda dev, rev: _plate_case(dev, rev, bf=0.0), "cpu", param=None)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_plate_reverse_sweep_matches_dual_gpu():
    _check_generic(_plate_case, "cuda", param=None)


# ---------------------------------------------------------------- d2q9_kuper_adj
def _kuper_case(device, reverse, steps=10):
    nx, ny = 16, 10
    lat = Lattice("d2q9_kuper_adj", (nx, ny, 1), device=torch.device(device))
    m = lat.model
    mrt = m.node_type("MRT").value
    fl = np.full((lat.NZ, lat.NY, nx), mrt, dtype=np.uint32)
    fl[:, 0, :] = m.node_type("Wall").value
    fl[:, 0, 4:8] |= m.node_type("Wet").value
    fl[:, ny - 1, :] = m.node_type("MovingWall").value
    fl[:, 1:5, 0] = m.node_type("WVelocity").value | mrt
    fl[:, 5:ny - 1, 0] = m.node_type("WPressure").value | mrt
    fl[:, 1:5, nx - 1] = m.node_type("EPressure").value | mrt
    fl[:, 5:ny - 1, nx - 1] = m.node_type("EVelocity").value | mrt
    fl[:, 2:5, 5:9] |= m.node_type("Obj1").value
    fl[:, 6:8, 5:9] |= m.node_type("Obj2").value
    fl[:, 1, 10:13] |= m.node_type("Obj3").value
    fl[:, 4, 11] = m.node_type("BGK").value
    fl[:, 6, 12] = m.node_type("Solid").value
    lat.set_flags(fl)
    for k, v in dict(InitDensity=1.0, WallDensity=1.05, WetDensity=1.1, Temperature=0.56, FAcc=1.0, Magic=0.01,
                     MagicA=-0.152, MagicF=1.0, Wetting=0.7, GravitationX=1e-3, GravitationY=-2e-4, nu=0.1,
                     InletVelocity=0.01, InletDensity=1.02, OutletDensity=0.99, MovingWallVelocity=0.02,
                     FluidVelocityXInObj=1.0, Pressure1InObj=0.5, Pressure2InObj=-0.3, Pressure3InObj=0.2,
                     Density1InObj=0.4, Density2InObj=0.1, Density3InObj=-0.7).items():
        lat.set_setting(k, v)
    lat.init()
    f = lat.fields_interior().clone()
    g = torch.Generator().manual_seed(13)
    f = f * (1 + 0.02 * torch.rand(f.shape, generator=g, dtype=f.dtype)).to(f.device)
    wi = m.field_index("w")
    f[wi] = (0.4 + 0.5 * torch.rand(f[wi].shape, generator=g, dtype=f.dtype)).to(f.device)
    lat.set_fields_interior(f)
    ad = Adjoint(lat, reverse=reverse)
    ad.unsteady(steps)
    return lat, ad


def test_kuper_adj_reverse_sweep_matches_dual_cpu():
    _check_generic(_kuper_case, "cpu")


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="no GPU")
def test_kuper_adj_reverse_sweep_matches_dual_gpu():
    _check_generic(_kuper_case, "cuda")
