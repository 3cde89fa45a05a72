"""d3q27_pf_velocity option variants (reference models/multiphase/d3q27_pf_velocity):

* ``thermo``: the explicit energy-equation stages reproduce the reference's RK scheme
  exactly (thermo.c.Rt:96-170, including the sign of its fourth conduction slope), and a
  drop in a temperature gradient migrates towards the hot side (sigma_T < 0) at the
  order of the Young-Goldstein-Block velocity;
* ``thermo_planarBenchmark``: the heated bottom wall / cold top wall initialisation and
  the tanh layer of the planar thermocapillary benchmark;
* ``OutFlow``: Neumann outlets copy the upstream populations; ``autosym``: a half domain
  with a symmetry plane reproduces the full domain.
"""
import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice


def _lat(model, shape, flags_fn=None, **settings):
    lat = Lattice(model, shape)
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, shape[0]), m.node_type("MRT").value, dtype=np.uint32)
    if flags_fn is not None:
        flags_fn(m, lat, fl)
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    base = dict(Density_h=1.0, Density_l=1.0, sigma=0.01, IntWidth=4, M=0.02, Viscosity_l=0.1,
                Viscosity_h=0.1, PhaseField=1.0)
    base.update(settings)
    for k, v in base.items():
        lat.set_setting(k, v)
    return lat


def test_thermo_rk_scheme_matches_reference_polynomial():
    n = 16
    k_h, cp_h, rho_h, stab = 0.3, 2.0, 1.5, 0.8
    lat = _lat("d3q27_pf_velocity_thermo", (n, 4, 4), k_h=k_h, k_l=k_h, cp_h=cp_h, cp_l=cp_h,
               Density_h=rho_h, Density_l=rho_h, stabiliser=stab, T_init=0.0)
    lat.init()
    fi = lat.model.field_index("Temp")
    st = lat.fields_interior().clone()
    x = np.arange(n)
    k = 2 * np.pi / n
    T0 = 0.7 * np.cos(k * x)
    st[fi] = torch.as_tensor(np.broadcast_to(T0, st[fi].shape).copy(), dtype=st.dtype)
    st[lat.model.field_index("Cond")] = k_h
    lat.set_fields_interior(st)
    lat.run_action("TempToSteadyState", glob=True)
    T1 = lat.field("Temp")[0, 0].numpy()
    lam = stab * k_h / (rho_h * cp_h) * 2 * (np.cos(k) - 1)
    G = 1 + 2 * lam / 3 + lam ** 2 / 6 - lam ** 4 / 24
    np.testing.assert_allclose(T1, G * T0, rtol=0, atol=1e-13)
    assert lat.globals["TempChange"] > 0


def test_thermo_surface_tension_follows_temperature():
    lat = _lat("d3q27_pf_velocity_thermo", (8, 8, 4), T_init=2.0, sigma_T=-0.002, T_ref=1.0,
               k_h=0.1, k_l=0.1, cp_h=1.0, cp_l=1.0)
    lat.init()
    lat.iterate(2)
    st = lat.quantity("ST")[0].numpy()
    np.testing.assert_allclose(st, 0.01 - 0.002 * (2.0 - 1.0), rtol=1e-12)
    np.testing.assert_allclose(lat.quantity("T")[0].numpy(), 2.0, rtol=1e-12)


def _centroid_y(lat):
    phi = lat.quantity("PhaseField")[0].double().numpy()
    w = np.clip(phi, 0, 1)
    y = np.arange(phi.shape[1])[None, :, None]
    return float((w * y).sum() / w.sum())


def test_thermocapillary_drop_migrates_to_hot_side():
    nx, ny, nz, R0 = 24, 44, 24, 6.0
    dT, sigma_T, nu = 0.05, -0.002, 0.1

    def walls(m, lat, fl):
        w = m.node_type("Wall").value | m.node_type("ConstantTemp").value
        fl[:, lat.gy, :] = w
        fl[:, lat.gy + ny - 1, :] = w
    lat = _lat("d3q27_pf_velocity_thermo", (nx, ny, nz), walls, Radius=R0, CenterX=nx / 2, CenterY=ny / 2,
               CenterZ=nz / 2, BubbleType=1.0, PhaseField=0.0, sigma_T=sigma_T, T_ref=0.0, T_init=0.0, dT=dT,
               k_h=0.05, k_l=0.05, cp_h=1.0, cp_l=1.0, Viscosity_l=nu, Viscosity_h=nu)
    lat.init()
    lat.iterate(300)
    y1 = _centroid_y(lat)
    lat.iterate(300)
    y2 = _centroid_y(lat)
    v = (y2 - y1) / 300
    # Young-Goldstein-Block drift of a drop with equal viscosity and conductivity
    mu = nu * 1.0
    v_ygb = 2 * abs(sigma_T) * dT * R0 / ((2 * mu + 3 * mu) * (2 + 1))
    assert v > 0, v                       # towards increasing temperature
    assert 0.2 * v_ygb < v < 1.5 * v_ygb, (v, v_ygb)


def test_planar_benchmark_initialisation():
    nx, ny = 20, 12

    def walls(m, lat, fl):
        fl[:, lat.gy, :] = m.node_type("Wall").value | m.node_type("BWall").value
        fl[:, lat.gy + ny - 1, :] = m.node_type("Wall").value | m.node_type("TWall").value
    lat = _lat("d3q27_pf_velocity_thermo_planarBenchmark", (nx, ny, 2), walls, T_h=20, T_c=10, T_0=4, myL=10,
               MIDPOINT=6, PLUSMINUS=1, IntWidth=4, k_h=0.1, k_l=0.2, cp_h=1, cp_l=1, T_init=15)
    lat.init()
    T = lat.field("Temp")[0].numpy()
    x = np.arange(nx)
    np.testing.assert_allclose(T[0], 20 + 4 * np.cos(np.pi / 10 * ((x - 0.5) - 10)), rtol=1e-12)
    np.testing.assert_allclose(T[ny - 1], 10.0)
    np.testing.assert_allclose(T[3], 15.0)
    phi = lat.field("PhaseF")[0, :, 0].numpy()
    y = np.arange(ny)
    np.testing.assert_allclose(phi[1:-1], (0.5 + 0.5 * np.tanh((y - 6) / 2.0))[1:-1], rtol=1e-12)


def test_outflow_neumann_copies_upstream():
    """an ENeumann column takes the populations pulled one node upstream (x-1)"""
    nx = 12

    def outlet(m, lat, fl):
        fl[:, :, nx - 1] = m.node_type("ENeumann").value | m.node_type("MRT").value
    lat = _lat("d3q27_pf_velocity_OutFlow", (nx, 6, 4), outlet, VelocityX=0.01, PhaseField=1.0)
    lat.init()
    lat.iterate(20)
    u = lat.quantity("U")[0].numpy()
    assert np.isfinite(u).all()
    np.testing.assert_allclose(u[..., nx - 1], u[..., nx - 2], rtol=0, atol=2e-3)


def test_autosym_half_domain_matches_full_domain():
    """symmetry planes at x = 0 (SymmetryX_minus) and x = L (SymmetryX_plus): a drop
    centred on the first plane in the half domain evolves like the drop in the periodic
    full domain of length 2L, which is even about both planes"""
    L, ny, nz = 10, 16, 4
    st = dict(Density_h=1.0, Density_l=0.5, Radius=5.0, CenterY=ny / 2, CenterZ=nz / 2, BubbleType=1.0,
              PhaseField=0.0, GravitationY=-1e-5)
    full = _lat("d3q27_pf_velocity", (2 * L, ny, nz), CenterX=L, **st)
    full.init()
    full.iterate(40)
    phi_full = full.quantity("PhaseField")[0].numpy()

    def sym(m, lat, fl):
        fl[..., 0] = m.node_type("SymmetryX_minus").value | m.node_type("MRT").value
        fl[..., L] = m.node_type("SymmetryX_plus").value | m.node_type("MRT").value
    half = _lat("d3q27_pf_velocity_autosym", (L + 1, ny, nz), sym, CenterX=0.0, **st)
    half.init()
    half.iterate(40)
    phi_half = half.quantity("PhaseField")[0].numpy()
    ref = phi_full[..., [(L + i) % (2 * L) for i in range(L + 1)]]
    # equal up to round-off: mirrored stencils sum the same values in another order
    # (1e-16 after one step, grown to ~1e-8 after 40)
    np.testing.assert_allclose(phi_half, ref, rtol=0, atol=1e-7)
    assert np.abs(phi_half - phi_half[..., ::-1]).max() > 0.1     # the drop is not trivially uniform
