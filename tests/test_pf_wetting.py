"""d3q27_pf_velocity wetting options (reference models/multiphase/d3q27_pf_velocity/
Boundary.c.Rt:260-1053, Dynamics.R:30-169): geometric contact-angle condition,
staircase improvement (exact wall normal, barycentric interpolation on the D3Q27 cube
surface), isograd and tprec."""
import math

import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice


def _lat(model, shape, solid_fn, angle, **settings):
    lat = Lattice(model, shape)
    m = lat.model
    nx, ny, nz = shape
    fl = np.full((lat.NZ, lat.NY, nx), m.node_type("MRT").value, dtype=np.uint32)
    z, y, x = np.meshgrid(np.arange(nz), np.arange(ny), np.arange(nx), indexing="ij")
    fl[solid_fn(x, y, z)] = m.node_type("Wall").value
    lat.add_zone("liquid")
    liquid = (x >= nx // 4) & (x < 3 * nx // 4) & ~solid_fn(x, y, z)
    fl[liquid] |= 1 << m.zone_shift
    lat.set_flags(fl.astype(np.uint16 if m.flag_bits == 16 else np.uint32))
    base = dict(Density_h=1.0, Density_l=1.0, sigma=0.01, IntWidth=4, M=0.02, Viscosity_l=0.1, Viscosity_h=0.1)
    base.update(settings)
    for k, v in base.items():
        lat.set_setting(k, v)
    lat.set_setting("PhaseField", 0.0)
    lat.set_setting("PhaseField", 1.0, zone="liquid")
    lat.set_setting("radAngle", angle)
    return lat


def floor(x, y, z):
    # two solid layers: z = 1 wets the fluid above it (a single layer would have fluid on
    # both sides through the periodic z wrap, and no defined normal)
    return z < 2


def test_geometric_wall_value_follows_contact_angle():
    """geometric condition: phi_wall = phi_1 + cot(theta) |grad_t phi| (2 h, h = 1/2), with
    the tangential gradient extrapolated from the first two fluid nodes (equal for a
    wall-normal interface)"""
    theta = math.radians(60)
    lat = _lat("d3q27_pf_velocity_geometric", (32, 4, 10), floor, theta)
    lat.init()
    phi = lat.quantity("PhaseField")[0].numpy()         # (z, y, x)
    g = lat.quantity("GradPhi")[0].numpy()               # x component
    for x in (6, 8, 10, 22, 24):
        # (the reference's PI = 3.14159265 enters tan(PI/2 - theta))
        expect = phi[2, 2, x] + abs(g[2, 2, x]) * math.tan(3.14159265 / 2 - theta)
        assert phi[1, 2, x] == pytest.approx(expect, abs=1e-12), x
    n = lat.quantity("Normal").numpy()
    assert (n[2, 1] == 1).all() and (n[:2, 1] == 0).all()


def test_staircase_on_axis_aligned_wall_equals_plain():
    """on a flat, lattice-aligned wall the exact normal is the lattice normal and the
    interpolation weights collapse onto one node: staircaseimp reproduces the plain
    surface-energy condition"""
    theta = math.radians(70)
    a = _lat("d3q27_pf_velocity", (24, 4, 8), floor, theta)
    b = _lat("d3q27_pf_velocity_staircaseimp", (24, 4, 8), floor, theta)
    for lat in (a, b):
        lat.init()
        lat.iterate(30)
    np.testing.assert_allclose(a.quantity("PhaseField").numpy(), b.quantity("PhaseField").numpy(), atol=1e-12)
    an = b.quantity("ActualNormal").numpy()[:, 1]
    np.testing.assert_allclose(an[2], 1.0)


def test_staircase_inclined_wall_normals():
    """45-degree wall (y + z < 4): the exact normal hits the cube surface at (0, 1, 1)/1,
    the lattice normal is the diagonal; interpolation weights are a partition of unity"""
    def slope(x, y, z):
        return y + z < 4
    lat = _lat("d3q27_pf_velocity_staircaseimp_tprec", (8, 12, 12), slope, math.radians(80))
    lat.init()
    m = lat.model
    an = lat.quantity("ActualNormal").numpy()
    nw = lat.quantity("Normal").numpy()
    fl = lat.get_flags()
    wall = (fl & m.group_masks["BOUNDARY"]) == m.node_type("Wall").value
    z, y, x = np.nonzero(wall)
    # wall nodes on the surface layer (a fluid neighbour along the diagonal)
    surf = (y + z == 3) & (y > 0) & (z > 0) & (y < 11) & (z < 11)
    assert surf.sum() > 10
    for k in np.nonzero(surf)[0]:
        np.testing.assert_allclose(an[:, z[k], y[k], x[k]], [0, 1, 1], atol=1e-12)
        np.testing.assert_allclose(nw[:, z[k], y[k], x[k]], [0, 1, 1], atol=1e-12)
    ci = [m.field_index(f"coeff_v{i}") for i in (1, 2, 3)]
    c = lat.fields_interior()[ci].numpy()
    s = c.sum(0)[wall & (lat.fields_interior()[m.field_index("triangle_index")].numpy() >= 0)]
    on = np.abs(lat.quantity("Normal").numpy()).sum(0)[wall] > 0
    np.testing.assert_allclose(s[on], 1.0, atol=1e-12)


@pytest.mark.parametrize("model", ["d3q27_pf_velocity_geometric", "d3q27_pf_velocity_geometric_isograd",
                                   "d3q27_pf_velocity_geometric_staircaseimp_isograd_tprec",
                                   "d3q27_pf_velocity_q27_staircaseimp"])
def test_wetting_variants_run_and_conserve_phase(model):
    def slope(x, y, z):
        return y + z < 3
    lat = _lat(model, (16, 10, 10), slope, math.radians(60))
    lat.init()
    fl = lat.get_flags()
    fluid = (fl & lat.model.group_masks["BOUNDARY"]) == 0
    phi0 = lat.quantity("PhaseField")[0].numpy()[fluid].sum()
    lat.iterate(40)
    phi = lat.quantity("PhaseField")[0].numpy()
    assert np.isfinite(phi).all() and np.isfinite(lat.quantity("U").numpy()).all()
    assert abs(phi[fluid].sum() - phi0) < 0.02 * phi0
    assert np.abs(phi[~fluid]).max() < 1e9           # every special point was corrected
