"""d3q27_pf_velocity (two distribution sets: g D3Q27 hydrodynamics + h D3Q15 phase field).

Oracle: the Laplace law dp = 2 sigma / R for a resting droplet, conservation of the
phase field, and a droplet that stays put.  The reference ships no goldens for this
model (tests/external is empty), so these are analytic checks ("parity unpinned").
Also covered: the multi-stage Iteration action (BaseIter, calcPhase, calcWall,
calcWallPhase_correction) and wall-normal initialisation next to a solid plate."""
import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice

SET = {"Density_h": 1.0, "Density_l": 0.1, "sigma": 0.01, "Viscosity_l": 0.1, "Viscosity_h": 0.1,
       "M": 0.05, "BubbleType": 1.0, "IntWidth": 4.0}


def droplet(n=24, R=6.0, device="cpu", name="d3q27_pf_velocity"):
    lat = Lattice(name, (n, n, n), device=torch.device(device), precision="double")
    fl = np.full((lat.NZ, lat.NY, n), lat.model.node_type("MRT").value, dtype=np.uint32)
    lat.set_flags(fl)
    for k, v in SET.items():
        lat.set_setting(k, v)
    c = n / 2
    for k, v in {"Radius": R, "CenterX": c, "CenterY": c, "CenterZ": c}.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


@pytest.mark.parametrize("name", ["d3q27_pf_velocity", "d3q27_pf_velocity_q27"])
def test_laplace_droplet(name):
    n, R = 24, 6.0
    lat = droplet(n, R, name=name)
    pf0 = lat.quantity("PhaseField").numpy().sum()
    lat.iterate(300)
    P = lat.quantity("P").numpy()[0]
    pf = lat.quantity("PhaseField").numpy()[0]
    c = n // 2
    dp = P[c, c, c] - P[1, 1, 1]
    assert abs(dp - 2 * SET["sigma"] / R) < 0.1 * 2 * SET["sigma"] / R, dp
    assert abs(pf.sum() / pf0 - 1) < 1e-11
    assert pf[c, c, c] > 0.99 and pf[1, 1, 1] < 0.01
    u = lat.quantity("U").numpy()
    assert np.abs(u).max() < 2e-3           # spurious currents stay small
    assert lat.globals["TotalDensity"] > 0


def test_wall_normals_and_contact():
    """channel walls at y=0 and y=n-1: wall normals point into the fluid (+y / -y),
    wall phase is set by the surface-energy condition each iteration."""
    n = 16
    lat = Lattice("d3q27_pf_velocity", (n, n, n), device=torch.device("cpu"), precision="double")
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, n), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, lat.gy + 0, :] = m.node_type("Wall").value
    fl[:, lat.gy + n - 1, :] = m.node_type("Wall").value
    lat.set_flags(fl)
    for k, v in SET.items():
        lat.set_setting(k, v)
    lat.set_setting("PhaseField", 1.0)
    lat.set_setting("radAngle", 1.2)
    lat.init()
    nrm = lat.quantity("Normal").numpy()        # (3, nz, ny, nx)
    assert np.allclose(nrm[:, :, 0, :], np.array([0, 1, 0])[:, None, None])
    assert np.allclose(nrm[:, :, n - 1, :], np.array([0, -1, 0])[:, None, None])
    assert np.allclose(nrm[:, :, 1:n - 1, :], 0)
    ib = lat.quantity("IsItBoundary").numpy()
    assert np.all(ib[:, :, 0, :] == 1) and np.all(ib[:, :, 1:n - 1, :] == 0)
    lat.iterate(20)
    assert torch.isfinite(lat.fields_interior()).all()
    assert lat.globals["NumBoundaryPoints"] == 2 * n * n
    assert lat.globals["NumFluidCells"] == n * n * (n - 2)   # wall flags carry no COLLISION bit
    # surface-energy wetting: wall phase from the neighbour (pf=1 liquid everywhere)
    # a = -h (4/W) cos(theta), h = 1/2 -> phi_w = (1 + a - sqrt((1+a)^2 - 4 a))/a - 1
    a = -0.5 * (4 / SET["IntWidth"]) * np.cos(1.2)
    phw = (1 + a - np.sqrt((1 + a) ** 2 - 4 * a * 1.0)) / (a + 1e-12) - 1.0
    pf = lat.quantity("PhaseField").numpy()[0]
    assert np.allclose(pf[:, 0, :], phw, atol=1e-3)
