"""d2q9_npe_guo (Nernst-Planck-Poisson LB, reference models/electrokinetic/d2q9_npe_guo).

The reference ships no goldens (its test_eof.py needs an external run), so these are
invariants of the scheme ("parity unpinned"):
* without ions the Poisson LB relaxes to the Dirichlet wall potential everywhere;
* with ions and charged walls the steady state is a Boltzmann double layer:
  n0 n1 = n_inf^2 at every node, counter-ions enriched at the wall, the potential
  screened over the Debye length kappa^-1."""
import numpy as np
import torch

from tclb_amd.lattice import Lattice


def channel(ny=41, **settings):
    lat = Lattice("d2q9_npe_guo", (4, ny, 1), device=torch.device("cpu"), precision="double")
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, 4), m.node_type("MRT").value, dtype=np.uint32)
    fl[:, lat.gy + 0, :] = m.node_type("Wall").value
    fl[:, lat.gy + ny - 1, :] = m.node_type("Wall").value
    lat.set_flags(fl)
    base = {"el": 1.0, "el_kbT": 1.0, "psi0": 0.0, "phi0": 0.0, "nu": 0.1, "D": 0.1, "phi_bc": 0.0}
    base.update(settings)
    for k, v in base.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


def test_poisson_without_ions():
    zeta = 0.02
    lat = channel(n_inf_0=0.0, n_inf_1=0.0, epsilon=1.0, psi_bc=zeta)
    lat.iterate(9000)
    psi = lat.quantity("Psi").numpy()[0, 0, 1:-1, 1]
    assert np.allclose(psi, zeta, rtol=1e-6)
    assert np.abs(lat.quantity("U").numpy()).max() < 1e-12


def test_boltzmann_double_layer():
    zeta, n_inf, kappa = 0.01, 1.0, 0.2
    eps = 2 * n_inf / kappa ** 2
    lat = channel(n_inf_0=n_inf, n_inf_1=n_inf, epsilon=eps, psi_bc=zeta)
    lat.iterate(6000)
    n0 = lat.quantity("n0").numpy()[0, 0, :, 1]
    n1 = lat.quantity("n1").numpy()[0, 0, :, 1]
    psi = lat.quantity("Psi").numpy()[0, 0, :, 1]
    assert np.allclose(n0 * n1, n_inf ** 2, atol=1e-4)
    assert n1[1] > n1[10] > n_inf * 0.999 and n0[1] < n0[10]        # counter-ions at the wall
    assert psi[1] > psi[3] > psi[6] > 0                               # screened potential
    assert abs(psi[20]) < 0.15 * zeta
    assert np.isfinite(lat.quantity("U").numpy()).all()


def test_poisson_boltzmann_debye_huckel():
    """d2q9_poison_boltzmann (reference models/electrokinetic/d2q9_poison_boltzmann): for a
    small wall potential the steady Poisson-Boltzmann solution between two walls is the
    Debye-Hueckel profile psi = zeta cosh(kappa (y - yc)) / cosh(kappa h),
    kappa^2 = 2 n_inf z^2 e^2 / (eps kT)."""
    ny, zeta, kappa = 41, 1e-3, 0.15
    lat = Lattice("d2q9_poison_boltzmann", (4, ny, 1), device=torch.device("cpu"), precision="double")
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, 4), m.node_type("Collision").value, dtype=np.uint32)
    fl[:, lat.gy + 0, :] = m.node_type("Wall").value
    fl[:, lat.gy + ny - 1, :] = m.node_type("Wall").value
    lat.set_flags(fl)
    for k, v in {"tau_psi": 1.0, "dt": 1.0, "epsilon": 1.0, "n_inf": kappa ** 2 / 2, "z": 1.0, "el": 1.0,
                 "kb": 1.0, "T": 1.0, "psi_bc": zeta, "psi0": 0.0}.items():
        lat.set_setting(k, v)
    lat.init()
    lat.iterate(1500)
    psi = lat.quantity("Psi").numpy()[0, 0, :, 1]
    y = np.arange(ny)
    exact = zeta * np.cosh(kappa * (y - (ny - 1) / 2)) / np.cosh(kappa * (ny - 1) / 2)
    assert np.abs(psi - exact)[1:-1].max() < 0.01 * zeta, np.abs(psi - exact)[1:-1].max() / zeta
    assert lat.quantity("Subiter").numpy().max() > 0
