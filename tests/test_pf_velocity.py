"""d2q9_pf_velocity: a static drop at density ratio 10 conserves the phase field, stays
centred with small spurious currents and satisfies Laplace's law dp = sigma / R for the
MRT, central-moment and BGK collisions; a drop on a wall with a contact angle spreads
(geometric wetting through the wall normals) (reference models/multiphase/d2q9_pf_velocity)."""
import numpy as np
import pytest
import torch

from conftest import DEVICES
from tclb_amd.lattice import Lattice


def _drop(model, coll, n=40, R0=9.0, sigma=0.01, steps=1000, flags=None, device="cpu", **extra):
    lat = Lattice(model, (n, n, 1), device=torch.device(device))
    m = lat.model
    fl = np.full((lat.NZ, lat.NY, n), m.node_type(coll).value, dtype=np.uint32) if flags is None else flags(m, lat)
    lat.set_flags(fl)
    s = dict(Density_h=1.0, Density_l=0.1, sigma=sigma, W=4, M=0.02, Viscosity_l=0.1, Viscosity_h=0.1,
             Radius=R0, CenterX=n / 2, CenterY=n / 2, BubbleType=1, PhaseField_init=0.0, bulk_visc=1 / 6)
    s.update(extra)
    for k, v in s.items():
        lat.set_setting(k, v)
    lat.init()
    phi0 = float(lat.quantity("PhaseField").double().sum())
    lat.iterate(steps)
    return lat, phi0


@pytest.mark.parametrize("model,coll", [("d2q9_pf_velocity", "MRT"), ("d2q9_pf_velocity_CM", "CM"),
                                        ("d2q9_pf_velocity_BGK", "BGK")])
@pytest.mark.parametrize("device", DEVICES)
def test_pf_velocity_static_drop(model, coll, device):
    n, R0, sigma = 40, 9.0, 0.01
    lat, phi0 = _drop(model, coll, n, R0, sigma, device=device)
    phi = lat.quantity("PhaseField")[0, 0].double().cpu().numpy()
    p = lat.quantity("Pressure")[0, 0].double().cpu().numpy()
    u = lat.quantity("U")[:2].double().cpu().numpy()
    assert np.isfinite(p).all()
    assert abs(phi.sum() - phi0) < 1e-8 * phi0
    c = n // 2
    assert phi[c, c] > 0.95 and phi[0, 0] < 0.05
    dp = p[c - 3:c + 3, c - 3:c + 3].mean() - p[:4, :4].mean()
    assert abs(dp - sigma / R0) / (sigma / R0) < 0.15, (dp, sigma / R0)
    assert np.abs(u).max() < 1e-3


def test_pf_velocity_wetting_spreads():
    """the wetted length on the wall shrinks as the contact angle grows (45, 90, 135 deg)"""
    n = 48

    def flags(m, lat):
        fl = np.full((lat.NZ, lat.NY, n), m.node_type("MRT").value, dtype=np.uint32)
        fl[:, lat.gy:lat.gy + 2, :] = m.node_type("Wall").value
        return fl

    def footprint(angle):
        lat, _ = _drop("d2q9_pf_velocity", "MRT", n, 9.0, 0.01, 1200, flags=flags, CenterY=10.0,
                       radAngle=angle)
        phi = lat.quantity("PhaseField")[0, 0].double().numpy()
        return (phi[2] > 0.5).sum()
    assert footprint(np.pi / 4) > footprint(np.pi / 2) + 4 > footprint(3 * np.pi / 4) + 8
