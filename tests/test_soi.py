"""d2q9_AllenCahn_SourceTerm_SOI: exact discrete decay of the ExpotentialDecay variant,
the Allen-Cahn ODE through the implicit reconstruction, and advection-diffusion of a
Gaussian profile (mean moves with u, variance grows 2 D t) for every collision kernel
(reference models/reaction/d2q9_AllenCahn_SourceTerm_SOI)."""
import math

import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice

CV = (0, 1, -1)


def _lat(model, coll, shape, **settings):
    lat = Lattice(model, shape)
    m = lat.model
    lat.set_flags(np.full((lat.NZ, lat.NY, shape[0]), m.node_type(coll).value, dtype=np.uint32))
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


def test_soi_exponential_decay():
    lam, n = 0.05, 40
    lat = _lat("d2q9_AllenCahn_SourceTerm_SOI_ExpotentialDecay", "SRT_M_SOI", (8, 4, 1), Init_PhaseField=1.0,
               **{"lambda": lam})
    p0 = float(lat.quantity("PhaseField").double().mean())
    lat.iterate(n)
    p = float(lat.quantity("PhaseField").double().mean())
    assert abs(p / p0 - ((2 - lam) / (2 + lam)) ** n) < 1e-12


@pytest.mark.parametrize("coll", ["SRT_DF_SOI", "TRT_M_SOI", "TRT_CM_SOI"])
def test_soi_allen_cahn_ode(coll):
    lam, phi0, n = 0.1, 0.3, 60
    lat = _lat("d2q9_AllenCahn_SourceTerm_SOI", coll, (8, 4, 1), Init_PhaseField=phi0, **{"lambda": lam})
    assert abs(float(lat.quantity("PhaseField").double().mean()) - phi0) < 1e-12
    lat.iterate(n)
    exact = 1.0 / math.sqrt(1.0 + (1.0 / phi0 ** 2 - 1.0) * math.exp(-2 * lam * n))
    assert abs(float(lat.quantity("PhaseField").double().mean()) - exact) < 2e-3


@pytest.mark.parametrize("coll", ["SRT_DF_SOI", "TRT_M_SOI", "TRT_CM_SOI"])
def test_soi_advection_diffusion(coll):
    nx, D, ux, s0, steps = 128, 0.02, 0.05, 6.0, 400
    lat = _lat("d2q9_AllenCahn_SourceTerm_SOI", coll, (nx, 4, 1), Init_PhaseField=0.0, Init_UX=ux,
               diffusivity_phi=D, **{"lambda": 0.0})
    m = lat.model
    f = lat.fields_interior().clone()
    x = torch.arange(nx, dtype=f.dtype)
    x0 = 40.0
    prof = torch.exp(-(x - x0) ** 2 / (2 * s0 * s0))
    s2 = 1.0 / 3.0
    names = [fl.name for fl in m.fields]
    for k in range(9):
        cx, cy = CV[k % 3], CV[k // 3]
        gx = {0: 1 - (s2 + ux * ux), 1: (s2 + ux * ux + ux) / 2, -1: (s2 + ux * ux - ux) / 2}[cx]
        gy = {0: 1 - s2, 1: s2 / 2, -1: s2 / 2}[cy]
        f[names.index(f"f[{k}]"), 0] = (prof * gx * gy)[None, :]
    lat.set_fields_interior(f)
    xs = np.arange(nx)

    def moments():
        p = lat.quantity("PhaseField")[0, 0, 0].double().numpy()
        mean = (p * xs).sum() / p.sum()
        return mean, (p * (xs - mean) ** 2).sum() / p.sum()
    mean0, var0 = moments()      # quantities are read from the streamed populations
    lat.iterate(steps)
    mean, var = moments()
    assert abs(mean - mean0 - ux * steps) < 1e-3
    assert abs(var - var0 - 2 * D * steps) / (2 * D * steps) < 0.03, (var - var0, 2 * D * steps)
