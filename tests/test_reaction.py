"""d2q9_reaction_diffusion_system: source-term integrators against closed forms
(uniform fields, so the LBM part only carries the reaction), diffusion-mode decay for the
SRT_DF and TRT_M collisions, and the implicit-trapezoid phi reconstruction
(reference models/reaction/d2q9_reaction_diffusion_system/Dynamics.c.Rt)."""
import math

import numpy as np
import pytest
import torch

from tclb_amd.lattice import Lattice


def _lat(model, coll="SRT_DF", shape=(8, 4, 1), **settings):
    lat = Lattice(model, shape)
    m = lat.model
    lat.set_flags(np.full((lat.NZ, lat.NY, shape[0]), m.node_type(coll).value, dtype=np.uint32))
    for k, v in settings.items():
        lat.set_setting(k, v)
    lat.init()
    return lat


def _mean(lat, q):
    return float(lat.quantity(q).double().mean())


@pytest.mark.parametrize("integrator,factor", [
    ("Trapezoidal", lambda k: (2 + k) / (2 - k)),
    ("Euler", lambda k: 1 + k),
    ("Heun", lambda k: 1 + k + k * k / 2),
    ("Midpoint", lambda k: 1 + k + k * k / 2),
])
def test_linear_reaction_integrators(integrator, factor):
    k = -0.05
    lat = _lat(f"d2q9_reaction_diffusion_system_LinearReaction_{integrator}", Init_PHI=1.0,
               LinearReactionRate=k)
    assert abs(_mean(lat, "PHI") - 1.0) < 1e-12
    n = 40
    lat.iterate(n)
    assert abs(_mean(lat, "PHI") - factor(k) ** n) < 1e-10
    # second order: the trapezoid stays within O(k^3 n) of the exact exponential
    if integrator == "Trapezoidal":
        assert abs(_mean(lat, "PHI") - math.exp(k * n)) < 2e-4


def test_allen_cahn_implicit_reconstruction_and_ode():
    lam, phi0 = 0.1, 0.3
    lat = _lat("d2q9_reaction_diffusion_system_AllenCahn", Init_PHI=phi0, Lambda=lam)
    assert abs(_mean(lat, "PHI") - phi0) < 1e-12     # CalcPhi inverts phi - q(phi)/2 exactly
    n = 60
    lat.iterate(n)
    exact = 1.0 / math.sqrt(1.0 + (1.0 / phi0 ** 2 - 1.0) * math.exp(-2 * lam * n))
    assert abs(_mean(lat, "PHI") - exact) < 2e-3


@pytest.mark.parametrize("coll", ["SRT_DF", "TRT_M"])
def test_simple_diffusion_mode_decay(coll):
    nx, D, steps, a = 32, 0.05, 300, 0.05
    lat = _lat("d2q9_reaction_diffusion_system_SimpleDiffusion", coll, (nx, 4, 1), Init_PHI=1.0,
               Diffusivity_PHI=D)
    m = lat.model
    f = lat.fields_interior().clone()
    x = torch.arange(nx, dtype=f.dtype)
    prof = 1 + a * torch.sin(2 * math.pi * x / nx)
    sel = [i for i, fl in enumerate(m.fields) if fl.group == "dre_1"]
    f[sel] = f[sel] * prof[None, None, None, :]
    lat.set_fields_interior(f)
    lat.iterate(steps)
    p = lat.quantity("PHI")[0, 0].numpy()
    amp = (p.max() - p.min()) / 2
    kk = 2 * math.pi / nx
    expect = a * math.exp(-D * kk * kk * steps)
    assert abs(amp - expect) / expect < 0.02, (amp, expect)


def test_sir_simple_laplace_conserves_population():
    lat = _lat("d2q9_reaction_diffusion_system_SIR_SimpleLaplace", Init_S=0.95, Init_I=0.05, Init_R=0.0,
               Beta=0.3, Gamma=0.1)
    tot0 = sum(_mean(lat, q) for q in ("S", "I", "R"))
    i0 = _mean(lat, "I")
    lat.iterate(30)
    s, i, r = (_mean(lat, q) for q in ("S", "I", "R"))
    assert abs(s + i + r - tot0) < 1e-10
    # epidemic grows while beta S > gamma
    assert i > i0 and r > 0 and s < 0.95
    # compare with a fine explicit integration of the SIR ODE
    S, I, R = 0.95, 0.05, 0.0
    h = 0.001
    for _ in range(30000):
        dS, dI = -0.3 * S * I, 0.3 * S * I - 0.1 * I
        S, I, R = S + h * dS, I + h * dI, R + h * 0.1 * I
    assert abs(i - I) < 2e-3 and abs(s - S) < 2e-3


def test_sir_modified_peng_newton():
    lat = _lat("d2q9_reaction_diffusion_system_SIR_ModifiedPeng", Init_W=0.0, Init_S=0.9, Init_I=0.1,
               Init_R=0.0, Init_N=1.0, Beta=0.4, Beta_w=0.2, Gamma=0.1)
    for q, v in (("S", 0.9), ("I", 0.1), ("R", 0.0), ("N", 1.0)):
        assert abs(_mean(lat, q) - v) < 1e-4, q
    lat.iterate(20)
    s, i, r, w = (_mean(lat, q) for q in ("S", "I", "R", "W"))
    assert abs(s + i + r - 1.0) < 1e-3
    assert w > 0 and s < 0.9 and r > 0
