"""auto model options (reference models/flow/auto, OPT="d3q19*part*(TRT+BGK+WMRT)*FMT*HiOrd*autosym"):
FMT is a different transform algorithm with the same moments, HiOrd keeps the
untruncated equilibrium, WMRT decorrelates the equilibrium moments."""
import numpy as np
import sympy as sp
import torch

from tclb_amd.emit.symbolic import mrt_eq
from tclb_amd.lattice import Lattice
from tclb_amd.models.flow.auto import lattice, wmrt_matrix


def _run(model, steps=30):
    lat = Lattice(model, (8, 6, 4))
    m = lat.model
    lat.set_flags(np.full((lat.NZ, lat.NY, 8), m.node_type("MRT").value, dtype=np.uint16))
    lat.set_setting("Viscosity", 0.05)
    lat.init()
    rng = np.random.default_rng(3)
    st = lat.fields_interior().clone()
    nf = 27 if "d3q19" not in model else 19
    st[:nf] = st[:nf] * torch.as_tensor(1 + 0.05 * rng.standard_normal(st[:nf].shape))
    lat.set_fields_interior(st)
    lat.iterate(steps)
    return lat.fields_interior()[:nf].numpy().copy()


def test_fmt_equals_dense_transform():
    np.testing.assert_allclose(_run("auto_FMT"), _run("auto"), rtol=0, atol=1e-13)
    np.testing.assert_allclose(_run("auto_FMT_HiOrd"), _run("auto_HiOrd"), rtol=0, atol=1e-13)


def test_hiord_differs_from_truncated_at_finite_velocity():
    a, b = _run("auto_HiOrd"), _run("auto")
    assert np.abs(a - b).max() > 1e-9
    np.testing.assert_allclose(a.sum(), b.sum(), rtol=1e-12)   # both conserve total mass


def test_wmrt_equilibrium_moments_are_orthogonal_polynomials():
    for q19 in (False, True):
        P, U = lattice(q19)
        raw12 = mrt_eq(U, orthogonal=False, order=12)
        M = wmrt_matrix(raw12)
        eq = mrt_eq(U, mat=M, order=12)
        cd = [sp.expand(e).as_coefficients_dict() for e in eq.Req]
        monos = sorted({k for d in cd for k in d}, key=str)
        A = sp.Matrix(len(monos), len(cd), lambda r, c: cd[c].get(monos[r], 0))
        G = A.T * A
        assert G == sp.diag(*[G[i, i] for i in range(G.shape[0])])
        # conserved moments (density, momentum) keep their meaning
        assert sp.simplify(eq.Req[0] - sp.Symbol("rho")) == 0
