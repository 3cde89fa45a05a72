"""d2q9 — weighted-orthogonal MRT with Zou/He (rewrite form) velocity/pressure
boundaries, symmetry and bounce-back; objective globals on Inlet/Outlet nodes.
Reference: models/flow/d2q9/Dynamics.R, Dynamics.c.Rt (OPT="bc*autosym": variants
d2q9, d2q9_bc, d2q9_autosym, d2q9_bc_autosym)."""
import numpy as np
import sympy as sp

from ..dsl import Model
from ...emit.symbolic import mrt_eq, poly_matrix, weights_from_eq
from ...emit.blocks import mrt_block

U9 = np.array([[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]])


def d2q9_mrt_basis():
    """B = M H^T with H from the Cholesky factor of M^-1 diag(1/w) M^-T (reversed order),
    rows scaled by (1, sqrt3/3, sqrt3/3, sqrt2, sqrt2, 1, sqrt6/3, sqrt6/3, 2)
    (reference models/flow/d2q9/Dynamics.c.Rt:8-24)."""
    raw = mrt_eq(U9, orthogonal=False)
    M = raw.mat
    w = weights_from_eq(raw)
    Minv = M.inv()
    W = Minv * sp.diag(*[1 / x for x in w]) * Minv.T
    n = W.shape[0]
    rev = list(range(n))[::-1]
    Wr = W.extract(rev, rev)
    L = Wr.cholesky(hermitian=False)   # Wr = L L^T
    Ur = L.T                           # R's chol(): upper factor
    H = Ur.extract(rev, rev)
    scale = [1, sp.sqrt(3) / 3, sp.sqrt(3) / 3, sp.sqrt(2), sp.sqrt(2), 1, sp.sqrt(6) / 3, sp.sqrt(6) / 3, 2]
    H = sp.Matrix(n, n, lambda r, c: sp.nsimplify(sp.simplify(H[r, c] * scale[r])))
    B = (M * H.T).applyfunc(sp.simplify)
    return B


def build(bc: bool = False, autosym: int = 0, par: bool = False, part: bool = False) -> Model:
    """par: d2q9_par (reference models/flow/d2q9_par) — the node momentum is stored in
    parameter densities ux, uy by a CalcU stage and overwritten with the rigid-body
    velocity of covering particles in a particle stage CalcF (velocity imposition, no
    force feedback).  part: d2q9_part (models/flow/d2q9_part) — single particle stage;
    the velocity mismatch to covering particles is removed from the fluid and applied to
    the particles as force."""
    name = "d2q9_part" if part else ("d2q9_par" if par else "d2q9")
    m = Model(name, dims=2, family="flow", reference=f"models/flow/{name}",
              description="D2Q9 MRT (weighted orthogonal basis) with Zou/He and symmetry boundaries"
              + (", particle velocity coupling" if par or part else ""))
    shifts = [4 / 9] + [1 / 9] * 4 + [1 / 36] * 4
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", int(x), int(y), 0, group="f", shift=shifts[i])
    if bc:
        m.add_density("BC[0]", group="BC", parameter=True)
        m.add_density("BC[1]", group="BC", parameter=True)
    if par or part:
        for n in ("ux", "uy", "sol"):
            m.add_density(n, group="u", parameter=True)
    if part:
        for n in ("thx", "thy", "thz"):
            m.add_density(n, group="th")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    if par or part:
        m.add_quantity("Solid", unit="1")
    if part:
        m.add_quantity("Checks", unit="1")
        m.add_quantity("Thread", unit="1", vector=True)
    if par:
        m.add_stage("BaseIteration", "Run", save_fields=["f"], load_densities=["f", "u"])
        m.add_stage("CalcU", "CalcU", save_fields=["ux", "uy", "sol"], load_densities=["f"])
        m.add_stage("CalcF", "CalcF", save_fields=["ux", "uy", "sol"], load_densities=["u"], particle=True)
        m.add_stage("BaseInit", "Init", save_fields=True, init=True)
        m.add_action("Iteration", ["BaseIteration", "CalcU", "CalcF"])
        m.add_action("Init", ["BaseInit", "CalcU", "CalcF"])
    if part:
        m.add_stage("BaseIteration", "Run", load_densities=True, save_fields=True, particle=True)
    m.add_setting("RelaxationRate", comment="one over relaxation time", S2="1-RelaxationRate")
    m.add_setting("Viscosity", default=0.16666666, comment="viscosity", RelaxationRate="1.0/(3*Viscosity + 0.5)")
    m.add_setting("VelocityX", default=0, comment="inlet/outlet/init velocity", zonal=True, unit="m/s")
    m.add_setting("VelocityY", default=0, comment="inlet/outlet/init velocity", zonal=True, unit="m/s")
    m.add_setting("Pressure", default=0, comment="inlet/outlet/init density", zonal=True, unit="Pa")
    m.add_setting("GravitationX")
    m.add_setting("GravitationY")
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="pressure loss", unit="1m2/s")
    m.add_global("InletFlux", comment="pressure loss", unit="1m2/s")
    m.add_setting("S2", default=0, comment="MRT Sx")
    m.add_setting("S3", default=0, comment="MRT Sx")
    m.add_setting("S4", default=0, comment="MRT Sx")
    for n in ["EPressure", "WPressure", "NVelocity", "SVelocity", "WVelocity", "EVelocity", "NSymmetry", "SSymmetry"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"bc": bc, "autosym": autosym, "par": par, "part": part}
    B = d2q9_mrt_basis()
    eq = mrt_eq(U9, mat=B)
    m.add_codegen(lambda _m: mrt_block("mrt", eq))
    m.set_dynamics("flow/d2q9.inc")
    return m
