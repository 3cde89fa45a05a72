"""d2q9_optimalMixing — D2Q9 BGK flow driven by a moving lid plus a D2Q5 passive scalar
(temperature) for mixing optimisation: objective pieces TotalTempSqr/CountCells, wall
force and power on the moving lid.  Adjoint quantities RhoB/TB from the reverse sweep
(Model.set_reverse: rev_run in the .inc, with the emitted equilibria's VJPs).
Reference: models/optimization/d2q9_optimalMixing/{Dynamics.R, Dynamics.c.Rt}."""
import numpy as np

from ..dsl import Model
from ...emit.blocks import feq_block, vjp_function
from ...emit.symbolic import mrt_eq

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]
U5 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1]]


def _blocks(_m):
    out = [feq_block("feq9", U9), feq_block("feq5", U5)]
    for name, U in (("feq9", U9), ("feq5", U5)):     # (d feq / d (rho, J))^T a
        eq = mrt_eq(np.asarray(U, dtype=int), orthogonal=False, order=2)
        out.append(vjp_function(f"{name}_T", ["rho"] + [str(j) for j in eq.J], eq.feq))
    return "\n".join(out)


def build() -> Model:
    m = Model("d2q9_optimalMixing", dims=2, family="optimization",
              reference="models/optimization/d2q9_optimalMixing",
              description="D2Q9 lid-driven flow + D2Q5 passive scalar (optimal mixing)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("T", unit="K")
    m.add_quantity("U", unit="m/s", vector=True)
    for i, (x, y) in enumerate(U5):
        m.add_density(f"g[{i}]", x, y, 0, group="g")
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("omegaT", comment="one over relaxation time - thermal")
    S("K", default=0.16666666, comment="thermal_diffusivity", omegaT="1.0/(3*K + 0.5)")
    S("MovingWallVelocity", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Velocity", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default="0Pa", comment="Inlet pressure", zonal=True, unit="Pa")
    S("Temperature", default="0K", comment="Temperature", zonal=True, unit="K")
    m.add_node_type("NMovingWall", "BOUNDARY")
    m.add_node_type("SWall", "BOUNDARY")
    for g in ("TotalTempSqr", "CountCells", "NMovingWallForce", "SWallForce", "MovingWallPower"):
        m.add_global(g)
    m.add_quantity("RhoB", adjoint=True, adjoint_of="f")
    m.add_quantity("TB", adjoint=True, adjoint_of="g")
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_codegen(_blocks)
    m.set_dynamics("optimization/d2q9_optimalmixing.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
