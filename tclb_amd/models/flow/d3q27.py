"""d3q27 — raw-moment MRT (BGK-equivalent by default) with Smagorinsky LES and an
entropic stabiliser.  Reference: models/flow/d3q27/Dynamics.R, Dynamics.c.Rt."""
import numpy as np

from ..dsl import Model
from ...emit.symbolic import mrt_eq
from ...emit.blocks import mrt_block

# expand.grid(-1:1,-1:1,-1:1) order: x fastest (reference Dynamics.R:1)
U27 = np.array([[x, y, z] for z in (-1, 0, 1) for y in (-1, 0, 1) for x in (-1, 0, 1)])


def build() -> Model:
    m = Model("d3q27", dims=3, family="flow", reference="models/flow/d3q27",
              description="D3Q27 raw-moment MRT with optional Smagorinsky LES and entropic stabilisation")
    for i, (x, y, z) in enumerate(U27):
        m.add_density(f"f[{i}]", int(x), int(y), int(z), group="f", comment=f"density F{i}")
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Fd", unit="N", vector=True)
    m.add_setting("omega", comment="One over relaxation time")
    m.add_setting("nu", default=0.16666666, comment="Viscosity", omega="1.0/(3*nu + 0.5)")
    m.add_setting("Velocity", default="0m/s", comment="Inlet velocity", zonal=True, unit="m/s")
    m.add_setting("Pressure", default="0Pa", comment="Inlet pressure", zonal=True, unit="Pa")
    m.add_setting("Smag", comment="Smagorinsky constant")
    m.add_setting("Turbulence", comment="Turbulence intensity", zonal=True)
    for a in "XYZ":
        m.add_setting(f"Force{a}", comment=f"Force {a}")
    for a in "XYZ":
        m.add_global(f"{a}Flux", comment="Volume flux", unit="m3/s")
    for a in "XYZ":
        m.add_global(f"{a}DragForce", comment="Solid drag force", unit="N")
    m.add_node_type("Smagorinsky", "LES")
    m.add_node_type("Stab", "ENTROPIC")
    for n in ["NSymmetry", "SSymmetry", "ISymmetry", "EPressure", "Solid", "Wall", "WPressure", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    eq = mrt_eq(U27, orthogonal=False)
    m.add_codegen(lambda _m: mrt_block("mrt", eq, tensor=True))
    m.set_dynamics("flow/d3q27.inc")
    return m
