"""d3q19_les — d'Humieres MRT D3Q19 with Smagorinsky LES (eddy viscosity from the
non-equilibrium stress).  Reference: models/flow/d3q19_les/Dynamics.R, Dynamics.c.Rt."""
from ..dsl import Model
from ...emit.symbolic import d3q19_mrt
from .d3q19 import mrt19_block


def build() -> Model:
    m = Model("d3q19_les", dims=3, family="flow", reference="models/flow/d3q19_les",
              description="D3Q19 MRT + Smagorinsky LES")
    U = d3q19_mrt().U
    for i in range(19):
        m.add_density(f"f[{i}]", int(U[i, 0]), int(U[i, 1]), int(U[i, 2]), group="f", comment=f"density F{i}")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_setting("nu", default=0.16666666, comment="viscosity")
    m.add_setting("Velocity", default="0m/s", comment="inlet velocity", zonal=True, unit="m/s")
    m.add_setting("Density", default=1, comment="inlet density", zonal=True)
    m.add_setting("Theta", default=1, comment="inlet density")
    m.add_setting("Turbulence", default=0, comment="amount of turbulence in init and on inlet", zonal=True)
    for a in "XYZ":
        m.add_setting(f"Force{a}", default="0N", comment=f"Force[{a.lower()}]")
    for g in ["Flux", "EnergyFlux", "PressureFlux", "PressureDiff", "MaterialPenalty"]:
        m.add_global(g, comment="pressure loss")
    m.add_setting("Smag", default=0, comment="Smagorynsky constant")
    for n in ["EPressure", "Solid", "Wall", "WPressure", "WPressureL", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_codegen(mrt19_block)
    m.set_dynamics("flow/d3q19_les.inc")
    return m
