"""d2q9_les — D2Q9 MRT (Lallemand-Luo moments) with a Smagorinsky LES relaxation time
computed from the non-equilibrium moments, a porosity parameter density w that scales
the equilibrium velocity, Zou/He inlets/outlets and pressure-loss objectives.
Reference: models/flow/d2q9_les/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_les", dims=2, family="flow", reference="models/flow/d2q9_les",
              description="D2Q9 MRT + Smagorinsky LES with a porosity parameter")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_density("w", 0, 0, 0, group="w", parameter=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("W")
    S = m.add_setting
    S("tau0", comment="one over relaxation time")
    S("nu", tau0="3*nu + 0.5", default=0.16666666, comment="viscosity")
    S("Velocity", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Density", default=1, comment="inlet/outlet/init density", zonal=True)
    S("Smag", default=1, comment="Smagorinsky constant")
    for g in ["PressDiff", "TotalPressureFlux", "OutletFlux", "InletPressureIntegral"]:
        m.add_global(g, comment="pressure loss")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    for n in ["EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("flow/d2q9_les.inc")
    return m
