"""d2q9_heat (experimental) — incompressible D2Q9 MRT flow (Lallemand-Luo moments) with a
D2Q9 advection-diffusion temperature set (MRT, diffusivity FluidAlfa), Zou/He velocity and
pressure inlets carrying an inlet temperature, and Dirichlet "Heater" nodes (T = 100).
Reference: models/heat/experimental/d2q9_heat/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_heat", dims=2, family="heat", reference="models/heat/experimental/d2q9_heat",
              description="D2Q9 incompressible MRT flow + D2Q9 MRT temperature")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("T", unit="K")
    m.add_quantity("U", unit="m/s", vector=True)
    for i, (x, y) in enumerate(U9):
        m.add_density(f"T[{i}]", x, y, 0, group="T")
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("InletVelocity", default="0m/s", comment="inlet velocity", unit="m/s")
    S("InletPressure", default="0Pa", comment="inlet pressure", unit="Pa", InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, comment="inlet density")
    S("InletTemperature", default=1, comment="inlet temperature")
    S("InitTemperature", default=1, comment="initial temperature")
    S("FluidAlfa", default=1, comment="thermal diffusivity")
    m.add_global("OutFlux")
    m.add_node_type("Heater", "ADDITIONALS")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.set_dynamics("heat/d2q9_heat.inc")
    return m
