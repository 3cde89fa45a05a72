"""d2q9_heat_adj (experimental) — incompressible D2Q9 MRT flow through a solid/fluid
design field w (momentum damped by w, conductivity blended FluidAlpha/SolidAlpha) with a
D2Q9 MRT temperature: the 2-D heat-exchanger topology-optimisation model.
Reference: models/optimization/experimental/d2q9_heat_adj/{Dynamics.R, Dynamics.c.Rt}
(ADJOINT=1; gradients here from the generic AD adjoint).  The reference's derived setting
``nu0 -> omega`` refers to an undefined ``nu``; here it is 1/(3 nu0 + 1/2)."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_heat_adj", dims=2, family="optimization",
              reference="models/optimization/experimental/d2q9_heat_adj",
              description="D2Q9 incompressible MRT + MRT temperature with a solid/fluid design field")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"T[{i}]", x, y, 0, group="T")
    m.add_density("w", 0, 0, 0, group="w", parameter=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("T", unit="K")
    m.add_quantity("W")
    m.add_quantity("WB", adjoint=True)
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu0", default=0.16666666, comment="viscosity", omega="1.0/(3*nu0 + 0.5)")
    S("InletVelocity", default="0m/s", comment="inlet velocity", unit="m/s")
    S("InletPressure", default="0Pa", comment="inlet pressure", unit="Pa", InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, comment="inlet density")
    S("InletTemperature", default=1, comment="inlet temperature")
    S("InitTemperature", default=1, comment="initial temperature")
    S("HeaterTemperature", default=1, comment="heater temperature")
    S("FluidAlpha", default=1, comment="thermal diffusivity of fluid")
    S("SolidAlpha", default=1, comment="thermal diffusivity of solid")
    S("LimitTemperature", comment="temperature limit")
    S("InletTotalPressure", comment="inlet total pressure")
    S("OutletTotalPressure", comment="outlet total pressure")
    for g, c in (("HeatFlux", "heat flux"), ("HeatSquareFlux", "flux of T^2"), ("Flux", "volume flux"),
                 ("Temperature", "integral of temperature"), ("HighTemperature", "penalty for high temperature"),
                 ("LowTemperature", "penalty for low temperature")):
        m.add_global(g, comment=c)
    m.add_node_type("Heater", "ADDITIONALS")
    m.add_node_type("HeatSource", "ADDITIONALS")
    m.add_node_type("Thermometer", "OBJECTIVE")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.set_dynamics("optimization/d2q9_heat_adj.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
