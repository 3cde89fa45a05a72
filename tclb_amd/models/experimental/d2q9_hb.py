"""d2q9_hb — incompressible D2Q9 MRT flow with an MRT advection-diffusion scalar (the
"temperature" T, used as a cell-viability/concentration field) that is destroyed at
``Destroy`` nodes at a rate DestructionRate * SS^DestructionPower, SS being a von-Mises
type norm of the viscous stress; stress diagnostics Q, Qxx, Qxy, Qyy, SS are exported.
Reference: models/experimental/d2q9_hb/{Dynamics.R, Dynamics.c}.
"""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_hb", dims=2, family="experimental", reference="models/experimental/d2q9_hb",
              description="D2Q9 MRT flow + MRT scalar with stress-driven destruction")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    for q, u in (("Rho", "kg/m3"), ("T", "K"), ("Q", "1"), ("Qxx", "1"), ("Qxy", "1"), ("Qyy", "1"),
                 ("SS", "N/m2")):
        m.add_quantity(q, unit=u)
    m.add_quantity("U", unit="m/s", vector=True)
    for i, (x, y) in enumerate(U9):
        m.add_density(f"T[{i}]", x, y, 0, group="T")
    m.add_node_type("Destroy", "ADDITIONALS")
    m.add_node_type("Outlet2", "ADDITIONALS")
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("DestructionRate")
    S("DestructionPower")
    S("nu", default=0.16666666, unit="m2/s", comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("InletVelocity", default=0, unit="m/s", comment="inlet velocity")
    S("InletPressure", default=0, unit="Pa", comment="inlet pressure", InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, unit="kg/m3", comment="inlet density")
    S("InletTemperature", default=1, comment="inlet density")
    S("InitTemperature", default=1, comment="inlet density")
    S("FluidAlfa", default=1, comment="inlet density")
    m.add_global("OutFlux")
    m.add_global("DestroyedCellFlux")
    m.add_node_type("Heater", "ADDITIONALS")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("Outlet", "OBJECTIVE")
    m.set_dynamics("experimental/d2q9_hb.inc")
    return m
