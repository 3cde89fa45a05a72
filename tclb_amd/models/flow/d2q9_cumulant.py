"""d2q9_cumulant — D2Q9 cumulant collision (raw moments -> cumulants -> relaxation ->
back), separate viscosity in a boundary buffer layer, Zou/He velocity/pressure inlets.
Reference: models/flow/d2q9_cumulant/{Dynamics.R, Dynamics.c}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_cumulant", dims=2, family="flow", reference="models/flow/d2q9_cumulant",
              description="D2Q9 cumulant LBM")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    S = m.add_setting
    S("nu", default=0.16666666, comment="viscosity")
    S("nubuffer", default=0.01, comment="Viscosity in the buffer layer")
    S("Velocity", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Pressure", default=0, comment="inlet/outlet/init density", zonal=True)
    S("Density", default=1, comment="inlet/outlet/init density", zonal=True)
    S("ForceX")
    S("ForceY")
    for n in ["EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("flow/d2q9_cumulant.inc")
    return m
