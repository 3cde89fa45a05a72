"""d2q9_inc — incompressible (He-Luo) D2Q9 MRT: equilibria linear in the density
fluctuation, Lallemand-Luo moments with user relaxation rates (S3, S4, S56, S78 = 1-omega),
body force as a momentum shift, symmetry planes, pressure inlet/outlet (the velocity
closures are disabled in the reference and are no-ops here too).
Reference: models/experimental/d2q9_inc/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_inc", dims=2, family="experimental", reference="models/experimental/d2q9_inc",
              description="Incompressible D2Q9 MRT (He-Luo equilibrium)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    S = m.add_setting
    S("omega", comment="one over relaxation time", S78="1-omega")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("Velocity", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("Density", default=1, comment="inlet/outlet/init density", zonal=True)
    S("GravitationY", comment="Gravitation in the direction of y")
    S("GravitationX", comment="Gravitation in the direction of x")
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="outlet flux", unit="1m2/s")
    m.add_global("InletFlux", comment="inlet flux", unit="1m2/s")
    S("S3", default="-0.333333333", comment="MRT Sx")
    S("S4", default="0", comment="MRT Sx")
    S("S56", default="0", comment="MRT Sx")
    S("S78", default="0", comment="MRT Sx")
    for n in ("BottomSymmetry", "TopSymmetry"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("experimental/d2q9_inc.inc")
    return m
