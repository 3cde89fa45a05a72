"""sw — lattice Boltzmann shallow-water equations on D2Q9 (Lallemand-Luo MRT, the
gravity term g h^2 in the energy equilibria), a damping parameter field w on the
momentum (obstacles / energy sinks), adjoint-ready.
Reference: models/shallowwater/sw/{Dynamics.R, Dynamics.c.Rt} (ADJOINT=1)."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("sw", dims=2, family="shallowwater", reference="models/shallowwater/sw",
              description="Shallow water equations (D2Q9 MRT) with a momentum-damping parameter field")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_density("w", 0, 0, 0, group="w", parameter=True)
    m.add_quantity("Rho", unit="m")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("RhoB", adjoint=True, adjoint_of="f")
    m.add_quantity("UB", adjoint=True, vector=True)
    m.add_quantity("W")
    m.add_quantity("WB", adjoint=True)
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("InletVelocity", default="0m/s", comment="inlet velocity", unit="m/s")
    S("InletPressure", default="0Pa", comment="inlet pressure", unit="Pa", InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, comment="inlet density")
    S("Gravity", default=1, comment="gravity")
    S("SolidH", default=1, comment="height of solid")
    S("EnergySink", default=0, comment="energy sink on Obj1 nodes")
    S("Height", default=0, zonal=True, comment="water height")
    m.add_global("PressDiff", comment="pressure loss")
    m.add_global("TotalDiff", comment="total variation of velocity")
    m.add_global("Material", comment="total material")
    m.add_global("EnergyGain", comment="energy gain")
    m.add_node_type("Obj1", "OBJECTIVE")
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("shallowwater/sw.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
