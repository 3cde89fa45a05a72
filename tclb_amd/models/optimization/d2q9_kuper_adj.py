"""d2q9_kuper_adj — experimental adjoint-capable Kupershtokh pseudopotential model on D2Q9
with a porosity-like design parameter w (velocity damping u <- w u in the MRT collision).
The interaction potential is carried by nine *streamed* densities phi_i (each node writes
its own potential into all of them, so after streaming phi_i holds the neighbour's value
at x - c_i) instead of a stencil field, and the streamed / resting copies f and fs are
swapped at the start of every iteration as in the reference (two interleaved time
sub-sequences).
Reference: models/optimization/experimental/d2q9_kuper_adj/{Dynamics.R, Dynamics.c.Rt,
Dynamics_adj.c.Rt} (ADJOINT=1).
"""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_kuper_adj", dims=2, family="optimization",
              reference="models/optimization/experimental/d2q9_kuper_adj",
              description="D2Q9 Kupershtokh multiphase with design parameter w (adjoint)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f", comment=f"streamed density F{i}")
    for i in range(9):
        m.add_density(f"fs[{i}]", 0, 0, 0, group="fs", comment=f"density F{i}")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"phi[{i}]", x, y, 0, group="phi", comment=f"streamed potential {i}")
    m.add_density("w", 0, 0, 0, group="w", parameter=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("RhoB", adjoint=True, adjoint_of="f")
    m.add_quantity("UB", adjoint=True, vector=True)
    m.add_quantity("WB", adjoint=True, adjoint_of="w")
    m.add_quantity("W")
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("InletVelocity", default=0, comment="inlet velocity", unit="m/s")
    S("InletPressure", default=0, comment="inlet pressure", unit="Pa", InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, comment="inlet density")
    S("OutletDensity", default=1, comment="inlet density")
    S("InitDensity", comment="inlet density")
    S("WallDensity", comment="vapor/liquid density of wall")
    S("Temperature", comment="temperature of the liquid/gas")
    S("FAcc", comment="Multiplier of potential")
    S("Magic", comment="K")
    S("MagicA", comment="A in force calculation")
    S("MagicF", comment="Force multiplier")
    S("GravitationY", comment="Gravitation in the direction of y")
    S("GravitationX", comment="Gravitation in the direction of x")
    S("MovingWallVelocity", comment="Velocity of the MovingWall")
    S("WetDensity", comment="wet density")
    S("DryDensity", comment="dry density")
    S("Wetting", comment="wetting factor")
    for g, c in (("MovingWallForceX", "force x"), ("MovingWallForceY", "force y"),
                 ("Pressure1", "pressure at Obj1"), ("Pressure2", "pressure at Obj2"), ("Pressure3", "pressure at Obj3"),
                 ("Density1", "density at Obj1"), ("Density2", "density at Obj2"), ("Density3", "density at Obj3"),
                 ("FluidVelocityX", "velocity x")):
        m.add_global(g, comment=c)
    for n in ("EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("Dry", "ADDITIONALS")
    m.add_node_type("MovingWall", "BOUNDARY")
    for n in ("Obj1", "Obj2", "Obj3"):
        m.add_node_type(n, "OBJECTIVE")
    m.add_node_type("Wet", "ADDITIONALS")
    m.set_dynamics("optimization/d2q9_kuper_adj.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
