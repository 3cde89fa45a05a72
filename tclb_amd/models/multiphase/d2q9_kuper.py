"""d2q9_kuper — pseudopotential (Kupershtokh-type) liquid-vapour model with a
Carnahan-Starling-like equation of state; two-stage Iteration (BaseIteration +
CalcPhi), MRT collision with velocity-shift forcing.
Reference: models/multiphase/d2q9_kuper/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_kuper", dims=2, family="multiphase", reference="models/multiphase/d2q9_kuper",
              description="D2Q9 pseudopotential multiphase (Kupershtokh forcing, CS-like EOS)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_field("phi", stencil2d=1)
    # (an LDS tile of the phi stencil made the collision 2.5-9 % slower, profiles/README.md
    # r04e: the stage streams all populations, so its tile marches one plane per group)
    m.add_stage("BaseIteration", "Run", save_fields=["f"], load_densities=["f"])
    m.add_stage("CalcPhi", "CalcPhi", save_fields=["phi"], load_densities=["f"])
    m.add_stage("BaseInit", "Init", save_fields=["f"])
    m.add_action("Iteration", ["BaseIteration", "CalcPhi"])
    m.add_action("Init", ["BaseInit", "CalcPhi"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("P", unit="Pa")
    m.add_quantity("F", unit="N", vector=True)
    S = m.add_setting
    S("omega", comment="relaxation factor", default=1)
    S("nu", comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("Velocity", default="0m/s", comment="inlet velocity", unit="m/s")
    S("Temperature", comment="temperature of the liquid/gas")
    S("FAcc", comment="Multiplier of potential")
    S("Magic", comment="K", default="0.01")
    S("MagicA", comment="A in force calculation", default="-0.152")
    S("MagicF", comment="Force multiplier", default="-0.66666666666666")
    S("GravitationY", comment="Gravitation in the direction of y")
    S("GravitationX", comment="Gravitation in the direction of x")
    S("MovingWallVelocity", comment="Velocity of the MovingWall")
    S("Density", comment="zonal density", zonal=True)
    S("Wetting", comment="wetting factor")
    for g, c in [("Pressure1", "pressure at Obj1"), ("Pressure2", "pressure at Obj2"),
                 ("Pressure3", "pressure at Obj3"), ("Density1", "density at Obj1"),
                 ("Density2", "density at Obj2"), ("Density3", "density at Obj3"),
                 ("SumUsqr", "Sumo o U**2"), ("WallForceX", "force x"), ("WallForceY", "force y")]:
        m.add_global(g, comment=c)
    for n in ["NMovingWall", "MovingWall", "ESymmetry", "NSymmetry", "SSymmetry", "EPressure", "EVelocity",
              "Solid", "Wall", "WPressure", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.set_color("color_value_()", "getRho() < R(1) ? 0 : 1")  # reference Color(): |U|, 0 below rho 1
    m.set_dynamics("multiphase/d2q9_kuper.inc")
    return m
