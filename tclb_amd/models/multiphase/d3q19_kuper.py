"""d3q19_kuper — D3Q19 pseudopotential (Kupershtokh) liquid-vapour model: d'Humieres MRT
collision, phi = FAcc sqrt(rho/3 - K p_EOS(rho)) computed in its own stage (CalcPhi) and
read with a one-node stencil by the interaction force.
Reference: models/multiphase/d3q19_kuper/{Dynamics.R, Dynamics.c.Rt}, src/lib/d3q19.R.

Not carried over: the sympy-generated ``MovingWallBC_e<i>``/``PressureBC_e<i>`` helpers of
the reference template — they are emitted there but never dispatched from Run()."""
from ..dsl import Model
from ...emit.symbolic import d3q19_mrt
from ..flow.d3q19 import mrt19_block


def build() -> Model:
    m = Model("d3q19_kuper", dims=3, family="multiphase", reference="models/multiphase/d3q19_kuper",
              description="D3Q19 MRT pseudopotential multiphase (Kupershtokh forcing, CS-like EOS)")
    U = d3q19_mrt().U
    for i in range(19):
        m.add_density(f"f[{i}]", int(U[i, 0]), int(U[i, 1]), int(U[i, 2]), group="f", comment=f"density F{i}")
    m.add_field("phi", stencil3d=1)
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
    m.add_quantity("Phi", unit="1")
    m.add_quantity("F", unit="N", vector=True)
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("InletVelocity", default="0m/s", comment="inlet velocity", unit="m/s")
    S("Temperature", comment="temperature of the liquid/gas")
    S("FAcc", default="1", comment="Multiplier of potential")
    for a in "xyz":
        S(f"BoundaryVelocity_{a}", default="0m/s", comment="boundary velocity", unit="m/s")
    S("Boundary_rho", default="0m/s", comment="boundary density")
    S("Magic", default="0.01", comment="K")
    S("MagicA", default="-0.152", comment="A in force calculation")
    for a in "YXZ":
        S(f"Gravitation{a}", comment=f"Gravitation in the direction of {a.lower()}")
    S("MovingWallVelocity", comment="Velocity of the MovingWall")
    S("Density", comment="zonal density", zonal=True)
    S("Wetting", comment="wetting factor")
    for a in "XYZ":
        m.add_global(f"MovingWallForce{a}", comment=f"force {a.lower()}")
    for g, c in [("Pressure1", "pressure at Obj1"), ("Pressure2", "pressure at Obj2"),
                 ("Pressure3", "pressure at Obj3"), ("Density1", "density at Obj1"),
                 ("Density2", "density at Obj2"), ("Density3", "density at Obj3")]:
        m.add_global(g, comment=c)
    for n in ["EPressure", "Solid", "Wall", "WPressure", "WPressureL", "WVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("MovingWall", "BOUNDARY")
    m.add_codegen(mrt19_block)
    m.set_color("color_value_()", "getRho() < R(1) ? 0 : 1")  # reference Color(): |U|, 0 below rho 1
    m.set_dynamics("multiphase/d3q19_kuper.inc")
    return m
