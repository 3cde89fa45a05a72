"""d2q9_pp_LBL — single-component pseudopotential (Shan-Chen type) multiphase model with a
Carnahan-Starling equation of state and the Lycett-Brown & Luo forcing of the BGK
collision ("Improved forcing scheme in pseudopotential lattice Boltzmann methods for
multiphase flow at arbitrarily high density ratios").  The potential psi is a one-cell
stencil field recomputed from the EoS after every iteration.
Reference: models/multiphase/experimental/d2q9_pp_LBL/{Dynamics.R, Dynamics.c.Rt}
(the node type MRT selects the BGK+forcing collision, as in the reference; the
reference's unused MRT and BodyForce routines are not carried over).
The EoS constant ``R`` is exposed under its reference name; in the generated C++ it is
the member ``R_`` (``R`` is the scalar type of the node).
"""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_pp_LBL", dims=2, family="multiphase",
              reference="models/multiphase/experimental/d2q9_pp_LBL",
              description="D2Q9 pseudopotential multiphase (Carnahan-Starling EoS, Lycett-Brown/Luo forcing)")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_field("psi", stencil2d=1)
    m.add_stage("BaseIteration", "Run", save_fields=["f"], load_densities=["f"])
    m.add_stage("calcPsi", "calcPsi", save_fields=["psi"], load_densities=["f"])
    m.add_stage("BaseInit", "Init", save_fields=["f"], load_densities=["f"])
    m.add_action("Iteration", ["BaseIteration", "calcPsi"])
    m.add_action("Init", ["BaseInit", "calcPsi"])
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("F", unit="N", vector=True)
    m.add_quantity("P", unit="Pa")
    m.add_quantity("Psi", unit="1")
    S = m.add_setting
    S("G", default=-1.0, comment="interaction strength")
    S("T", default=0.0585, comment="effective temperature")
    S("alpha", default=0.25, comment="CS EoS parameter")
    S("R", default=0.25, comment="CS EoS parameter")
    S("beta", default=1, comment="CS EoS parameter")
    S("kappa", default=0, comment="surface tension parameter")
    S("eps_0", default=2, comment="mechanical stability coef")
    S("betaforcing", default=1.0, comment="beta forcing scheme")
    S("omega", comment="one over relaxation time", S7="1-omega")
    S("tempomega", default=1, comment="omega seems to get overwritten in preamble??")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("Velocity", default=0, comment="inlet/outlet/init velocity", zonal=True)
    S("VelocityY", default=0, comment="init velocity in y dirn", zonal=True)
    S("Density", default=1, comment="inlet/outlet/init density", zonal=True)
    S("GravitationY", comment="Gravitation in the direction of y")
    S("GravitationX", comment="Gravitation in the direction of x")
    for k, d in (("S0", 0), ("S1", 0), ("S2", 0), ("S3", -0.333333333), ("S4", 0), ("S5", 0), ("S6", 0),
                 ("S7", 0), ("S8", 0)):
        S(k, default=d, comment="MRT Sx")
    m.add_global("PressureLoss", comment="pressure loss", unit="1mPa")
    m.add_global("OutletFlux", comment="pressure loss", unit="1m2/s")
    m.add_global("InletFlux", comment="pressure loss", unit="1m2/s")
    for n in ("BottomSymmetry", "TopSymmetry", "RightSymmetry", "EPressure", "EVelocity", "Solid", "Wall",
              "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("multiphase/d2q9_pp_LBL.inc")
    return m
